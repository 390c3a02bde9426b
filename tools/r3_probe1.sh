set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/replay_probe.py > gpurun_out/r3_probe_eao.txt 2>&1 &&
timeout -k 10 300 python -u tools/replay_probe.py full > gpurun_out/r3_probe_full.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3_kt_replay -o run -- python3 tools/replay_probe.py > gpurun_out/r3_kt_replay.log 2>&1
