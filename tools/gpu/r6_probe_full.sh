# Round 6: the replay probe on the Full stream (2582 frames) and the EAO step's kernel trace on the
# HSA lanes (rocprofv3 --kernel-trace --stats of the bench itself).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
EAO_PROBE_PASSES=2 timeout -k 10 200 python -u tools/replay_probe.py full > gpurun_out/r6p_probe_full.log 2>&1 &&
EAO_PROBE_PASSES=3 timeout -k 10 200 python -u tools/replay_probe.py > gpurun_out/r6p_probe.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6p_kt -o run -- python3 bench.py --steps 2 --no-cpu-baseline --no-dropin --chain-frames 0 > gpurun_out/r6p_kt.log 2>&1
