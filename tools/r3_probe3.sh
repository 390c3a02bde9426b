set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/replay_probe.py > gpurun_out/r3_probe3_eao.txt 2>&1 &&
EAO_NO_LOOKAHEAD=1 timeout -k 10 300 python -u tools/replay_probe.py > gpurun_out/r3_probe3_eao_nola.txt 2>&1 &&
timeout -k 10 300 python -u tools/replay_probe.py > gpurun_out/r3_probe3_eao_b.txt 2>&1 &&
timeout -k 10 300 python -u tools/replay_probe.py full > gpurun_out/r3_probe3_full.txt 2>&1 &&
EAO_NO_LOOKAHEAD=1 timeout -k 10 300 python -u tools/replay_probe.py full > gpurun_out/r3_probe3_full_nola.txt 2>&1
