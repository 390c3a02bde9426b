set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_replay.py tests/test_gpu_fr3.py tests/test_gpu_assoc.py tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_gpu_replay4.log 2>&1 &&
timeout -k 10 300 python -u tools/replay_probe.py > gpurun_out/r3_probe4_eao.txt 2>&1 &&
timeout -k 10 300 python -u tools/replay_probe.py full > gpurun_out/r3_probe4_full.txt 2>&1
