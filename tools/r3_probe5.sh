set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_assoc.py tests/test_gpu_golden.py tests/test_gpu_replay.py tests/test_gpu_fr3.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_gpu5.log 2>&1 &&
timeout -k 10 120 python -u tools/micro/if_probe.py > gpurun_out/r3_if_probe5.txt 2>&1 &&
EAO_ACCEL_LIB=eao-slam_amd/lib/prof/libeao_accel.so timeout -k 10 120 python -u tools/micro/if_probe.py > gpurun_out/r3_if_probe5_prof.txt 2>&1 &&
timeout -k 10 300 python -u tools/replay_probe.py > gpurun_out/r3_probe5_eao.txt 2>&1 &&
timeout -k 10 300 python -u tools/replay_probe.py full > gpurun_out/r3_probe5_full.txt 2>&1
