# Closing run: line parity + line-stage A/B (tiled edge walk vs the previous library), then the
# closing measurement set (GPU suite, smoke, EAO / Full / B / C benches, probe, kernel trace).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lines.py -x -q --timeout 300 --timeout-method thread > gpurun_out/lab2_tests.log 2>&1 &&
EAO_ACCEL_LIB=eao-slam_amd/lib/ab/libeao_old.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 > gpurun_out/lab2_old_1.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 > gpurun_out/lab2_new_1.log 2>&1 &&
bash tools/r3_final_s3.sh
