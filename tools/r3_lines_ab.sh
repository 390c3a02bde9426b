# k_edlines across chains (8 waves per frame) vs one wave per frame: line parity tests, then the EAO
# bench's line-detection stage (in the step) old / new alternating, and a kernel trace of the new one.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lines.py -x -q --timeout 300 --timeout-method thread > gpurun_out/lab2_tests.log 2>&1 &&
for r in 1 2; do
  EAO_ACCEL_LIB=eao-slam_amd/lib/ab/libeao_old.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 > gpurun_out/lab2_old_$r.log 2>&1 &&
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 > gpurun_out/lab2_new_$r.log 2>&1 || exit 1
done
