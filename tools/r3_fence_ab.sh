# Tiled edge walk without the per-step release fence (new) vs with it (old): line tests, line stage A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lines.py -x -q --timeout 200 --timeout-method thread > gpurun_out/fab3_tests.log 2>&1 &&
for r in 1 2; do
  EAO_ACCEL_LIB=eao-slam_amd/lib/ab/libeao_old.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 > gpurun_out/fab3_old_$r.log 2>&1 &&
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 > gpurun_out/fab3_new_$r.log 2>&1 || exit 1
done
