# Line stage: the fused walk + EDline workgroup (k_edge_lines, 8 or 4 waves) against the two-kernel
# path (EAO_LINES_FUSED=0): parity first, then alternating same-box timings.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lines.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4f_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/micro/lines_bench.py --check > gpurun_out/r4f_f8_0.log 2>&1 &&
EAO_ACCEL_LIB=eao-slam_amd/lib/ab/fused4/libeao_accel.so timeout -k 10 200 python -u tools/micro/lines_bench.py --check > gpurun_out/r4f_f4_0.log 2>&1 &&
for r in 1 2; do
  EAO_LINES_FUSED=0 timeout -k 10 200 python -u tools/micro/lines_bench.py > gpurun_out/r4f_two_$r.log 2>&1 &&
  timeout -k 10 200 python -u tools/micro/lines_bench.py > gpurun_out/r4f_f8_$r.log 2>&1 &&
  EAO_ACCEL_LIB=eao-slam_amd/lib/ab/fused4/libeao_accel.so timeout -k 10 200 python -u tools/micro/lines_bench.py > gpurun_out/r4f_f4_$r.log 2>&1 || exit 1
done &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4f_kt -o run -- python3 tools/micro/lines_bench.py > gpurun_out/r4f_kt.log 2>&1
