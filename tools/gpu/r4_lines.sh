# Line stage: move-byte edge drawing (k_line_moves + k_edge_draw) against the base build:
# parity (GPU line tests, oracle check), then alternating same-box timings.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lines.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4l_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/micro/lines_bench.py --check > gpurun_out/r4l_new_0.log 2>&1 &&
for r in 1 2; do
  EAO_ACCEL_LIB=eao-slam_amd/lib/ab/base/libeao_accel.so timeout -k 10 200 python -u tools/micro/lines_bench.py > gpurun_out/r4l_base_$r.log 2>&1 &&
  timeout -k 10 200 python -u tools/micro/lines_bench.py > gpurun_out/r4l_new_$r.log 2>&1 || exit 1
done &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4l_kt -o run -- python3 tools/micro/lines_bench.py > gpurun_out/r4l_kt.log 2>&1
