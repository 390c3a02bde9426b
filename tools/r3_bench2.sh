set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bow.py tests/test_gpu_lines.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_gpu_bow.log 2>&1 &&
timeout -k 10 500 python -u bench.py > gpurun_out/r3_bench2.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config b > gpurun_out/r3_bench2_b.log 2>&1
