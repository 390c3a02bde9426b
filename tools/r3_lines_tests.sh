# Line-detection GPU tests (incl. the small-cap placement case).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lines.py -x -v --timeout 200 --timeout-method thread > gpurun_out/lines_tests.log 2>&1
