# Round 6: the line call's two halves (eao_lines_detect_color_start / _finish) on the caller's thread vs
# the one-call form on a second thread: line tests, then the drop-in leg (both forms in every run).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lines.py > gpurun_out/r6as_tests.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 300 python -u tools/micro/dropin_only.py > gpurun_out/r6as_$r.log 2>&1 || exit 1
done
