# Round 6 A/B: single line calls spinning on a sequence word written by k_lines_out (default) vs a stream
# synchronisation (EAO_LINES_SYNC=1): line tests, oracle check + digest, single-call time, drop-in leg.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lines.py > gpurun_out/r6ls_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/micro/lines_single.py 64 --check > gpurun_out/r6ls_check.log 2>&1 &&
EAO_LINES_SYNC=1 timeout -k 10 120 python -u tools/micro/lines_single.py 64 > gpurun_out/r6ls_single_sync.log 2>&1 || exit 1
for r in 1 2 3 4; do
  timeout -k 10 300 python -u tools/micro/dropin_only.py > gpurun_out/r6ls_k_$r.log 2>&1 &&
  EAO_LINES_SYNC=1 timeout -k 10 300 python -u tools/micro/dropin_only.py > gpurun_out/r6ls_s_$r.log 2>&1 || exit 1
done
