# Round 6: single-frame lines determinism -- three runs' digests and every frame against the oracle,
# then the GPU line tests and the drop-in leg.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-r6ld}
for i in 1 2 3; do timeout -k 10 120 python -u tools/micro/lines_single.py 64 > gpurun_out/${P}_run$i.log 2>&1 || exit 1; done
timeout -k 10 200 python -u tools/micro/lines_single.py 64 --check > gpurun_out/${P}_check.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_lines.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${P}_lines.log 2>&1 &&
timeout -k 10 300 python -u tools/micro/dropin_only.py > gpurun_out/${P}_dropin.log 2>&1
