# Round 6 A/B: single motion-search calls moving staging and matches by kernel (default) vs copy-engine
# transfers (EAO_MATCH_DMA=1): ORB + matcher GPU tests, then the drop-in leg alternating.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_orb.py tests/test_c99_consumer.py tests/test_gpu_match.py > gpurun_out/r6mi_tests.log 2>&1 || exit 1
for r in 1 2 3 4; do
  timeout -k 10 300 python -u tools/micro/dropin_only.py > gpurun_out/r6mi_k_$r.log 2>&1 &&
  EAO_MATCH_DMA=1 timeout -k 10 300 python -u tools/micro/dropin_only.py > gpurun_out/r6mi_dma_$r.log 2>&1 || exit 1
done
