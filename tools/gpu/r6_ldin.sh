# Round 6 A/B: single line calls reading the pinned frame in place vs a DMA copy first (EAO_LINES_DMA_IN=1):
# single-call time, digest, the drop-in leg (alternating).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/micro/lines_single.py 64 > gpurun_out/r6di_check.log 2>&1 &&
EAO_LINES_DMA_IN=1 timeout -k 10 120 python -u tools/micro/lines_single.py 64 > gpurun_out/r6di_single_dma.log 2>&1 || exit 1
for r in 1 2 3 4; do
  timeout -k 10 300 python -u tools/micro/dropin_only.py > gpurun_out/r6di_zc_$r.log 2>&1 &&
  EAO_LINES_DMA_IN=1 timeout -k 10 300 python -u tools/micro/dropin_only.py > gpurun_out/r6di_dma_$r.log 2>&1 || exit 1
done
