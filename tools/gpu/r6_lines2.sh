# Round 6: k_lines_fused workgroup count A/B inside the drop-in leg (overlapped pass: lines beside
# extraction + matching), single-call times.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-r6n}
timeout -k 10 120 python -u tools/micro/lines_single.py 64 > gpurun_out/${P}_single.log 2>&1 &&
timeout -k 10 300 python -u tools/micro/dropin_only.py > gpurun_out/${P}_dropin32.log 2>&1 &&
EAO_LINES_ONE_LAUNCH=16 timeout -k 10 300 python -u tools/micro/dropin_only.py > gpurun_out/${P}_dropin16.log 2>&1 &&
EAO_LINES_ONE_LAUNCH=0 timeout -k 10 300 python -u tools/micro/dropin_only.py > gpurun_out/${P}_dropin0.log 2>&1
