# Round 6: single-frame lines in one launch (k_lines_fused) -- line parity, the single-call time and
# kernel split (A/B: EAO_LINES_ONE_LAUNCH=0, the three launches), the drop-in leg.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-r6l}
timeout -k 10 120 python -u tools/micro/lines_single.py 64 --check > gpurun_out/${P}_single.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_lines.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${P}_lines.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_kt_one -o run -- python3 tools/micro/lines_single.py 64 > gpurun_out/${P}_single_kt.log 2>&1 &&
EAO_LINES_ONE_LAUNCH=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_kt_three -o run -- python3 tools/micro/lines_single.py 64 > gpurun_out/${P}_single_kt3.log 2>&1 &&
timeout -k 10 300 python -u tools/micro/dropin_only.py > gpurun_out/${P}_dropin.log 2>&1
