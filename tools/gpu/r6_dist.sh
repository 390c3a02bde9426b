# Round 6: the single-frame quadtree (k_distribute_mw, keys in LDS) -- ORB parity, the single-call
# split under a kernel trace (A/B: EAO_DIST_MW=0 one wave per tree), and the drop-in leg.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-r6d}
timeout -k 10 300 python -u -m pytest tests/test_gpu_orb.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${P}_orb.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_kt_mw -o run -- python3 tools/micro/dropin_single.py 64 > gpurun_out/${P}_single_mw.log 2>&1 &&
EAO_DIST_MW=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_kt_1w -o run -- python3 tools/micro/dropin_single.py 64 > gpurun_out/${P}_single_1w.log 2>&1 &&
timeout -k 10 300 python -u tools/micro/dropin_only.py > gpurun_out/${P}_dropin.log 2>&1
