# Round 6: where the single-frame merge's time goes (EAO_LINES_PROF=1 counters of k_lines_fused's merge
# wave), then the plain timing, parity and kernel split of both single-frame paths.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-r6r}
EAO_LINES_PROF=1 timeout -k 10 120 python -u tools/micro/lines_single.py 64 > gpurun_out/${P}_lprof.log 2>&1 &&
timeout -k 10 120 python -u tools/micro/lines_single.py 64 --check > gpurun_out/${P}_single.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_lines.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${P}_lines.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_kt_one -o run -- python3 tools/micro/lines_single.py 64 > gpurun_out/${P}_single_kt.log 2>&1 &&
EAO_LINES_ONE_LAUNCH=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_kt_three -o run -- python3 tools/micro/lines_single.py 64 > gpurun_out/${P}_single_kt3.log 2>&1
