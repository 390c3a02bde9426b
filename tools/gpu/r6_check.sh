# Round 6 checkpoint: the GPU suite, smoke, the EAO bench (default run) and the Full bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-r6c}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs > gpurun_out/${P}_gputest.log 2>&1 &&
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${P}_smoke.log 2>&1 &&
timeout -k 10 500 python -u bench.py > gpurun_out/${P}_bench.log 2>&1 &&
timeout -k 10 600 python -u bench.py --config full > gpurun_out/${P}_bench_full.log 2>&1
