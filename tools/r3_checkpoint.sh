# Round-3 checkpoint on one MI355X: GPU suite, smoke, EAO bench, Config B bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs > gpurun_out/ck_gputest.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ck_smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/ck_bench.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config b > gpurun_out/ck_bench_b.log 2>&1
