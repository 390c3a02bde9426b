# Round-3 final measurements, part 1: GPU suite, smoke, EAO bench, kernel trace of the bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs > gpurun_out/f1_gputest.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f1_smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/f1_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f1_kt -o run -- python3 bench.py --steps 2 --no-cpu-baseline > gpurun_out/f1_kt.log 2>&1
