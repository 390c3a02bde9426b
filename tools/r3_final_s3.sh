# Round-3 session-2 closing measurements: GPU suite, smoke, EAO bench (+ kernel trace), Full, Config B, Config C, probe.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs > gpurun_out/s3_gputest.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3_smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/s3_bench.log 2>&1 &&
timeout -k 10 400 python -u bench.py --config full > gpurun_out/s3_bench_full.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config b > gpurun_out/s3_bench_b.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c > gpurun_out/s3_bench_c.log 2>&1 &&
timeout -k 10 200 python -u tools/replay_probe.py > gpurun_out/s3_probe.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s3_kt -o run -- python3 bench.py --steps 2 --no-cpu-baseline > gpurun_out/s3_kt.log 2>&1
