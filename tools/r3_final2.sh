# Round-3 final measurements, part 2: Full, Config B, Config C benches and the association probe.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --config full > gpurun_out/f2_bench_full.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config b > gpurun_out/f2_bench_b.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c > gpurun_out/f2_bench_c.log 2>&1 &&
timeout -k 10 300 python -u tools/replay_probe.py > gpurun_out/f2_probe.log 2>&1
