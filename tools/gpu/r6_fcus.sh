# Round 6: the frame work's CU mask (bench.py --frame-cus K) against the association stalls beside the
# frame kernels: A/B of the step (alternating, same box), then a kernel trace at K = 28.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-r6y}
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-dropin > gpurun_out/${P}_base$i.log 2>&1 &&
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-dropin --frame-cus 28 > gpurun_out/${P}_f28_$i.log 2>&1 &&
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-dropin --frame-cus 24 > gpurun_out/${P}_f24_$i.log 2>&1 || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${P}_kt28 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dropin --frame-cus 28 > gpurun_out/${P}_kt28.log 2>&1
