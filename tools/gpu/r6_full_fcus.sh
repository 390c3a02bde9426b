# Round 6: the Full step with the frame work CU-masked (bench.py --frame-cus K), alternating, same box.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-r6ff}
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config full --no-cpu-baseline --no-dropin > gpurun_out/${P}_base$i.log 2>&1 &&
  timeout -k 10 300 python -u bench.py --config full --no-cpu-baseline --no-dropin --frame-cus 24 > gpurun_out/${P}_f24_$i.log 2>&1 &&
  timeout -k 10 300 python -u bench.py --config full --no-cpu-baseline --no-dropin --frame-cus 16 > gpurun_out/${P}_f16_$i.log 2>&1 || exit 1
done
