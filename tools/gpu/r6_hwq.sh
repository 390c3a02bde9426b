# Round 6: HIP's hardware-queue count beside the association's HSA lanes (A/B of the step, alternating).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-r6q}
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-dropin > gpurun_out/${P}_q4_$i.log 2>&1 &&
  GPU_MAX_HW_QUEUES=2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-dropin > gpurun_out/${P}_q2_$i.log 2>&1 &&
  GPU_MAX_HW_QUEUES=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-dropin > gpurun_out/${P}_q1_$i.log 2>&1 || exit 1
done
