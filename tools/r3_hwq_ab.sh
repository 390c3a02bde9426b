# Hardware queues A/B for the EAO bench: GPU_MAX_HW_QUEUES default (4) vs 8, alternating.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/hwq_4_$r.log 2>&1 &&
  GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/hwq_8_$r.log 2>&1 || exit 1
done
