# Round 6 A/B: the line merge workgroup's wave priority in the drop-in's overlapped pass (alternating).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python -u tools/micro/dropin_only.py > gpurun_out/r6lp_1_$r.log 2>&1 &&
  EAO_LINES_WAVE_PRIO=0 timeout -k 10 300 python -u tools/micro/dropin_only.py > gpurun_out/r6lp_0_$r.log 2>&1 || exit 1
done
