# FAST occupancy A/B: current library vs the waves_per_eu(6) build (62 VGPRs), alternating.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 200 python -u tools/orb_stages.py --reps 8 > gpurun_out/fast_ab2_cur_$r.log 2>&1 &&
  EAO_ACCEL_LIB=eao-slam_amd/lib/ab/libeao_w6.so timeout -k 10 200 python -u tools/orb_stages.py --reps 8 > gpurun_out/fast_ab2_w6_$r.log 2>&1 || exit 1
done
