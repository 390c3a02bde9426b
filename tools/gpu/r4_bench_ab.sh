# Headline A/B on one box: the EAO bench with the fused line workgroup (default), with the
# two-kernel line path (EAO_LINES_FUSED=0), and with the round's base library (lib/ab/base).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python -u bench.py > gpurun_out/r4b_fused_$r.log 2>&1 &&
  EAO_LINES_FUSED=0 timeout -k 10 300 python -u bench.py > gpurun_out/r4b_two_$r.log 2>&1 &&
  EAO_ACCEL_LIB=eao-slam_amd/lib/ab/base/libeao_accel.so timeout -k 10 300 python -u bench.py > gpurun_out/r4b_base_$r.log 2>&1 || exit 1
done
