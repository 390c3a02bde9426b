# Round 6 A/B: single line calls staging the pinned frame into HBM by copy kernel (default) vs the maps
# kernel reading it in place over PCIe (EAO_LINES_IN=pcie): oracle check + digest, single-call time,
# the drop-in leg (alternating).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/micro/lines_single.py 64 --check > gpurun_out/r6dk_check.log 2>&1 &&
EAO_LINES_IN=pcie timeout -k 10 120 python -u tools/micro/lines_single.py 64 > gpurun_out/r6dk_single_pcie.log 2>&1 || exit 1
for r in 1 2 3 4; do
  timeout -k 10 300 python -u tools/micro/dropin_only.py > gpurun_out/r6dk_k_$r.log 2>&1 &&
  EAO_LINES_IN=pcie timeout -k 10 300 python -u tools/micro/dropin_only.py > gpurun_out/r6dk_p_$r.log 2>&1 || exit 1
done
