# Round 6 A/B: the NP direct-count threshold (EAO_NP_DIRECT = max m * n counted directly) on the
# replay probe (HSA lanes: the threshold now reaches the lanes' code object too), alternating.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for v in 131072 524288 2097152 8388608; do
    EAO_NP_DIRECT=$v EAO_PROBE_PASSES=3 timeout -k 10 120 python -u tools/replay_probe.py > gpurun_out/r6n_${v}_$r.log 2>&1 || exit 1
  done
done
