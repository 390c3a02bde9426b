# Round 6 A/B: four private counter copies in the NP rank path at Pm = 512 (EAO_NP_HIST4), replay probe
# alternating, then the association GPU tests with the new default.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in 0 1; do
    EAO_NP_HIST4=$v EAO_PROBE_PASSES=3 timeout -k 10 120 python -u tools/replay_probe.py > gpurun_out/r6h4_${v}_$r.log 2>&1 || exit 1
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_assoc.py tests/test_gpu_replay.py tests/test_gpu_fr3.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6h4_tests.log 2>&1
