# Look-ahead granularity: replay parity, then alternating probes (EAO_PREP_CHUNK points per
# look-ahead step; 1e9 = one step per phase, the earlier granularity).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fr3.py tests/test_gpu_replay.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4p_tests.log 2>&1 &&
for r in 1 2 3; do
  EAO_PREP_CHUNK=1000000000 timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" | sed "s/^/chunk=all /" &&
  EAO_PREP_CHUNK=128 timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" | sed "s/^/chunk=128 /" &&
  EAO_PREP_CHUNK=32 timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" | sed "s/^/chunk=32 /" || exit 1
done > gpurun_out/r4p_probe.log 2>&1
