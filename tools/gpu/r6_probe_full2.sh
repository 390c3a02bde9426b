# Round 6: the replay probe on the Full stream (2582 frames): the engine's per-phase profile on the box.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
EAO_PROBE_PASSES=2 timeout -k 10 300 python -u tools/replay_probe.py full > gpurun_out/r6pf_probe_full.log 2>&1
