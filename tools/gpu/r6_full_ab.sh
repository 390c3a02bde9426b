# Round 6: the Full replay probe, then the Full bench line (parity checked over all 2582 frames).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-r6fa}
EAO_PROBE_PASSES=2 timeout -k 10 300 python -u tools/replay_probe.py full > gpurun_out/${P}_probe_full.log 2>&1 &&
timeout -k 10 600 python -u bench.py --config full > gpurun_out/${P}_bench_full.log 2>&1
