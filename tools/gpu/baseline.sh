# Quick state check: EAO bench + association replay probe.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > gpurun_out/r4_bench0.log 2>&1 &&
timeout -k 10 200 python -u tools/replay_probe.py > gpurun_out/r4_probe0.log 2>&1
