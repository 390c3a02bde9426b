# Round 6: the association's single-frame calls alone (no gap, and 800 us between calls).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/micro/assoc_single.py > gpurun_out/r6as_0.log 2>&1 &&
timeout -k 10 120 python -u tools/micro/assoc_single.py 800 > gpurun_out/r6as_800.log 2>&1
