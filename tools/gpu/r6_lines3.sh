# Round 6: the line engine's stream priority inside the drop-in leg (A/B EAO_LINES_PRI=0), with the
# one-launch lines (and, for reference, the three launches).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-r6o}
timeout -k 10 300 python -u tools/micro/dropin_only.py > gpurun_out/${P}_dropin_pri.log 2>&1 &&
EAO_LINES_PRI=0 timeout -k 10 300 python -u tools/micro/dropin_only.py > gpurun_out/${P}_dropin_nopri.log 2>&1 &&
EAO_LINES_ONE_LAUNCH=0 timeout -k 10 300 python -u tools/micro/dropin_only.py > gpurun_out/${P}_dropin_three_pri.log 2>&1
