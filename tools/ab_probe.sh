#!/bin/bash
# A/B of the association replay: the probe under two engine libraries, alternating,
# in one process set on one box (development aid). usage: tools/ab_probe.sh LIB_A LIB_B [full]
set -e
for r in 1 2; do
  for L in "$1" "$2"; do
    echo "== $L"
    EAO_ACCEL_LIB=$L timeout -k 10 200 python -u tools/replay_probe.py $3 | grep "pass 2"
  done
done
