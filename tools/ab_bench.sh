#!/bin/bash
# A/B of bench.py under two engine libraries, alternating (development aid).
# usage: tools/ab_bench.sh LIB_A LIB_B ROUNDS [bench args...]
set -e
A=$1; B=$2; R=$3; shift 3
for r in $(seq 1 $R); do
  for L in "$A" "$B"; do
    v=$(EAO_ACCEL_LIB=$L timeout -k 10 600 python -u bench.py --no-cpu-baseline "$@" | tail -1 |
        python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.1f fps %.1f ms/step' % (d['value'], d['ms_per_step']))")
    echo "$(basename $(dirname $(dirname $L)))/$(basename $L): $v"
  done
done
