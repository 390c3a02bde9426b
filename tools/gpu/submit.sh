#!/bin/bash
# Submit a command to gpurun, retrying only while the pool has no free box (transient, nothing
# charged); any run that actually started is never retried. usage: tools/gpu/submit.sh LOG TIMEOUT 'cmd'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  if grep -q "status=transient" "$LOG" && ! grep -q "status=ok\|rc=[0-9]" "$LOG"; then
    sleep 120
    continue
  fi
  break
done
tail -5 "$LOG"
