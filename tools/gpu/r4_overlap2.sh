# Association on a second thread (--thread) vs the frame work enqueued before the association (default), 4 alternating pairs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3 4; do
  for v in "--thread" ""; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline $v > gpurun_out/r4o.log 2>&1 || exit 1
    tail -1 gpurun_out/r4o.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('[$v]', round(d['ms_per_step'],2), round(d['assoc_profile_us_per_frame']['frame'],1), round(d['assoc_profile_us_per_frame']['assoc_loop'],1))" || exit 1
  done
done > gpurun_out/r4o2_summary.txt 2>&1
