# Front / association overlap: step time with the front overlapped (line stage in 1, 4 or 8
# launches, association on a second thread) and enqueued before the association (default), alternating.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for v in "--thread --line-batches 1" "--thread --line-batches 4" "--thread --line-batches 8" ""; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline $v > gpurun_out/r4o.log 2>&1 || exit 1
    tail -1 gpurun_out/r4o.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$v', round(d['ms_per_step'],2), round(d['line_detect']['ms_per_step'],2), round(d['assoc_profile_us_per_frame']['frame'],1), round(d['assoc_profile_us_per_frame']['assoc_loop'],1))" || exit 1
  done
done > gpurun_out/r4o_summary.txt 2>&1
