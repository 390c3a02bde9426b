# Contention of the frame work with the association (default ordering): full CUs, CU-masked
# front stream (3/4, 2/4 of the CUs), line stage in 4 launches; alternating on one box.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in "" "--front-cus 3" "--front-cus 2" "--line-batches 4"; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline $v > gpurun_out/r4fr.log 2>&1 || exit 1
    tail -1 gpurun_out/r4fr.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('[$v]', round(d['ms_per_step'],2), round(d['line_detect']['ms_per_step'],2), round(d['extract_ms_per_step'],2), round(d['assoc_profile_us_per_frame']['frame'],1), d['parity']['assoc_ids_identical'] if 'parity' in d else '')" || exit 1
  done
done > gpurun_out/r4fr_summary.txt 2>&1
