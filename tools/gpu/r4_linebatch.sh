# Line stage split into K launches (fewer concurrent k_edge_lines workgroups, whose ~250-VGPR
# waves fill the register files of the CUs they hold) against one launch; default ordering;
# 3 alternating rounds on one box.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in 1 4 8; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --line-batches $v > gpurun_out/r4lb.log 2>&1 || exit 1
    tail -1 gpurun_out/r4lb.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('[line-batches $v]', round(d['ms_per_step'],2), round(d['line_detect']['ms_per_step'],2), round(d['assoc_profile_us_per_frame']['frame'],1), round(d['assoc_profile_us_per_frame']['assoc_loop'],1))" || exit 1
  done
done > gpurun_out/r4lb_summary.txt 2>&1
