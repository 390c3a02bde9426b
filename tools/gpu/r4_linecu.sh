# Line stage on a CU-masked stream (EAO_LINES_CU_QUARTERS=q: q of every 4 CUs) against the full
# device; EAO bench, default ordering, alternating on one box; then the line tests with q=2.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  for q in 4 3 2 1; do
    EAO_LINES_CU_QUARTERS=$q timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4cu.log 2>&1 || exit 1
    tail -1 gpurun_out/r4cu.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('[cu quarters $q]', round(d['ms_per_step'],2), round(d['line_detect']['ms_per_step'],2), round(d['assoc_profile_us_per_frame']['frame'],1), round(d['assoc_profile_us_per_frame']['assoc_loop'],1), d['parity']['lines_bitexact'] if 'parity' in d else '')" || exit 1
  done
done > gpurun_out/r4cu_summary.txt 2>&1 &&
EAO_LINES_CU_QUARTERS=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_lines.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4cu_tests.log 2>&1
