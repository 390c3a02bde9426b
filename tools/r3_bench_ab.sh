# bench A/B: main thread polling the extraction stream during the association (--poll) vs joining first
# (default), and --no-overlap; alternating on one box.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --poll > gpurun_out/bab_poll_$r.log 2>&1 &&
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bab_join_$r.log 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-overlap > gpurun_out/bab_noov.log 2>&1
