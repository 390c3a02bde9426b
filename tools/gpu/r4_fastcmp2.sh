# FAST compacted strengths vs dense on the EAO bench's own frames (structured texture) and on
# the plain texture (Config B's), alternating; the bench's own fast stage with both.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for c in 0 1; do
    EAO_FAST_CMP=$c timeout -k 10 200 python -u tools/micro/orb_stages.py > gpurun_out/r4c2_s_$c.log 2>&1 &&
    EAO_FAST_CMP=$c STRUCT=0 timeout -k 10 200 python -u tools/micro/orb_stages.py > gpurun_out/r4c2_p_$c.log 2>&1 &&
    EAO_FAST_CMP=$c STRUCT=0 timeout -k 10 200 python -u tools/micro/orb_stages.py 256 1920 1080 4000 > gpurun_out/r4c2_b_$c.log 2>&1 &&
    echo "cmp=$c struct640: $(tail -1 gpurun_out/r4c2_s_$c.log) | plain640: $(tail -1 gpurun_out/r4c2_p_$c.log | sed 's/.*fast/fast/;s/ distribute.*//') | plain1080: $(tail -1 gpurun_out/r4c2_b_$c.log | sed 's/.*fast/fast/;s/ distribute.*//')" || exit 1
  done
done > gpurun_out/r4c2_summary.txt 2>&1 &&
for c in 0 1; do
  EAO_FAST_CMP=$c timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4c2_bench_$c.log 2>&1 || exit 1
done
