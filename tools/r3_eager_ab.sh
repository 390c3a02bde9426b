# A/B of eager forest launches (EAO_EAGER_FOREST=1) on the EAO bench, alternating; then the
# Full stream once each; then GPU replay tests under the eager setting.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  for e in 0 1; do
    EAO_EAGER_FOREST=$e timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/eager_${e}_$r.log 2>&1 || exit 1
  done
done &&
for e in 0 1; do
  EAO_EAGER_FOREST=$e timeout -k 10 400 python -u bench.py --no-cpu-baseline --config full > gpurun_out/eager_full_${e}.log 2>&1 || exit 1
done &&
EAO_EAGER_FOREST=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_replay.py tests/test_gpu_fr3.py -x -q --timeout 300 --timeout-method thread > gpurun_out/eager_tests.log 2>&1
