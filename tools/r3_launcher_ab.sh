# Launcher thread A/B: association parity tests, then the replay probe without (EAO_NO_LAUNCHER=1)
# and with the GPU command thread, alternating, then the EAO bench with it.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_assoc.py tests/test_gpu_replay.py tests/test_gpu_fr3.py tests/test_gpu_golden.py tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread > gpurun_out/lab_tests.log 2>&1 &&
for r in 1 2 3; do
  EAO_NO_LAUNCHER=1 timeout -k 10 200 python -u tools/replay_probe.py > gpurun_out/lab_off_$r.log 2>&1 &&
  timeout -k 10 200 python -u tools/replay_probe.py > gpurun_out/lab_on_$r.log 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/lab_bench.log 2>&1
