# GPU suite, then the replay probe old (lib/ab/libeao_old.so) vs new alternating, 3 each.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs > gpurun_out/ab3_gputest.log 2>&1 &&
for r in 1 2 3; do
  EAO_ACCEL_LIB=eao-slam_amd/lib/ab/libeao_old.so timeout -k 10 200 python -u tools/replay_probe.py > gpurun_out/ab3_old_$r.log 2>&1 &&
  timeout -k 10 200 python -u tools/replay_probe.py > gpurun_out/ab3_new_$r.log 2>&1 || exit 1
done
