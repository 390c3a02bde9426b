# Forest kernel A/B: parity (forest / replay / fr3 / golden), phase probe (stamp build), then the
# replay probe, old (eao-slam_amd/lib/ab/libeao_old.so) vs new library alternating.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_assoc.py tests/test_gpu_replay.py tests/test_gpu_fr3.py tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread > gpurun_out/fab_tests.log 2>&1 &&
EAO_ACCEL_LIB=eao-slam_amd/lib/prof/libeao_accel.so timeout -k 10 120 python -u tools/micro/if_probe.py > gpurun_out/fab_if_probe_prof.txt 2>&1 &&
for r in 1 2 3; do
  EAO_ACCEL_LIB=eao-slam_amd/lib/ab/libeao_old.so timeout -k 10 200 python -u tools/replay_probe.py > gpurun_out/fab_old_$r.log 2>&1 &&
  timeout -k 10 200 python -u tools/replay_probe.py > gpurun_out/fab_new_$r.log 2>&1 || exit 1
done
