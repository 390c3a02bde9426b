# Forest score phase: points prefetched by the scoring waves during the build, CalculateC of every
# leaf size staged in LDS. Parity, then build / score cycles A/B and the replay probe A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_assoc.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_sc_assoc.log 2>&1 &&
for r in 1 2; do
  timeout -k 10 120 python -u tools/micro/if_probe.py | grep "^n=" | sed "s/load.*gather/gather/; s/^/new  /" &&
  EAO_ACCEL_LIB=eao-slam_amd/lib/ab/base/libeao_accel.so timeout -k 10 120 python -u tools/micro/if_probe.py | grep "^n=" | sed "s/load.*gather/gather/; s/^/base /" || break
done > gpurun_out/r4_sc_ifprobe.log 2>&1 &&
for r in 1 2; do
  EAO_ACCEL_LIB=eao-slam_amd/lib/ab/base/libeao_accel.so timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" | cut -c1-60 | sed "s/^/base /" &&
  timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" | cut -c1-60 | sed "s/^/new  /" || break
done > gpurun_out/r4_sc_probe.log 2>&1
