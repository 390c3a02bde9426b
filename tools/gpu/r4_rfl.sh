# Scalar RNG state of the forest's wave generator (readfirstlane): build cycles A/B, then closing measurements.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_assoc.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_rfl_assoc.log 2>&1 &&
timeout -k 10 120 python -u tools/micro/if_probe.py > gpurun_out/r4_rfl_ifprobe_new.log 2>&1 &&
EAO_ACCEL_LIB=eao-slam_amd/lib/ab/base/libeao_accel.so timeout -k 10 120 python -u tools/micro/if_probe.py > gpurun_out/r4_rfl_ifprobe_base.log 2>&1 &&
timeout -k 10 120 python -u tools/micro/if_probe.py > gpurun_out/r4_rfl_ifprobe_new2.log 2>&1 &&
EAO_ACCEL_LIB=eao-slam_amd/lib/ab/base/libeao_accel.so timeout -k 10 120 python -u tools/micro/if_probe.py > gpurun_out/r4_rfl_ifprobe_base2.log 2>&1
