set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/micro/if_probe.py > gpurun_out/r3_if_probe.txt 2>&1 &&
EAO_ACCEL_LIB=eao-slam_amd/lib/prof/libeao_accel.so timeout -k 10 120 python -u tools/micro/if_probe.py > gpurun_out/r3_if_probe_prof.txt 2>&1
