# Forest phase probe with big-node sub-step stamps (EAO_IF_PROF build).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
EAO_ACCEL_LIB=eao-slam_amd/lib/prof/libeao_accel.so timeout -k 10 120 python -u tools/micro/if_probe.py > gpurun_out/ifp2.txt 2>&1
