# Round 6: NP pair phases for the fr3 frame-start sizes (profiling build's stamps), direct and rank paths.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
EAO_ACCEL_LIB=eao-slam_amd/lib/prof/libeao_accel.so timeout -k 10 120 python -u tools/micro/np_probe.py 30,400 74,1162 100,1162 175,1162 300,1162 60,2000 > gpurun_out/r6np_prof.log 2>&1 &&
timeout -k 10 120 python -u tools/micro/np_probe.py 30,400 74,1162 100,1162 175,1162 300,1162 60,2000 > gpurun_out/r6np_plain.log 2>&1
