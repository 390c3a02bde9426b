# HEAD check on MI355X: GPU suite, EAO bench, forest phase probe (normal + stamp build), replay probe.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs > gpurun_out/h_gputest.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/h_bench.log 2>&1 &&
timeout -k 10 120 python -u tools/micro/if_probe.py > gpurun_out/h_if_probe.txt 2>&1 &&
EAO_ACCEL_LIB=eao-slam_amd/lib/prof/libeao_accel.so timeout -k 10 120 python -u tools/micro/if_probe.py > gpurun_out/h_if_probe_prof.txt 2>&1 &&
timeout -k 10 200 python -u tools/replay_probe.py > gpurun_out/h_probe.log 2>&1
