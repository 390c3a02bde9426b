# Association kernels at <= 64 VGPRs (4 waves per SIMD fit beside one k_edge_lines wave) against
# the base build, with the line stage in 1 or 2 launches; EAO bench, alternating on one box.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_assoc.py tests/test_gpu_fr3.py tests/test_gpu_replay.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4co_tests.log 2>&1 &&
for r in 1 2 3; do
  for v in "base 1" "new 1" "new 2"; do
    set -- $v
    lib=""; [ "$1" = base ] && lib=eao-slam_amd/lib/ab/base/libeao_accel.so
    EAO_ACCEL_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --line-batches $2 > gpurun_out/r4co.log 2>&1 || exit 1
    tail -1 gpurun_out/r4co.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('[$1 lb=$2]', round(d['ms_per_step'],2), round(d['line_detect']['ms_per_step'],2), round(d['assoc_profile_us_per_frame']['frame'],1), round(d['assoc_profile_us_per_frame']['assoc_loop'],1))" || exit 1
  done
done > gpurun_out/r4co_summary.txt 2>&1 &&
timeout -k 10 200 python -u tools/replay_probe.py > gpurun_out/r4co_probe_new.log 2>&1 &&
EAO_ACCEL_LIB=eao-slam_amd/lib/ab/base/libeao_accel.so timeout -k 10 200 python -u tools/replay_probe.py > gpurun_out/r4co_probe_base.log 2>&1
