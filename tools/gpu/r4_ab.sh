# Round-4 kernel changes: forest (mask path, rank conversion, scalar RNG state) and the FAST
# whole-row ring gather (EAO_FAST_ROWS=1): parity first, then same-box A/B timings.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_assoc.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4_ab_assoc.log 2>&1 &&
EAO_FAST_ROWS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_orb.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4_ab_orb_rows.log 2>&1 &&
timeout -k 10 200 python -u tools/orb_stages.py --reps 10 > gpurun_out/r4_ab_orb_stages_base.log 2>&1 &&
EAO_FAST_ROWS=1 timeout -k 10 200 python -u tools/orb_stages.py --reps 10 > gpurun_out/r4_ab_orb_stages_rows.log 2>&1 &&
EAO_FAST_XCD=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_orb.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_ab_orb_xcd.log 2>&1 &&
EAO_FAST_XCD=1 timeout -k 10 200 python -u tools/orb_stages.py --reps 10 > gpurun_out/r4_ab_orb_stages_xcd.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r4_ab_pmc_fetch_base -o run -- python3 tools/pmc_extract.py > gpurun_out/r4_ab_pmc_fetch_base.log 2>&1 &&
EAO_FAST_XCD=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r4_ab_pmc_fetch_xcd -o run -- python3 tools/pmc_extract.py > gpurun_out/r4_ab_pmc_fetch_xcd.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_fr3.py tests/test_gpu_replay.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r4_ab_replay.log 2>&1 &&
for r in 1 2; do
  EAO_ACCEL_LIB=eao-slam_amd/lib/ab/base/libeao_accel.so timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" | sed "s/^/base /" &&
  EAO_SENTINEL_WAIT=0 timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" | sed "s/^/forest /" &&
  timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" | sed "s/^/forest+sentinel /" || break
done > gpurun_out/r4_ab_probe.log 2>&1 &&
timeout -k 10 120 python -u tools/micro/if_probe.py > gpurun_out/r4_ab_ifprobe_new.log 2>&1 &&
EAO_ACCEL_LIB=eao-slam_amd/lib/ab/base/libeao_accel.so timeout -k 10 120 python -u tools/micro/if_probe.py > gpurun_out/r4_ab_ifprobe_base.log 2>&1 &&
echo "== kernarg A/B" > gpurun_out/r4_ab_kernarg.log &&
for v in 0 1 0 1; do HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python -u tools/replay_probe.py 2>&1 | grep "pass 2" | sed "s/^/kernarg=$v /" >> gpurun_out/r4_ab_kernarg.log || break; done
