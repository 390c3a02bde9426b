# Round 6, the HSA lanes: GPU tests of the lanes and the replays on them, then rocprofv3 over the
# lane self-test and the replay probe with the ring-end split (the fix), and last the self-test with
# the split off (EAO_HSA_WRAP_SPLIT=0, the round-5 behaviour) and the SIGSEGV diagnosis on: the
# expected reproduction of the round-5 host fault, so it runs last.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-r6a}
SELF="import sys; sys.path.insert(0, 'eao-slam_amd/python'); import eao_accel as ea; print('packets', ea.lane_selftest(0))"
timeout -k 10 400 python -u -m pytest tests/test_gpu_lanes.py tests/test_c99_consumer.py tests/test_gpu_shard.py tests/test_gpu_replay.py tests/test_gpu_fr3.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${P}_tests.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${P}_rp_self -o run -- python3 -c "$SELF" > gpurun_out/${P}_rp_self.log 2>&1 &&
EAO_PROBE_PASSES=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${P}_rp_probe -o run -- python3 tools/replay_probe.py > gpurun_out/${P}_rp_probe.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c --shard --steps 3 > gpurun_out/${P}_bench_c_shard.log 2>&1 &&
EAO_SHARD_HSA=0 timeout -k 10 300 python -u bench.py --config c --shard --steps 3 --no-cpu-baseline > gpurun_out/${P}_bench_c_shard_hip.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c --steps 3 --no-cpu-baseline > gpurun_out/${P}_bench_c.log 2>&1 &&
EAO_HSA_WRAP_SPLIT=0 EAO_SEGV_DIAG=1 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${P}_rp_nosplit -o run -- python3 -c "$SELF" > gpurun_out/${P}_rp_nosplit.log 2>&1
