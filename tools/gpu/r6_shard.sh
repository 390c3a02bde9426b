# Round 6, the sharded association on the HSA lanes: GPU shard tests, then Config C at world 1 --
# unsharded, sharded (exchanges started with their launches, the default), sharded with exchanges
# started where they are read (EAO_SHARD_EAGER=0), alternating, same box.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-r6s}
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_lanes.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${P}_tests.log 2>&1 &&
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --config c --steps 3 --no-cpu-baseline > gpurun_out/${P}_c_$i.log 2>&1 &&
  timeout -k 10 200 python -u bench.py --config c --shard --steps 3 --no-cpu-baseline > gpurun_out/${P}_cs_$i.log 2>&1 &&
  EAO_SHARD_EAGER=0 timeout -k 10 200 python -u bench.py --config c --shard --steps 3 --no-cpu-baseline > gpurun_out/${P}_csl_$i.log 2>&1 || exit 1
done
