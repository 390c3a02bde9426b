# Round 6: kernel trace of the sharded Config C replay at world 1 on the HSA lanes (one timed step).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6k_shard -o run -- python3 bench.py --config c --shard --steps 1 --warmup 1 --frames 300 --no-cpu-baseline > gpurun_out/r6k_shard.log 2>&1
