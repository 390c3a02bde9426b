# Round 6: kernel trace of the EAO bench step on the HSA lanes (2 timed steps), for the association
# dispatch outliers beside the line stage (tools/kt_outliers.py).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-r6x}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${P}_kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dropin > gpurun_out/${P}_bench.log 2>&1
