# Round 6: the default bench line (EAO) and the Full line, nothing else.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-r6z}
timeout -k 10 500 python -u bench.py > gpurun_out/${P}_bench.log 2>&1 &&
timeout -k 10 600 python -u bench.py --config full > gpurun_out/${P}_bench_full.log 2>&1
