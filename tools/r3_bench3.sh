set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py > gpurun_out/r3_bench3.log 2>&1 &&
timeout -k 10 900 python -u bench.py --config full --steps 2 > gpurun_out/r3_bench3_full.log 2>&1
