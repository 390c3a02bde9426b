# Two ranks on one MI355X (gloo: RCCL refuses two ranks on one device): the bench's --gpus N launcher path.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
EAO_DIST_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --steps 3 --no-cpu-baseline > gpurun_out/n2.log 2>&1
