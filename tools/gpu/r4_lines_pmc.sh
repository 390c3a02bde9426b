set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d gpurun_out/r4l_pmc_sq -o run -- python3 tools/micro/lines_bench.py > gpurun_out/r4l_pmc_sq.log 2>&1
