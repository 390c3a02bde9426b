# FAST compacted strengths (EAO_FAST_CMP, default on) vs the dense sweep: ORB parity first, then
# alternating stage timings (405 frames 640x480, and a 1080p batch), then FAST counter passes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_orb.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4c_tests.log 2>&1 &&
for r in 1 2; do
  EAO_FAST_CMP=0 timeout -k 10 200 python -u tools/micro/orb_stages.py > gpurun_out/r4c_dense_$r.log 2>&1 &&
  timeout -k 10 200 python -u tools/micro/orb_stages.py > gpurun_out/r4c_cmp_$r.log 2>&1 &&
  EAO_FAST_CMP=0 timeout -k 10 200 python -u tools/micro/orb_stages.py 256 1920 1080 4000 > gpurun_out/r4c_dense1080_$r.log 2>&1 &&
  timeout -k 10 200 python -u tools/micro/orb_stages.py 256 1920 1080 4000 > gpurun_out/r4c_cmp1080_$r.log 2>&1 || exit 1
done &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY -d gpurun_out/r4c_pmc_sq -o run -- python3 tools/pmc_extract.py > gpurun_out/r4c_pmc_sq.log 2>&1
