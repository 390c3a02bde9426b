# FAST LDS-row A/B: ORB parity tests, then alternating stage timings old/new, then an SQ pass.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_orb.py -x -q --timeout 200 --timeout-method thread > gpurun_out/fast_ab_tests.log 2>&1 &&
for r in 1 2; do
  EAO_ACCEL_LIB=eao-slam_amd/lib/ab/libeao_old.so timeout -k 10 200 python -u tools/orb_stages.py > gpurun_out/fast_ab_old_$r.log 2>&1 &&
  timeout -k 10 200 python -u tools/orb_stages.py > gpurun_out/fast_ab_new_$r.log 2>&1 || exit 1
done &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmc_lds_new -o run -- python3 tools/pmc_extract.py > gpurun_out/pmc_lds_new.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_new -o run -- python3 tools/pmc_extract.py > gpurun_out/kt_new.log 2>&1 &&
db=$(python3 -c "import glob,sys; print(glob.glob(sys.argv[1] + '/**/*.db', recursive=True)[0])" gpurun_out/pmc_lds_new) && python3 tools/pmc_summary.py "$db" gpurun_out/pmc_lds_new.txt > /dev/null
