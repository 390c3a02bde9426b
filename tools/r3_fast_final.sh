# Extraction kernels after the resize bands / FAST LDS rows: parity, stage times, counter passes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_golden.py tests/test_gpu_match.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ff_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/orb_stages.py --reps 10 > gpurun_out/ff_stages.log 2>&1 &&
P="timeout -s KILL 120 rocprofv3 --kernel-trace" &&
$P --pmc FETCH_SIZE -d gpurun_out/ff_fetch -o run -- python3 tools/pmc_extract.py > gpurun_out/ff_fetch.log 2>&1 &&
$P --pmc WRITE_SIZE -d gpurun_out/ff_write -o run -- python3 tools/pmc_extract.py > gpurun_out/ff_write.log 2>&1 &&
$P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/ff_sq -o run -- python3 tools/pmc_extract.py > gpurun_out/ff_sq.log 2>&1 &&
$P --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU -d gpurun_out/ff_wait -o run -- python3 tools/pmc_extract.py > gpurun_out/ff_wait.log 2>&1 &&
$P --pmc FETCH_SIZE -d gpurun_out/ff_fetch_b -o run -- python3 tools/pmc_extract.py --config b --reps 2 > gpurun_out/ff_fetch_b.log 2>&1 &&
$P --pmc WRITE_SIZE -d gpurun_out/ff_write_b -o run -- python3 tools/pmc_extract.py --config b --reps 2 > gpurun_out/ff_write_b.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ff_kt -o run -- python3 tools/pmc_extract.py > gpurun_out/ff_kt.log 2>&1 &&
for d in ff_fetch ff_write ff_sq ff_wait ff_fetch_b ff_write_b; do
  db=$(python3 -c "import glob,sys; print(glob.glob(sys.argv[1] + '/**/*.db', recursive=True)[0])" gpurun_out/$d) && python3 tools/pmc_summary.py "$db" gpurun_out/$d.txt > /dev/null || exit 1
done
