# Round-3 counter passes of the extraction kernels (one rocprofv3 --pmc pass per group,
# each under its own time limit; MI355X_MICROARCH.md HBM / LDS sections for the units).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P="timeout -s KILL 120 rocprofv3 --kernel-trace"
$P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmc_lds -o run -- python3 tools/pmc_extract.py > gpurun_out/pmc_lds.log 2>&1 &&
$P --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU -d gpurun_out/pmc_wait -o run -- python3 tools/pmc_extract.py > gpurun_out/pmc_wait.log 2>&1 &&
$P --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_b -o run -- python3 tools/pmc_extract.py --config b --reps 2 > gpurun_out/pmc_fetch_b.log 2>&1 &&
$P --pmc WRITE_SIZE -d gpurun_out/pmc_write_b -o run -- python3 tools/pmc_extract.py --config b --reps 2 > gpurun_out/pmc_write_b.log 2>&1 &&
$P --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_a -o run -- python3 tools/pmc_extract.py > gpurun_out/pmc_fetch_a.log 2>&1 &&
for d in pmc_lds pmc_wait pmc_fetch_b pmc_write_b pmc_fetch_a; do
  db=$(python3 -c "import glob,sys; print(glob.glob(sys.argv[1] + '/**/*.db', recursive=True)[0])" gpurun_out/$d) && python3 tools/pmc_summary.py "$db" gpurun_out/$d.txt > /dev/null || exit 1
done
