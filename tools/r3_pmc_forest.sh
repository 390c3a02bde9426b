# Counter passes of the isolation-forest kernels (tools/micro/if_probe.py: 7 cloud sizes x 23 calls),
# one rocprofv3 --pmc pass per group, each under its own time limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P="timeout -s KILL 120 rocprofv3 --kernel-trace"
$P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmcf_lds -o run -- python3 tools/micro/if_probe.py > gpurun_out/pmcf_lds.log 2>&1 &&
$P --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU -d gpurun_out/pmcf_wait -o run -- python3 tools/micro/if_probe.py > gpurun_out/pmcf_wait.log 2>&1 &&
for d in pmcf_lds pmcf_wait; do
  db=$(python3 -c "import glob,sys; print(glob.glob(sys.argv[1] + '/**/*.db', recursive=True)[0])" gpurun_out/$d) && python3 tools/pmc_summary.py "$db" gpurun_out/$d.txt > /dev/null || exit 1
done
