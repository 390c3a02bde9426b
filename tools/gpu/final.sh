# Closing measurements of a round (prefix P): GPU suite, smoke, EAO bench (+ kernel trace), Config C
# sharded at world 1, Full, Config B, replay probe, FAST counter passes (FETCH / WRITE / SQ).
set -o pipefail
P=${P:-r5}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs > gpurun_out/${P}_gputest.log 2>&1 &&
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${P}_smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/${P}_bench.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c --shard > gpurun_out/${P}_bench_c_shard.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c > gpurun_out/${P}_bench_c.log 2>&1 &&
timeout -k 10 400 python -u bench.py --config full > gpurun_out/${P}_bench_full.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config b > gpurun_out/${P}_bench_b.log 2>&1 &&
timeout -k 10 200 python -u tools/replay_probe.py > gpurun_out/${P}_probe.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${P}_kt -o run -- python3 bench.py --steps 2 --no-cpu-baseline > gpurun_out/${P}_kt.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${P}_pmc_fetch -o run -- python3 tools/pmc_extract.py > gpurun_out/${P}_pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${P}_pmc_write -o run -- python3 tools/pmc_extract.py > gpurun_out/${P}_pmc_write.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY -d gpurun_out/${P}_pmc_sq -o run -- python3 tools/pmc_extract.py > gpurun_out/${P}_pmc_sq.log 2>&1
