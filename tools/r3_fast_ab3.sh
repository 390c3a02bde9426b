# Resize tiles + FAST LDS rows: ORB parity, then alternating stage timings, then FETCH of the tiles.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_orb.py tests/test_gpu_golden.py -rs -x -q --timeout 200 --timeout-method thread > gpurun_out/fast_ab3_tests.log 2>&1 &&
for r in 1 2; do
  timeout -k 10 200 python -u tools/orb_stages.py --reps 8 > gpurun_out/fast_ab3_cur_$r.log 2>&1 &&
  EAO_ACCEL_LIB=eao-slam_amd/lib/ab/libeao_rs288.so timeout -k 10 200 python -u tools/orb_stages.py --reps 8 > gpurun_out/fast_ab3_rs288_$r.log 2>&1 || exit 1
done &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_tile -o run -- python3 tools/pmc_extract.py > gpurun_out/pmc_fetch_tile.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_tile_b -o run -- python3 tools/pmc_extract.py --config b --reps 2 > gpurun_out/pmc_fetch_tile_b.log 2>&1 &&
for d in pmc_fetch_tile pmc_fetch_tile_b; do
  db=$(python3 -c "import glob,sys; print(glob.glob(sys.argv[1] + '/**/*.db', recursive=True)[0])" gpurun_out/$d) && python3 tools/pmc_summary.py "$db" gpurun_out/$d.txt > /dev/null || exit 1
done
