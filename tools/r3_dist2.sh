# k_distribute grid order (levels outermost): ORB parity (405 frames 640x480, 1080p), stage times.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_golden.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dist_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/orb_stages.py --reps 10 > gpurun_out/dist_stages.log 2>&1
