# Round 6: kernel trace of the drop-in leg (both passes), to see where the overlapped pass's matching waits.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${P:-r6dk} -o run -- python3 tools/micro/dropin_only.py 120 > gpurun_out/${P:-r6dk}.log 2>&1
