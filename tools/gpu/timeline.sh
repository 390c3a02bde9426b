# Association timeline: host events (EAO_REPLAY_TRACE) + kernel trace of the replay probe (tools/replay_timeline.py).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/tl_trace.bin
EAO_REPLAY_TRACE=gpurun_out/tl_trace.bin timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl_kt -o run -- python3 tools/replay_probe.py > gpurun_out/tl_kt.log 2>&1 &&
python3 tools/replay_timeline.py gpurun_out/tl_trace.bin "$(find gpurun_out/tl_kt -name "*.db" -print -quit)" > gpurun_out/tl_summary.txt 2>&1 &&
rm -f gpurun_out/tl_trace2.bin &&
EAO_REPLAY_TRACE=gpurun_out/tl_trace2.bin timeout -k 10 300 python3 tools/replay_probe.py > gpurun_out/tl_probe.log 2>&1 &&
python3 tools/replay_timeline.py gpurun_out/tl_trace2.bin > gpurun_out/tl_summary_noprof.txt 2>&1
