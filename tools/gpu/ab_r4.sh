#!/bin/bash
# Round-4 same-box A/B experiments on the GPU box, one function each (records under profiles/r04_ab_*):
#   bash tools/gpu/ab_r4.sh <name>      names: forest_fast rfl score lines lines_pmc lines_fused prep bench_ab overlap overlap2 front fastcmp fastcmp2 linebatch coreside linecu
# Switches of rejected variants live in the patches named beside them.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp

# forest_fast: Round-4 kernel changes: forest (mask path, rank conversion, scalar RNG state) and the FAST whole-row ring gather (EAO_FAST_ROWS=1): parity first, then same-box A/B timings. (EAO_FAST_ROWS and the forest variants: tools/patches/r4_forest_mask_rank_rejected.patch; removed since)
forest_fast() {
  timeout -k 10 300 python -u -m pytest tests/test_gpu_assoc.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4_ab_assoc.log 2>&1 &&
  EAO_FAST_ROWS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_orb.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4_ab_orb_rows.log 2>&1 &&
  timeout -k 10 200 python -u tools/orb_stages.py --reps 10 > gpurun_out/r4_ab_orb_stages_base.log 2>&1 &&
  EAO_FAST_ROWS=1 timeout -k 10 200 python -u tools/orb_stages.py --reps 10 > gpurun_out/r4_ab_orb_stages_rows.log 2>&1 &&
  EAO_FAST_XCD=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_orb.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_ab_orb_xcd.log 2>&1 &&
  EAO_FAST_XCD=1 timeout -k 10 200 python -u tools/orb_stages.py --reps 10 > gpurun_out/r4_ab_orb_stages_xcd.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r4_ab_pmc_fetch_base -o run -- python3 tools/pmc_extract.py > gpurun_out/r4_ab_pmc_fetch_base.log 2>&1 &&
  EAO_FAST_XCD=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r4_ab_pmc_fetch_xcd -o run -- python3 tools/pmc_extract.py > gpurun_out/r4_ab_pmc_fetch_xcd.log 2>&1 &&
  timeout -k 10 400 python -u -m pytest tests/test_gpu_fr3.py tests/test_gpu_replay.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r4_ab_replay.log 2>&1 &&
  for r in 1 2; do
    EAO_ACCEL_LIB=eao-slam_amd/lib/ab/base/libeao_accel.so timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" | sed "s/^/base /" &&
    EAO_SENTINEL_WAIT=0 timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" | sed "s/^/forest /" &&
    timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" | sed "s/^/forest+sentinel /" || break
  done > gpurun_out/r4_ab_probe.log 2>&1 &&
  timeout -k 10 120 python -u tools/micro/if_probe.py > gpurun_out/r4_ab_ifprobe_new.log 2>&1 &&
  EAO_ACCEL_LIB=eao-slam_amd/lib/ab/base/libeao_accel.so timeout -k 10 120 python -u tools/micro/if_probe.py > gpurun_out/r4_ab_ifprobe_base.log 2>&1 &&
  echo "== kernarg A/B" > gpurun_out/r4_ab_kernarg.log &&
  for v in 0 1 0 1; do HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python -u tools/replay_probe.py 2>&1 | grep "pass 2" | sed "s/^/kernarg=$v /" >> gpurun_out/r4_ab_kernarg.log || break; done
}

# rfl: Scalar RNG state of the forest's wave generator (readfirstlane): build cycles A/B, then closing measurements.
rfl() {
  timeout -k 10 300 python -u -m pytest tests/test_gpu_assoc.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_rfl_assoc.log 2>&1 &&
  timeout -k 10 120 python -u tools/micro/if_probe.py > gpurun_out/r4_rfl_ifprobe_new.log 2>&1 &&
  EAO_ACCEL_LIB=eao-slam_amd/lib/ab/base/libeao_accel.so timeout -k 10 120 python -u tools/micro/if_probe.py > gpurun_out/r4_rfl_ifprobe_base.log 2>&1 &&
  timeout -k 10 120 python -u tools/micro/if_probe.py > gpurun_out/r4_rfl_ifprobe_new2.log 2>&1 &&
  EAO_ACCEL_LIB=eao-slam_amd/lib/ab/base/libeao_accel.so timeout -k 10 120 python -u tools/micro/if_probe.py > gpurun_out/r4_rfl_ifprobe_base2.log 2>&1
}

# score: Forest score phase: points prefetched by the scoring waves during the build, CalculateC of every leaf size staged in LDS. Parity, then build / score cycles A/B and the replay probe A/B.
score() {
  timeout -k 10 300 python -u -m pytest tests/test_gpu_assoc.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_sc_assoc.log 2>&1 &&
  for r in 1 2; do
    timeout -k 10 120 python -u tools/micro/if_probe.py | grep "^n=" | sed "s/load.*gather/gather/; s/^/new  /" &&
    EAO_ACCEL_LIB=eao-slam_amd/lib/ab/base/libeao_accel.so timeout -k 10 120 python -u tools/micro/if_probe.py | grep "^n=" | sed "s/load.*gather/gather/; s/^/base /" || break
  done > gpurun_out/r4_sc_ifprobe.log 2>&1 &&
  for r in 1 2; do
    EAO_ACCEL_LIB=eao-slam_amd/lib/ab/base/libeao_accel.so timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" | cut -c1-60 | sed "s/^/base /" &&
    timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" | cut -c1-60 | sed "s/^/new  /" || break
  done > gpurun_out/r4_sc_probe.log 2>&1
}

# lines: Line stage: move-byte edge drawing (k_line_moves + k_edge_draw) against the base build: parity (GPU line tests, oracle check), then alternating same-box timings.
lines() {
  timeout -k 10 300 python -u -m pytest tests/test_gpu_lines.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4l_tests.log 2>&1 &&
  timeout -k 10 200 python -u tools/micro/lines_bench.py --check > gpurun_out/r4l_new_0.log 2>&1 &&
  for r in 1 2; do
    EAO_ACCEL_LIB=eao-slam_amd/lib/ab/base/libeao_accel.so timeout -k 10 200 python -u tools/micro/lines_bench.py > gpurun_out/r4l_base_$r.log 2>&1 &&
    timeout -k 10 200 python -u tools/micro/lines_bench.py > gpurun_out/r4l_new_$r.log 2>&1 || exit 1
  done &&
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4l_kt -o run -- python3 tools/micro/lines_bench.py > gpurun_out/r4l_kt.log 2>&1
}

# lines_pmc: 
lines_pmc() {
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d gpurun_out/r4l_pmc_sq -o run -- python3 tools/micro/lines_bench.py > gpurun_out/r4l_pmc_sq.log 2>&1
}

# lines_fused: Line stage: the fused walk + EDline workgroup (k_edge_lines, 8 or 4 waves) against the two-kernel path (EAO_LINES_FUSED=0): parity first, then alternating same-box timings.
lines_fused() {
  timeout -k 10 300 python -u -m pytest tests/test_gpu_lines.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4f_tests.log 2>&1 &&
  timeout -k 10 200 python -u tools/micro/lines_bench.py --check > gpurun_out/r4f_f8_0.log 2>&1 &&
  EAO_ACCEL_LIB=eao-slam_amd/lib/ab/fused4/libeao_accel.so timeout -k 10 200 python -u tools/micro/lines_bench.py --check > gpurun_out/r4f_f4_0.log 2>&1 &&
  for r in 1 2; do
    EAO_LINES_FUSED=0 timeout -k 10 200 python -u tools/micro/lines_bench.py > gpurun_out/r4f_two_$r.log 2>&1 &&
    timeout -k 10 200 python -u tools/micro/lines_bench.py > gpurun_out/r4f_f8_$r.log 2>&1 &&
    EAO_ACCEL_LIB=eao-slam_amd/lib/ab/fused4/libeao_accel.so timeout -k 10 200 python -u tools/micro/lines_bench.py > gpurun_out/r4f_f4_$r.log 2>&1 || exit 1
  done &&
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4f_kt -o run -- python3 tools/micro/lines_bench.py > gpurun_out/r4f_kt.log 2>&1
}

# prep: Look-ahead granularity: replay parity, then alternating probes (EAO_PREP_CHUNK points per look-ahead step; 1e9 = one step per phase, the earlier granularity).
prep() {
  timeout -k 10 400 python -u -m pytest tests/test_gpu_fr3.py tests/test_gpu_replay.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4p_tests.log 2>&1 &&
  for r in 1 2 3; do
    EAO_PREP_CHUNK=1000000000 timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" | sed "s/^/chunk=all /" &&
    EAO_PREP_CHUNK=128 timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" | sed "s/^/chunk=128 /" &&
    EAO_PREP_CHUNK=32 timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" | sed "s/^/chunk=32 /" || exit 1
  done > gpurun_out/r4p_probe.log 2>&1
}

# bench_ab: Headline A/B on one box: the EAO bench with the fused line workgroup (default), with the two-kernel line path (EAO_LINES_FUSED=0), and with the round's base library (lib/ab/base).
bench_ab() {
  for r in 1 2; do
    timeout -k 10 300 python -u bench.py > gpurun_out/r4b_fused_$r.log 2>&1 &&
    EAO_LINES_FUSED=0 timeout -k 10 300 python -u bench.py > gpurun_out/r4b_two_$r.log 2>&1 &&
    EAO_ACCEL_LIB=eao-slam_amd/lib/ab/base/libeao_accel.so timeout -k 10 300 python -u bench.py > gpurun_out/r4b_base_$r.log 2>&1 || exit 1
  done
}

# overlap: Front / association overlap: step time with the front overlapped (line stage in 1, 4 or 8 launches, association on a second thread) and enqueued before the association (default), alternating.
overlap() {
  for r in 1 2; do
    for v in "--thread --line-batches 1" "--thread --line-batches 4" "--thread --line-batches 8" ""; do
      timeout -k 10 300 python -u bench.py --no-cpu-baseline $v > gpurun_out/r4o.log 2>&1 || exit 1
      tail -1 gpurun_out/r4o.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$v', round(d['ms_per_step'],2), round(d['line_detect']['ms_per_step'],2), round(d['assoc_profile_us_per_frame']['frame'],1), round(d['assoc_profile_us_per_frame']['assoc_loop'],1))" || exit 1
    done
  done > gpurun_out/r4o_summary.txt 2>&1
}

# overlap2: Association on a second thread (--thread) vs the frame work enqueued before the association (default), 4 alternating pairs.
overlap2() {
  for r in 1 2 3 4; do
    for v in "--thread" ""; do
      timeout -k 10 300 python -u bench.py --no-cpu-baseline $v > gpurun_out/r4o.log 2>&1 || exit 1
      tail -1 gpurun_out/r4o.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('[$v]', round(d['ms_per_step'],2), round(d['assoc_profile_us_per_frame']['frame'],1), round(d['assoc_profile_us_per_frame']['assoc_loop'],1))" || exit 1
    done
  done > gpurun_out/r4o2_summary.txt 2>&1
}

# front: Contention of the frame work with the association (default ordering): full CUs, CU-masked front stream (3/4, 2/4 of the CUs), line stage in 4 launches; alternating on one box. (its CU-mask variant was a bench option removed after the run)
front() {
  for r in 1 2 3; do
    for v in "" "--front-cus 3" "--front-cus 2" "--line-batches 4"; do
      timeout -k 10 300 python -u bench.py --no-cpu-baseline $v > gpurun_out/r4fr.log 2>&1 || exit 1
      tail -1 gpurun_out/r4fr.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('[$v]', round(d['ms_per_step'],2), round(d['line_detect']['ms_per_step'],2), round(d['extract_ms_per_step'],2), round(d['assoc_profile_us_per_frame']['frame'],1), d['parity']['assoc_ids_identical'] if 'parity' in d else '')" || exit 1
    done
  done > gpurun_out/r4fr_summary.txt 2>&1
}

# fastcmp: FAST compacted strengths (EAO_FAST_CMP, default on) vs the dense sweep: ORB parity first, then alternating stage timings (405 frames 640x480, and a 1080p batch), then FAST counter passes. (EAO_FAST_CMP: tools/patches/r4_fast_compacted_rejected.patch)
fastcmp() {
  timeout -k 10 300 python -u -m pytest tests/test_gpu_orb.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4c_tests.log 2>&1 &&
  for r in 1 2; do
    EAO_FAST_CMP=0 timeout -k 10 200 python -u tools/micro/orb_stages.py > gpurun_out/r4c_dense_$r.log 2>&1 &&
    timeout -k 10 200 python -u tools/micro/orb_stages.py > gpurun_out/r4c_cmp_$r.log 2>&1 &&
    EAO_FAST_CMP=0 timeout -k 10 200 python -u tools/micro/orb_stages.py 256 1920 1080 4000 > gpurun_out/r4c_dense1080_$r.log 2>&1 &&
    timeout -k 10 200 python -u tools/micro/orb_stages.py 256 1920 1080 4000 > gpurun_out/r4c_cmp1080_$r.log 2>&1 || exit 1
  done &&
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY -d gpurun_out/r4c_pmc_sq -o run -- python3 tools/pmc_extract.py > gpurun_out/r4c_pmc_sq.log 2>&1
}

# fastcmp2: FAST compacted strengths vs dense on the EAO bench's own frames (structured texture) and on the plain texture (Config B's), alternating; the bench's own fast stage with both. (EAO_FAST_CMP: tools/patches/r4_fast_compacted_rejected.patch)
fastcmp2() {
  for r in 1 2; do
    for c in 0 1; do
      EAO_FAST_CMP=$c timeout -k 10 200 python -u tools/micro/orb_stages.py > gpurun_out/r4c2_s_$c.log 2>&1 &&
      EAO_FAST_CMP=$c STRUCT=0 timeout -k 10 200 python -u tools/micro/orb_stages.py > gpurun_out/r4c2_p_$c.log 2>&1 &&
      EAO_FAST_CMP=$c STRUCT=0 timeout -k 10 200 python -u tools/micro/orb_stages.py 256 1920 1080 4000 > gpurun_out/r4c2_b_$c.log 2>&1 &&
      echo "cmp=$c struct640: $(tail -1 gpurun_out/r4c2_s_$c.log) | plain640: $(tail -1 gpurun_out/r4c2_p_$c.log | sed 's/.*fast/fast/;s/ distribute.*//') | plain1080: $(tail -1 gpurun_out/r4c2_b_$c.log | sed 's/.*fast/fast/;s/ distribute.*//')" || exit 1
    done
  done > gpurun_out/r4c2_summary.txt 2>&1 &&
  for c in 0 1; do
    EAO_FAST_CMP=$c timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4c2_bench_$c.log 2>&1 || exit 1
  done
}

# linebatch: Line stage split into K launches (fewer concurrent k_edge_lines workgroups, whose ~250-VGPR waves fill the register files of the CUs they hold) against one launch; default ordering; 3 alternating rounds on one box.
linebatch() {
  for r in 1 2 3; do
    for v in 1 4 8; do
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --line-batches $v > gpurun_out/r4lb.log 2>&1 || exit 1
      tail -1 gpurun_out/r4lb.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('[line-batches $v]', round(d['ms_per_step'],2), round(d['line_detect']['ms_per_step'],2), round(d['assoc_profile_us_per_frame']['frame'],1), round(d['assoc_profile_us_per_frame']['assoc_loop'],1))" || exit 1
    done
  done > gpurun_out/r4lb_summary.txt 2>&1
}

# coreside: Association kernels at <= 64 VGPRs (4 waves per SIMD fit beside one k_edge_lines wave) against the base build, with the line stage in 1 or 2 launches; EAO bench, alternating on one box.
coreside() {
  timeout -k 10 400 python -u -m pytest tests/test_gpu_assoc.py tests/test_gpu_fr3.py tests/test_gpu_replay.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4co_tests.log 2>&1 &&
  for r in 1 2 3; do
    for v in "base 1" "new 1" "new 2"; do
      set -- $v
      lib=""; [ "$1" = base ] && lib=eao-slam_amd/lib/ab/base/libeao_accel.so
      EAO_ACCEL_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --line-batches $2 > gpurun_out/r4co.log 2>&1 || exit 1
      tail -1 gpurun_out/r4co.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('[$1 lb=$2]', round(d['ms_per_step'],2), round(d['line_detect']['ms_per_step'],2), round(d['assoc_profile_us_per_frame']['frame'],1), round(d['assoc_profile_us_per_frame']['assoc_loop'],1))" || exit 1
    done
  done > gpurun_out/r4co_summary.txt 2>&1 &&
  timeout -k 10 200 python -u tools/replay_probe.py > gpurun_out/r4co_probe_new.log 2>&1 &&
  EAO_ACCEL_LIB=eao-slam_amd/lib/ab/base/libeao_accel.so timeout -k 10 200 python -u tools/replay_probe.py > gpurun_out/r4co_probe_base.log 2>&1
}

# linecu: Line stage on a CU-masked stream (EAO_LINES_CU_QUARTERS=q: q of every 4 CUs) against the full device; EAO bench, default ordering, alternating on one box; then the line tests with q=2. (EAO_LINES_CU_QUARTERS: tools/patches/r4_lines_cu_mask_rejected.patch)
linecu() {
  for r in 1 2 3; do
    for q in 4 3 2 1; do
      EAO_LINES_CU_QUARTERS=$q timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4cu.log 2>&1 || exit 1
      tail -1 gpurun_out/r4cu.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('[cu quarters $q]', round(d['ms_per_step'],2), round(d['line_detect']['ms_per_step'],2), round(d['assoc_profile_us_per_frame']['frame'],1), round(d['assoc_profile_us_per_frame']['assoc_loop'],1), d['parity']['lines_bitexact'] if 'parity' in d else '')" || exit 1
    done
  done > gpurun_out/r4cu_summary.txt 2>&1 &&
  EAO_LINES_CU_QUARTERS=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_lines.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4cu_tests.log 2>&1
}


# ldelay: marginal cost of forest-batch launch time on the association chain (knob EAO_LAUNCH_DELAY_US: a busy wait after each batch launch in kick(), removed after the measurement): replay probe pass 2 at 0 / 13 / 26 us of extra host time per batch launch, alternating.
ldelay() {
  for r in 1 2 3; do
    for d in 0 13 26; do
      EAO_LAUNCH_DELAY_US=$d timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" | cut -c1-60 | sed "s/^/delay=$d /" || exit 1
    done
  done > gpurun_out/r4_ldelay.log 2>&1
}

# fastd16: FAST kernel variant (the working tree build) against the base build (lib/ab/base): ORB parity, then stage timings alternating (structured / plain 640x480, plain 1080p). Used for the d16 ring gather (rejected) and the three-pair trip.
fastd16() {
  timeout -k 10 300 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4d_tests.log 2>&1 &&
  for r in 1 2; do
    for lib in eao-slam_amd/lib/ab/base/libeao_accel.so eao-slam_amd/lib/libeao_accel.so; do
      n=$(basename $(dirname $lib))
      EAO_ACCEL_LIB=$lib timeout -k 10 200 python -u tools/micro/orb_stages.py > gpurun_out/r4d_s.log 2>&1 &&
      EAO_ACCEL_LIB=$lib STRUCT=0 timeout -k 10 200 python -u tools/micro/orb_stages.py > gpurun_out/r4d_p.log 2>&1 &&
      EAO_ACCEL_LIB=$lib STRUCT=0 timeout -k 10 200 python -u tools/micro/orb_stages.py 256 1920 1080 4000 > gpurun_out/r4d_b.log 2>&1 &&
      echo "$n struct640: $(tail -1 gpurun_out/r4d_s.log) | plain640: $(tail -1 gpurun_out/r4d_p.log | sed 's/.*fast/fast/;s/ distribute.*//') | plain1080: $(tail -1 gpurun_out/r4d_b.log | sed 's/.*fast/fast/;s/ distribute.*//')" || exit 1
    done
  done > gpurun_out/r4d_summary.txt 2>&1
}

[ $# -eq 1 ] && declare -F "$1" > /dev/null || { echo "usage: $0 <experiment>"; exit 2; }
"$1"
