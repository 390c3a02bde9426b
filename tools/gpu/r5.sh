#!/bin/bash
# Round-5 GPU runs, one function each: bash tools/gpu/r5.sh <name> [args]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp

# base: state of the tree on this box: EAO bench, replay probe, extraction stages
base() {
  timeout -k 10 500 python -u bench.py > gpurun_out/r5_base_bench.log 2>&1 &&
  timeout -k 10 200 python -u tools/replay_probe.py > gpurun_out/r5_base_probe.log 2>&1 &&
  timeout -k 10 200 python -u tools/micro/orb_stages.py > gpurun_out/r5_base_orb.log 2>&1 &&
  timeout -k 10 200 python -u tools/micro/orb_stages.py 256 1920 1080 4000 >> gpurun_out/r5_base_orb.log 2>&1
}

# pyr: LDS-staged pyramid (k_resize_lds) against k_resize_tile (EAO_RESIZE=0): parity, stage A/B, traffic
pyr() {
  timeout -k 10 400 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_lines.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r5_pyr_tests.log 2>&1 &&
  for r in 1 2; do
    EAO_RESIZE=0 timeout -k 10 200 python -u tools/micro/orb_stages.py | sed "s/^/tile /" &&
    timeout -k 10 200 python -u tools/micro/orb_stages.py | sed "s/^/lds  /" &&
    EAO_RESIZE=0 timeout -k 10 200 python -u tools/micro/orb_stages.py 256 1920 1080 4000 | sed "s/^/tile /" &&
    timeout -k 10 200 python -u tools/micro/orb_stages.py 256 1920 1080 4000 | sed "s/^/lds  /" || exit 1
  done > gpurun_out/r5_pyr_stages.log 2>&1 &&
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_pyr_kt -o run -- python3 tools/pmc_extract.py > gpurun_out/r5_pyr_kt.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r5_pyr_pmc_fetch -o run -- python3 tools/pmc_extract.py > gpurun_out/r5_pyr_pmc_fetch.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r5_pyr_pmc_write -o run -- python3 tools/pmc_extract.py > gpurun_out/r5_pyr_pmc_write.log 2>&1
}

# lsingle: single-frame line detection latency, fused and two-kernel (walk / EDline split in the trace)
lsingle() {
  timeout -k 10 200 python -u tools/micro/lines_single.py 64 --check > gpurun_out/r5_lsingle.log 2>&1 &&
  EAO_LINES_FUSED=0 timeout -k 10 200 python -u tools/micro/lines_single.py 64 >> gpurun_out/r5_lsingle.log 2>&1 &&
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_lsingle_kt -o run -- python3 tools/micro/lines_single.py 32 > gpurun_out/r5_lsingle_kt.log 2>&1 &&
  EAO_LINES_FUSED=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_lsingle_kt2 -o run -- python3 tools/micro/lines_single.py 32 > gpurun_out/r5_lsingle_kt2.log 2>&1
}

# s2: NP direct counts + one-wave small forests + resize with early loads: parity, then A/B
s2() {
  timeout -k 10 500 python -u -m pytest tests/test_gpu_assoc.py tests/test_gpu_lines.py tests/test_gpu_orb.py tests/test_gpu_chain.py tests/test_gpu_fr3.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r5_s2_tests.log 2>&1 &&
  for r in 1 2; do
    EAO_RESIZE=0 timeout -k 10 200 python -u tools/micro/orb_stages.py | sed "s/^/tile /" &&
    timeout -k 10 200 python -u tools/micro/orb_stages.py | sed "s/^/lds  /" &&
    EAO_RESIZE=0 timeout -k 10 200 python -u tools/micro/orb_stages.py 256 1920 1080 4000 | sed "s/^/tile /" &&
    timeout -k 10 200 python -u tools/micro/orb_stages.py 256 1920 1080 4000 | sed "s/^/lds  /" || exit 1
  done > gpurun_out/r5_s2_stages.log 2>&1 &&
  timeout -k 10 200 python -u tools/micro/lines_single.py 64 --check > gpurun_out/r5_s2_lsingle.log 2>&1 &&
  EAO_LINES_SPEC=0 timeout -k 10 200 python -u tools/micro/lines_single.py 64 >> gpurun_out/r5_s2_lsingle.log 2>&1 &&
  for r in 1 2; do
    echo "## base (EAO_NP_DIRECT=0 EAO_IF_SMALL=0)" && EAO_NP_DIRECT=0 EAO_IF_SMALL=0 timeout -k 10 200 python -u tools/replay_probe.py &&
    echo "## np direct" && EAO_IF_SMALL=0 timeout -k 10 200 python -u tools/replay_probe.py &&
    echo "## np direct + small forest" && timeout -k 10 200 python -u tools/replay_probe.py || exit 1
  done > gpurun_out/r5_s2_probe.log 2>&1 &&
  timeout -k 10 300 python -u bench.py > gpurun_out/r5_s2_bench.log 2>&1
}

# s3: association timeline on this build, single-call extract / motion split, pyramid traffic
s3() {
  bash tools/gpu/timeline.sh &&
  timeout -k 10 200 python -u tools/micro/dropin_single.py 64 > gpurun_out/r5_s3_dropin.log 2>&1 &&
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_s3_dropin_kt -o run -- python3 tools/micro/dropin_single.py 32 > gpurun_out/r5_s3_dropin_kt.log 2>&1 &&
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_s3_lsingle_kt -o run -- python3 tools/micro/lines_single.py 32 > gpurun_out/r5_s3_lsingle_kt.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r5_s3_pmc_fetch -o run -- python3 tools/pmc_extract.py > gpurun_out/r5_s3_pmc_fetch.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r5_s3_pmc_write -o run -- python3 tools/pmc_extract.py > gpurun_out/r5_s3_pmc_write.log 2>&1 &&
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_s3_orb_kt -o run -- python3 tools/pmc_extract.py > gpurun_out/r5_s3_orb_kt.log 2>&1
}

# s4: merge look-ahead loads, motion search in rounds + wave-per-query candidates: parity, single-call split, bench
s4() {
  timeout -k 10 500 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_lines.py tests/test_gpu_chain.py tests/test_gpu_fr3.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r5_s4_tests.log 2>&1 &&
  timeout -k 10 200 python -u tools/micro/dropin_single.py 64 > gpurun_out/r5_s4_single.log 2>&1 &&
  timeout -k 10 200 python -u tools/micro/lines_single.py 64 --check >> gpurun_out/r5_s4_single.log 2>&1 &&
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_s4_dropin_kt -o run -- python3 tools/micro/dropin_single.py 32 > gpurun_out/r5_s4_dropin_kt.log 2>&1 &&
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_s4_lsingle_kt -o run -- python3 tools/micro/lines_single.py 32 > gpurun_out/r5_s4_lsingle_kt.log 2>&1 &&
  timeout -k 10 300 python -u bench.py > gpurun_out/r5_s4_bench.log 2>&1
}

# s5: merge with the writer wave: line parity, single-frame time and split
s5() {
  timeout -k 10 300 python -u -m pytest tests/test_gpu_lines.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r5_s5_tests.log 2>&1 &&
  timeout -k 10 200 python -u tools/micro/lines_single.py 64 --check > gpurun_out/r5_s5_single.log 2>&1 &&
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_s5_lsingle_kt -o run -- python3 tools/micro/lines_single.py 32 > gpurun_out/r5_s5_lsingle_kt.log 2>&1
}

# hsa: association launches through HSA lanes (AQL packets) against HIP streams (EAO_HSA_LANES=0)
hsa() {
  timeout -k 10 400 python -u -m pytest tests/test_gpu_fr3.py tests/test_gpu_replay.py tests/test_gpu_assoc.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r5_hsa_tests.log 2>&1 &&
  for r in 1 2; do
    echo "## hip streams" && EAO_HSA_LANES=0 timeout -k 10 200 python -u tools/replay_probe.py &&
    echo "## hsa lanes" && timeout -k 10 200 python -u tools/replay_probe.py || exit 1
  done > gpurun_out/r5_hsa_probe.log 2>&1 &&
  timeout -k 10 300 python -u bench.py > gpurun_out/r5_hsa_bench.log 2>&1
}

# hsa2: HSA lane variants (acquire scope, kernargs in device memory) against HIP streams
hsa2() {
  for r in 1 2; do
    echo "## hsa acq agent, host kernargs" && timeout -k 10 200 python -u tools/replay_probe.py &&
    echo "## hip streams" && EAO_HSA_LANES=0 timeout -k 10 200 python -u tools/replay_probe.py &&
    echo "## hsa acq system" && EAO_HSA_ACQ=system timeout -k 10 200 python -u tools/replay_probe.py || exit 1
  done > gpurun_out/r5_hsa2_probe.log 2>&1
}
# hsa3: kernel arguments in device memory (BAR writes, HDP flush, read-back) against the kernarg pool
hsa3() {
  for r in 1 2; do
    echo "## hsa host kernargs" && timeout -k 10 200 python -u tools/replay_probe.py &&
    echo "## hsa dev kernargs" && EAO_HSA_KARG=dev timeout -k 10 200 python -u tools/replay_probe.py || exit 1
  done > gpurun_out/r5_hsa3_probe.log 2>&1
}

# hsa4: device kernargs by default: association suite, A/B against HIP streams and host kernargs, bench
hsa4() {
  timeout -k 10 500 python -u -m pytest tests/test_gpu_fr3.py tests/test_gpu_replay.py tests/test_gpu_assoc.py tests/test_gpu_chain.py tests/test_gpu_shard.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r5_hsa4_tests.log 2>&1 &&
  for r in 1 2; do
    echo "## hsa dev kernargs" && timeout -k 10 200 python -u tools/replay_probe.py &&
    echo "## hip streams" && EAO_HSA_LANES=0 timeout -k 10 200 python -u tools/replay_probe.py &&
    echo "## hsa host kernargs" && EAO_HSA_KARG=host timeout -k 10 200 python -u tools/replay_probe.py || exit 1
  done > gpurun_out/r5_hsa4_probe.log 2>&1 &&
  timeout -k 10 300 python -u bench.py > gpurun_out/r5_hsa4_bench.log 2>&1
}

# fsst: the frame start's inputs staged to device memory ahead of its forest waits (EAO_FS_STAGE=1)
fsst() {
  EAO_FS_STAGE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_fr3.py tests/test_gpu_replay.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r5_fsst_tests.log 2>&1 &&
  for r in 1 2; do
    echo "## in place" && timeout -k 10 200 python -u tools/replay_probe.py &&
    echo "## staged" && EAO_FS_STAGE=1 timeout -k 10 200 python -u tools/replay_probe.py || exit 1
  done > gpurun_out/r5_fsst_probe.log 2>&1 &&
  rm -rf gpurun_out/tl_kt && EAO_FS_STAGE=1 bash tools/gpu/timeline.sh && cp gpurun_out/tl_summary.txt gpurun_out/tl_fsst_summary.txt && rm -rf gpurun_out/tl_kt
}

# hsa5: batched lane commits (one kernarg flush + doorbell per record): suite, A/B against HIP streams
hsa5() {
  timeout -k 10 500 python -u -m pytest tests/test_gpu_fr3.py tests/test_gpu_replay.py tests/test_gpu_assoc.py tests/test_gpu_chain.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r5_hsa5_tests.log 2>&1 &&
  for r in 1 2; do
    echo "## hsa lanes" && timeout -k 10 200 python -u tools/replay_probe.py &&
    echo "## hip streams" && EAO_HSA_LANES=0 timeout -k 10 200 python -u tools/replay_probe.py || exit 1
  done > gpurun_out/r5_hsa5_probe.log 2>&1
}

# eager: forests launched per detection (EAO_EAGER_KICK=1) on the HSA lanes
eager() {
  EAO_EAGER_KICK=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_fr3.py tests/test_gpu_replay.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_eager_tests.log 2>&1 &&
  for r in 1 2; do
    echo "## end-of-loop kick" && timeout -k 10 200 python -u tools/replay_probe.py &&
    echo "## eager kick" && EAO_EAGER_KICK=1 timeout -k 10 200 python -u tools/replay_probe.py || exit 1
  done > gpurun_out/r5_eager_probe.log 2>&1
}

# bar: forest batch inputs written through the BAR (no k_stage) against pinned + k_stage
bar() {
  timeout -k 10 500 python -u -m pytest tests/test_gpu_fr3.py tests/test_gpu_replay.py tests/test_gpu_assoc.py tests/test_gpu_chain.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_bar_tests.log 2>&1 &&
  for r in 1 2; do
    echo "## bar inputs" && timeout -k 10 200 python -u tools/replay_probe.py &&
    echo "## pinned + k_stage" && EAO_BAR_INPUTS=0 timeout -k 10 200 python -u tools/replay_probe.py || exit 1
  done > gpurun_out/r5_bar_probe.log 2>&1
}

# barfs: the frame start's inputs written through the BAR too (EAO_BAR_FS=0: pinned, read in place)
barfs() {
  timeout -k 10 500 python -u -m pytest tests/test_gpu_fr3.py tests/test_gpu_replay.py tests/test_gpu_chain.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_barfs_tests.log 2>&1 &&
  for r in 1 2 3; do
    echo "## bar fs" && timeout -k 10 200 python -u tools/replay_probe.py &&
    echo "## pinned fs" && EAO_BAR_FS=0 timeout -k 10 200 python -u tools/replay_probe.py || exit 1
  done > gpurun_out/r5_barfs_probe.log 2>&1
}

# ptail: the pyramid's small levels in one k_pyr_tail launch: ORB parity, stage times against
# EAO_PYR_TAIL=0 (per-level launches), alternating, and the kernels' durations (rocprofv3)
ptail() {
  timeout -k 10 400 python -u -m pytest tests/test_gpu_orb.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_ptail_tests.log 2>&1 &&
  for r in 1 2 3; do
    echo "## tail" && timeout -k 10 200 python -u tools/orb_stages.py &&
    echo "## per-level" && EAO_PYR_TAIL=0 timeout -k 10 200 python -u tools/orb_stages.py || exit 1
  done > gpurun_out/r5_ptail_stages.log 2>&1 &&
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ptail_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/orb_stages.py --reps 2 > $GRAFT_REPO_ROOT/gpurun_out/r5_ptail_prof.log 2>&1)
}

# ipt: k_resize_lds with 1 / 2 / 3 items per thread (smaller workgroups, more of them per CU)
ipt() {
  for r in 1 2; do
    for k in "1 4" "3 4" "4 4" "6 4" "8 4" "4 2" "4 3"; do
      set -- $k
      echo "## ipt $1 segs $2" && EAO_RESIZE_IPT=$1 EAO_RESIZE_SEGS=$2 timeout -k 10 200 python -u tools/orb_stages.py || exit 1
    done
  done > gpurun_out/r5_ipt_stages.log 2>&1 &&
  EAO_RESIZE_IPT=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_orb.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_ipt_tests.log 2>&1
}

# prio: the association kernels at wave priority 3 against the previous build (lib/ab/noprio), the
# bench step alternating, and the replay probe (no frame work beside it)
prio() {
  for r in 1 2 3; do
    echo "## prio" && timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-dropin | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],2), d['step_split_ms'])" &&
    echo "## noprio" && EAO_ACCEL_LIB=eao-slam_amd/lib/ab/noprio/libeao_accel.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-dropin | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],2), d['step_split_ms'])" || exit 1
  done > gpurun_out/r5_prio_bench.log 2>&1 &&
  for r in 1 2; do
    echo "## prio" && timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" &&
    echo "## noprio" && EAO_ACCEL_LIB=eao-slam_amd/lib/ab/noprio/libeao_accel.so timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" || exit 1
  done > gpurun_out/r5_prio_probe.log 2>&1
}

# npearly: the rank path's frame values placed during the first pass: NP / association suites,
# phase stamps (profiling library), replay A/B against the previous build (lib/ab/prev)
npearly() {
  timeout -k 10 500 python -u -m pytest tests/test_gpu_assoc.py tests/test_gpu_fr3.py tests/test_gpu_replay.py tests/test_gpu_chain.py tests/test_gpu_golden.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_npearly_tests.log 2>&1 &&
  EAO_ACCEL_LIB=eao-slam_amd/lib/prof/libeao_accel.so timeout -k 10 200 python -u tools/micro/np_probe.py 175,1162 300,1162 175,2500 > gpurun_out/r5_npearly_phases.log 2>&1 &&
  for r in 1 2 3; do
    echo "## early" && timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" &&
    echo "## prev" && EAO_ACCEL_LIB=eao-slam_amd/lib/ab/prev/libeao_accel.so timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" || exit 1
  done > gpurun_out/r5_npearly_probe.log 2>&1
}

# sort256: the six-wave P = 256 sort in the NP kernels: suites, phase stamps (EAO_NP_SORT256=0 / 1,
# profiling library), replay A/B against the previous build (lib/ab/prev)
sort256() {
  timeout -k 10 500 python -u -m pytest tests/test_gpu_assoc.py tests/test_gpu_fr3.py tests/test_gpu_replay.py tests/test_gpu_chain.py tests/test_gpu_golden.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_sort256_tests.log 2>&1 &&
  for k in 0 1 0 1; do
    echo "## EAO_NP_SORT256=$k" && EAO_NP_SORT256=$k EAO_ACCEL_LIB=eao-slam_amd/lib/prof/libeao_accel.so timeout -k 10 200 python -u tools/micro/np_probe.py 175,1162 300,200 100,240 || exit 1
  done > gpurun_out/r5_sort256_phases.log 2>&1 &&
  for r in 1 2 3; do
    echo "## sort256" && timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" &&
    echo "## prev" && EAO_ACCEL_LIB=eao-slam_amd/lib/ab/prev/libeao_accel.so timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" || exit 1
  done > gpurun_out/r5_sort256_probe.log 2>&1
}

# dppsum (also the prefix scan A/B): the NP kernels' wave sums in DPP / permlane moves: suites, phase stamps, replay A/B
# against the previous build (lib/ab/prev)
dppsum() {
  timeout -k 10 500 python -u -m pytest tests/test_gpu_assoc.py tests/test_gpu_fr3.py tests/test_gpu_replay.py tests/test_gpu_chain.py tests/test_gpu_golden.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_dppsum_tests.log 2>&1 &&
  EAO_ACCEL_LIB=eao-slam_amd/lib/prof/libeao_accel.so timeout -k 10 200 python -u tools/micro/np_probe.py 175,1162 300,1162 > gpurun_out/r5_dppsum_phases.log 2>&1 &&
  for r in 1 2 3; do
    echo "## dppsum" && timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" &&
    echo "## prev" && EAO_ACCEL_LIB=eao-slam_amd/lib/ab/prev/libeao_accel.so timeout -k 10 200 python -u tools/replay_probe.py | grep "pass 2" || exit 1
  done > gpurun_out/r5_dppsum_probe.log 2>&1
}

"$@"
