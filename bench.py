"""bench.py -- frames/s of the EAO-SLAM hot path (ORB extract + motion-model
match + EAO ensemble association) on TUM-fr3-shaped 640x480 streams.

Configs (BASELINE.json):
  --config eao   (default) configs[1] "mono_tum EAO fr3_long_office 640x480, 1xMI355X":
                 the demo list's 405 frames (rgb_seq_pose.txt), association flag EAO.
  --config full  configs[2] "mono_tum Full fr3_long_office": all 2582 frames of
                 rgb_full_demo.txt, flag Full (iForest + line alignment + EAO).
  --config c     configs[3] "Synthetic 640x480 stream, 64 objects x 2k map-points, assoc
                 sharded via RCCL": the object-sharded association.
  --config b     configs[4] "Synthetic 1920x1080 stream, 8-level pyramid, 4000 features/frame":
                 ORB extract + motion match of a 256-frame batch per rank (tools/bench_config_b.py).

One *step* (eao / full) is one pass of the hot path over the whole stream, every input
resident before timing:
  0. the frames arrive as 3-channel colour in HBM: cvtColor RGB2GRAY of every frame
     (mImGray, eao_color_to_gray_batch_device, src/Tracking.cc:349-362);
  1. ORBextractor::operator() of every frame (eao_orb_extract_batch_device,
     src/ORBextractor.cc:1043-1105) -- HBM-resident frames, one batch;
  2. SearchByProjection(CurrentFrame, LastFrame, 15, mono) of every consecutive pair
     (eao_match_motion_batch_device, src/ORBmatcher.cc:1328-1470);
  2b. the EAO Frame ctor's line detection on every colour frame (detect_raw_lines +
     filter_lines with detectImpl's COLOR_BGR2GRAY, eao_lines_detect_color_batch_device,
     src/Frame.cc:324-335) -- the association below consumes the stream's recorded line
     segments, as the replay trace holds them;
  3. the object-association replay of Tracking.cc:1241-1696 + LocalMapping's object
     maintenance (eao_replay_run: frame by frame, NP test / isolation forest / projected
     rects on the GPU, decisions on the host) over the stream's detections.
     It runs on its own host thread + HIP streams, overlapped with 1-2, the way the
     reference's Tracking thread overlaps the next frame's extraction.

Inputs: the association runs on the reference's own fr3_long_office detections
(data/yolo_txts, scores parsed as 0 -- SURVEY Q1) and GT poses (data/groundtruth.txt), as
committed in tests/golden/fr3_inputs.npz; the 3-D object clouds, tracked map points and
line segments are synthesised around them (tools/synth.assoc_stream_fr3_real). The TUM
images are not available: the extraction frames are procedurally rendered 640x480 views
(tools/synth.frame_stream with office-like straight structure in the texture, so the line
detector has edges to find; the Full config cycles 405 of them forth and back).

Multi-GPU: `--gpus N` without a torchrun environment starts N rank processes itself
(before anything touches the GPU). eao / full: every rank replays its own copy of the
stream -- independent camera streams, no data-path collective ("scaling": "weak"), value
= all ranks' frames / max-over-ranks time. c: every rank replays the same stream, object
o's GPU work runs on rank o.id % N and the result records are all-gathered over RCCL
("scaling": "strong").

cpu_baseline: the CPU restatement under oracle/ (kind "port") rebuilt here with
-O3 -march=native, timed on rank 0 on a bounded sample: (a) the reference's shape, one
thread for extraction + matching + association; (b) all cores: extraction and matching
frame-parallel over std::threads, the association (one decision chain) on one thread
beside them. `value` is (b); (a) is reported under "single_thread". The sample's outputs
are checked against the GPU's (parity block).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "eao-slam_amd", "python")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

W, H = 640, 480
NFEAT, NLEV, SCALE = 1000, 8, 1.2
MOTION_TH = 15            # Tracking::TrackWithMotionModel, monocular (th=15)
PEAK_HBM_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E peak
METRIC = "frames/sec (extract+match+EAO-assoc) on 640x480; CPU-ref parity on assoc IDs"
CONFIGS = {
    "eao": dict(flag="EAO", start=None, n=None, cpu_assoc=405,
                workload="mono_tum EAO fr3_long_office 640x480 (BASELINE configs[1]: rgb_seq_pose.txt, 405 frames)"),
    "full": dict(flag="Full", start=0, n=2582, cpu_assoc=2582,
                 workload="mono_tum Full fr3_long_office 640x480 (BASELINE configs[2]: rgb_full_demo.txt, "
                          "2582 frames)"),
}
RENDERED = 405  # procedurally rendered extraction frames per rank (longer streams cycle them)


def launch_ranks(nranks, argv, script=None):
    """--gpus N outside torchrun: start N fresh rank processes of `script` (this file by
    default; nothing in this process has touched the GPU) with the torchrun environment,
    rendezvous on 127.0.0.1, and return the worst exit status; rank 0 prints the JSON line."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(nranks):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nranks),
                   LOCAL_WORLD_SIZE=str(nranks), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


def level_sizes():
    s, out = 1.0, []
    for l in range(NLEV):
        inv = np.float32(1.0) / np.float32(s)
        out.append((int(np.rint(np.float32(W) * inv)), int(np.rint(np.float32(H) * inv))))
        s = float(np.float32(s) * np.float32(SCALE))
    return out


def algorithmic_bytes(n_kps):
    """Per-frame algorithmic bytes of each extraction stage:
    every input byte read once, every output byte written once."""
    lv = [w * h for w, h in level_sizes()]
    l0, upper = lv[0], sum(lv[1:])
    return {
        "pyramid": sum(lv[:-1]) + upper,        # resize: read level l-1, write level l (l = 1..7)
        "fast": l0 + upper,                     # FAST: every level plane read once
        # orient + blur + describe from the raw levels (each read once), 28 B kp + 32 B desc written
        "describe": l0 + upper + n_kps * 60,
        "extract": l0 + 2 * upper + n_kps * 60,     # SURVEY §8d per-frame figure for the whole extraction
    }


STAGES = ["pyramid", "fast", "distribute", "describe"]  # the level blur is fused into k_describe
KERNELS = {"pyramid": "k_resize_lds (x4) + k_pyr_tail", "fast": "k_fast_band", "distribute": "k_distribute",
           "describe": "k_describe"}


PEAK_VALU_LANE_OPS = 78.6e12  # 256 CUs x 4 SIMD-32 x 2.4 GHz x 32 lanes (MI355X_MICROARCH.md)


def _pmc_rows(fname):
    """(kernel base name, counter, corrected value) rows of a committed tools/pmc_summary.py
    table; template arguments and the "void" return type are dropped from the name."""
    p = os.path.join(ROOT, "profiles", fname)
    if not os.path.exists(p):
        return None
    rows = []
    for l in open(p):
        f = l.split()
        if f[:1] == ["void"]:
            f = f[1:]
        if len(f) >= 5 and f[0].startswith("eao::"):
            rows.append((f[0].split("<")[0], f[1], float(f[-1])))
    return rows


def _pmc_value(fname, kernel, counter):
    rows = _pmc_rows(fname)
    for k, c, v in rows or []:
        if k == "eao::" + kernel.split()[0] and c == counter:
            return v
    return None


PMC_FILES = {"fetch": "r05n_pmc_fetch.txt", "write": "r05n_pmc_write.txt", "sq": "r05n_pmc_sq.txt"}


def pmc_valu(kernel, frames):
    """VALU lane-ops per launch of `kernel` from the committed SQ counter pass
    (profiles/r05d_pmc_sq.txt: SQ_INSTS_VALU wave instructions x 64 lanes) over the same
    405-frame launch -- a profiled figure of the same launch shape, not a measurement of
    this run; None for another shape or when the summary is absent."""
    if frames != 405:
        return None
    v = _pmc_value(PMC_FILES["sq"], kernel, "SQ_INSTS_VALU")
    return None if v is None else v * 64


def cu_masked_stream(dev, per_xcd, layout):
    """A HIP stream whose kernels run on `per_xcd` CUs of every XCD (hipExtStreamCreateWithCUMask),
    wrapped for torch; the other CUs stay free for the association's latency-bound launches."""
    import ctypes
    import torch
    hip = ctypes.CDLL("libamdhip64.so")
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    nx = 8
    per = ncu // nx
    bits = [0] * ((ncu + 31) // 32)
    for i in range(ncu):
        xcd, cu = (i % nx, i // nx) if layout == "interleaved" else (i // per, i % per)
        if cu < per_xcd:
            bits[i // 32] |= 1 << (i % 32)
    arr = (ctypes.c_uint32 * len(bits))(*bits)
    h = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(len(bits)), arr)
    if rc != 0:
        raise RuntimeError("hipExtStreamCreateWithCUMask failed: %d" % rc)
    return torch.cuda.ExternalStream(h.value, device=dev)


def pingpong(n, m):
    """Frame index of step t when m rendered frames are cycled forth and back."""
    p = np.arange(n) % (2 * m - 2) if m > 1 else np.zeros(n, np.int64)
    return np.where(p < m, p, 2 * m - 2 - p)


def pmc_traffic(kernel, frames):
    """HBM bytes per launch of `kernel` from committed rocprofv3 --pmc passes (FETCH_SIZE and
    WRITE_SIZE in separate runs of tools/pmc_extract.py over the same 405-frame launch,
    FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950 note). A counter run cannot sit inside
    the timed region, so this is the profiled figure of the same launch shape, NOT a
    measurement of this run; None for another shape or when the summaries are absent."""
    if frames != 405:
        return None, None
    vals = [_pmc_value(PMC_FILES[k], kernel, c) for k, c in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE"))]
    if any(v is None for v in vals):
        return None, None
    src = ", ".join("profiles/" + PMC_FILES[k] for k in ("fetch", "write"))
    return sum(vals), "rocprofv3 --pmc (profiled, committed: %s), same launch shape; not measured in this run" % src


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", choices=["eao", "full", "c", "b"], default="eao")
    ap.add_argument("--frames", type=int, default=0, help="override the stream length")
    ap.add_argument("--unique", type=int, default=64, help="config b: rendered frames (repeated to --frames)")
    ap.add_argument("--cpu-frames", type=int, default=None,
                    help="extract+match single-thread CPU sample (60 frames; 3 at 1080p for config b)")
    ap.add_argument("--cpu-mt-frames", type=int, default=256, help="extract+match all-cores CPU sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--thread", action="store_true",
                    help="A/B: replay the association on a second thread while the frame work is enqueued")
    ap.add_argument("--shard", action="store_true",
                    help="config c: the object-sharded exchange path also at world 1 (one-rank RCCL communicator)")
    ap.add_argument("--poll", action="store_true", help="A/B: poll the extraction stream while the association runs")
    ap.add_argument("--line-batches", type=int, default=1, help="line detection in this many launches per step")
    ap.add_argument("--frame-cus", type=int, default=-1,
                    help="the frame work's stream limited to this many CUs of each XCD (0: all), the rest left to "
                         "the association's launches; default: 24 for the Full stream (its frame work overlaps more "
                         "of the replay: +2 %%, profiles/r06_ab_full_frame_cus.txt), all for the others")
    ap.add_argument("--cu-layout", choices=["interleaved", "linear"], default="interleaved",
                    help="A/B: CU-mask bit order (interleaved: bit i = CU i / 8 of XCD i % 8)")
    ap.add_argument("--no-dropin", action="store_true", help="skip the per-frame drop-in leg (dropin_leg)")
    ap.add_argument("--dropin-frames", type=int, default=405, help="frames of the per-frame drop-in leg")
    ap.add_argument("--chain-frames", type=int, default=120,
                    help="frames of the chained leg (tools/chain.py: the association on the same frames' own "
                         "keypoints and matches); 0 skips it")
    args = ap.parse_args()
    if args.cpu_frames is None:
        args.cpu_frames = 3 if args.config == "b" else 60
    if args.gpus > 1 and "RANK" not in os.environ:
        return launch_ranks(args.gpus, sys.argv[1:])

    import torch  # device memory, streams, torch.distributed: plumbing
    import torch.distributed as dist
    import eao_accel as ea
    import eao_dist

    rank, world, local = eao_dist.env_rank()
    if world != args.gpus:
        raise SystemExit("bench: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    ndev = torch.cuda.device_count()
    if ndev < 1:
        raise RuntimeError("no GPU visible: the engine has no CPU fallback")
    gpu = local % ndev  # ranks beyond the visible devices (a rehearsal on one card) share them
    if args.config == "c":
        return run_config_c(args, rank, world, gpu)
    if args.config == "b":
        # BASELINE configs[4]: synthetic 1920x1080, 8 levels, 4000 features, extract + match t vs t-1;
        # frames are independent units, so N ranks each run a frame shard ("scaling": "weak")
        from tools import bench_config_b
        if not args.frames:
            args.frames = 256
        return bench_config_b.main(args)
    if world > 1:
        backend = os.environ.get("EAO_DIST_BACKEND", "nccl")  # nccl == RCCL on ROCm
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if not ea.device_ok(gpu):
        raise RuntimeError("no gfx950 device: the engine has no CPU fallback")
    from tools import synth
    cfg = CONFIGS[args.config]

    # ---- inputs: the association stream (real fr3 detections + GT poses) and the frames
    assoc_frames = synth.assoc_stream_fr3_real(cfg["start"], cfg["n"])
    if args.frames:
        assoc_frames = assoc_frames[:args.frames]
    F = len(assoc_frames)
    rendered, rposes = synth.frame_stream(min(F, RENDERED), seed=0xEA0 + rank, structure=True)
    idx = pingpong(F, len(rendered))
    poses = rposes[idx].astype(np.float32)
    # the extraction / matching stream runs on a dedicated HIP stream (a NULL handle would
    # select the engine's own stream, which torch events do not see); buffers are made on it
    if args.frame_cus < 0:
        args.frame_cus = 24 if args.config == "full" else 0
    stream = torch.cuda.Stream(dev) if not args.frame_cus else cu_masked_stream(dev, args.frame_cus, args.cu_layout)
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    assert sptr != 0
    d_render = torch.from_numpy(rendered).to(dev)[torch.from_numpy(idx).to(dev)].contiguous()
    # the frames as the reference reads them: 3-channel colour (imread's BGR byte order), a
    # fixed smooth tint per channel over the rendered intensities, resident in HBM. The step
    # converts them twice, as the reference does: cvtColor RGB2GRAY for the tracker's mImGray
    # (Camera.RGB = 1, Tracking.cc:349-362) -> ORB; COLOR_BGR2GRAY inside the line
    # detector's blur (BinaryDescriptor::detectImpl, binary_descriptor.cpp:490-495).
    yy, xx = torch.meshgrid(torch.arange(H, device=dev), torch.arange(W, device=dev), indexing="ij")
    tb = (14 * torch.sin(xx.float() / 37.0)).round().to(torch.int16)
    tr = (11 * torch.cos(yy.float() / 29.0 + xx.float() / 83.0)).round().to(torch.int16)
    g16 = d_render.to(torch.int16)
    d_color = torch.stack([(g16 + tb).clamp(0, 255), g16, (g16 - tr).clamp(0, 255)], -1).to(torch.uint8).contiguous()
    del g16, d_render
    d_frames = torch.empty((F, H, W), dtype=torch.uint8, device=dev)

    orb = ea.Orb(NFEAT, SCALE, NLEV, 20, 7, W, H, max_batch=F, device=gpu)
    cap = orb.cap
    sc = orb.scale_tables()[0]
    cam = ea.camera()
    matcher = ea.Matcher(max_kps=cap, max_batch=F, device=gpu)
    assoc = ea.Assoc(device=gpu)

    u8, i32, f32 = torch.uint8, torch.int32, torch.float32
    d_kps = torch.zeros((F, cap, 28), dtype=u8, device=dev)
    d_desc = torch.zeros((F, cap, 32), dtype=u8, device=dev)
    d_cnt = torch.zeros(F, dtype=i32, device=dev)
    d_T = torch.from_numpy(poses.reshape(F, 16)).to(dev)
    d_has = torch.zeros((F, cap), dtype=u8, device=dev)
    d_mpos = torch.zeros((F, cap, 3), dtype=f32, device=dev)
    d_mdesc = torch.zeros((F, cap, 32), dtype=u8, device=dev)
    d_match = torch.full((F, cap), -1, dtype=i32, device=dev)
    d_nm = torch.zeros(F, dtype=i32, device=dev)
    stream.synchronize()

    lines = ea.Lines(W, H, max_batch=F, device=gpu)
    LCAP = 256
    d_lines = torch.zeros((F, LCAP, 6), dtype=f32, device=dev)
    d_lcnt = torch.zeros(F, dtype=i32, device=dev)

    def gray():  # mImGray of every frame (k_gray, RGB2GRAY code on the BGR bytes)
        ea.color_to_gray_batch_device(d_color.data_ptr(), F, W, H, 3 * W, 3, True, d_frames.data_ptr(), W, gpu, sptr)

    def detect_lines():  # Frame ctor's detect_raw_lines + filter_lines of every frame (Frame.cc:324-335)
        # in --line-batches launches of consecutive frames (each frame's walk holds its CU's LDS
        # for ~5 ms: fewer frames per launch leave CUs to the association's kernels)
        nbat = max(1, min(args.line_batches, F))
        for j in range(nbat):
            f0, f1 = j * F // nbat, (j + 1) * F // nbat
            lines.detect_color_batch_device(d_color.data_ptr() + f0 * H * W * 3, f1 - f0, 3 * W, 3, 50.0,
                                            d_lines.data_ptr() + f0 * LCAP * 6 * 4, d_lcnt.data_ptr() + f0 * 4,
                                            LCAP, sptr)

    def extract():
        orb.extract_batch_device(d_frames.data_ptr(), F, W, d_kps.data_ptr(), d_desc.data_ptr(), d_cnt.data_ptr(),
                                 cap, sptr)

    def match():
        matcher.motion_batch_device(cam, F, cap, d_T.data_ptr(), MOTION_TH, 1, d_kps.data_ptr(),
                                    d_desc.data_ptr(), d_cnt.data_ptr(), d_has.data_ptr(), d_mpos.data_ptr(),
                                    d_mdesc.data_ptr(), sc, d_match.data_ptr(), d_nm.data_ptr(), sptr)

    # -- the map the motion model tracks against: every keypoint of frame t-1 holds a map
    # point on the scene plane (backprojected with the pose, descriptor = its observation's).
    # Built once, untimed: it is map state (an input of SearchByProjection), not an output.
    gray()
    extract()
    torch.cuda.synchronize()
    cnt = d_cnt.cpu().numpy()
    kps = d_kps.cpu().numpy().view(ea.KP_DTYPE).reshape(F, cap)
    mpos = np.zeros((F, cap, 3), np.float32)
    has = np.zeros((F, cap), np.uint8)
    for t in range(F):
        n = int(cnt[t])
        mpos[t, :n] = synth.backproject(poses[t], kps[t, :n]["x"], kps[t, :n]["y"])
        has[t, :n] = 1
    d_mpos.copy_(torch.from_numpy(mpos))
    d_has.copy_(torch.from_numpy(has))
    d_mdesc.copy_(d_desc)

    # the recorded detections / map-point observations of the stream, packed once
    # (host-resident input of the association, like the frames in HBM)
    packed = ea.Replay.pack(assoc_frames)
    last = {"replay": None}

    def associate(out):
        # the previous pass's replay is torn down first, so its forest slots, streams and
        # pinned staging pass to this one (eao_replay_destroy hands them to the engine)
        t0 = time.perf_counter()
        if last["replay"] is not None:
            last["replay"].close()
        rp = ea.Replay(assoc, cfg["flag"])
        last["replay"] = rp
        t1 = time.perf_counter()
        out["det"] = rp.run(packed)  # eao_replay_run: frame-by-frame association + local mapping
        out["replay"] = rp  # object state read back after the timed region
        out["t_setup"], out["t_run"] = t1 - t0, time.perf_counter() - t1

    orb.set_timing(True)
    ev_g0, ev_g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev_m0 = torch.cuda.Event(enable_timing=True)
    ev_m1 = torch.cuda.Event(enable_timing=True)
    ev_l1 = torch.cuda.Event(enable_timing=True)
    ev_done = torch.cuda.Event()

    def front():  # the frame work of the step on the extraction stream
        ev_g0.record(stream)
        gray()
        ev_g1.record(stream)
        extract()
        ev_m0.record(stream)
        match()
        ev_m1.record(stream)
        detect_lines()
        ev_l1.record(stream)

    def step(record):
        out = {}
        th = None
        if not args.thread:
            # the frame work is only enqueued (asynchronous launches on the extraction stream),
            # so it runs on the GPU while this thread replays the association, the critical path
            tf = time.perf_counter()
            front()
            out["t_front"] = time.perf_counter() - tf
            associate(out)
        else:
            # A/B: the association on a second Python thread (it waits for the GIL while the
            # main thread enqueues the frame work: ~4 ms per step, r04_ab_front_enqueue.txt)
            th = threading.Thread(target=associate, args=(out,))
            th.start()
            front()
        # then wait for the extraction stream only (a device-wide synchronize would also
        # serialise against other streams)
        ev_done.record(stream)
        if args.poll:
            while not ev_done.query():
                time.sleep(2e-4)
        if th is not None:
            th.join()
        ev_done.synchronize()
        if record is not None:
            record["split"].append([out.get("t_front", 0.0), out["t_setup"], out["t_run"]])
            record["stage_ms"].append(orb.stage_ms())
            record["match_ms"].append(ev_m0.elapsed_time(ev_m1))
            record["gray_ms"].append(ev_g0.elapsed_time(ev_g1))
            record["lines_ms"].append(ev_m1.elapsed_time(ev_l1))
        return out

    for _ in range(args.warmup):
        step(None)

    rec = {"stage_ms": [], "match_ms": [], "gray_ms": [], "lines_ms": [], "split": []}
    eao_dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step(rec)
    eao_dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = eao_dist.max_over_ranks(time.perf_counter() - t0, dev)

    # frame input stage and per-frame line detection: stages of the step (HIP events on its stream)
    gray_ms = float(np.mean(rec["gray_ms"]))
    gray_bytes = F * W * H * 4  # read 3 B + write 1 B per pixel
    lines_ms = float(np.mean(rec["lines_ms"]))

    total_frames = F * args.steps * world
    ms_per_step = 1000.0 * elapsed / args.steps
    stage = np.mean(np.stack(rec["stage_ms"]), 0)
    match_ms = float(np.mean(rec["match_ms"]))
    searches = search_legs(ea, torch, matcher, cam, stream, F, cap, poses, kps, cnt, mpos, has, sc, d_kps, d_desc,
                           d_cnt, d_has, d_mpos, match_ms)
    hl = d_lcnt.cpu().numpy()
    lines_leg = {"in_step": True, "frames": F, "ms_per_step": lines_ms, "frames_per_s": F / (lines_ms * 1e-3),
                 "mean_lines": float(hl.mean()), "kernels": "k_line_maps<3> (COLOR_BGR2GRAY, blur, Sobel, code, move words, "
                 "anchor masks) + k_line_anchors + k_edge_lines (EdgeDrawing walk + EDline)",
                 "input": "the step's 3-channel colour frames (rawImage of the EAO Frame ctor, Frame.cc:324)"}
    pose = pose_leg(ea, torch, stream, F, cap, gpu, with_cpu=rank == 0 and not args.no_cpu_baseline)
    bow = bow_leg(ea, torch, stream, F, cap, gpu, d_kps, d_desc, d_cnt, kps, cnt,
                  with_cpu=rank == 0 and not args.no_cpu_baseline)
    n_kps = float(d_cnt.float().mean().item())
    ab = algorithmic_bytes(n_kps)
    dom = int(np.argmax(stage))
    dom_name = STAGES[dom]

    result = None
    if rank == 0:
        dom_bytes = ab.get(dom_name)
        if dom_bytes is None:  # distribute: candidates + selections, data dependent -> use the extract figure
            dom_bytes = ab["extract"]
        ach = dom_bytes * F / (stage[dom] * 1e-3) / 1e9
        ext_ms = float(stage.sum())
        traffic, traffic_src = pmc_traffic(KERNELS[dom_name], F)
        nb = np.array([len(f["boxes"]) for f in assoc_frames])
        result = {
            "metric": METRIC,
            "value": total_frames / elapsed,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "reference fr3_long_office inputs: the real YOLO boxes of data/yolo_txts (%d boxes, scores "
                    "parsed as 0 per Tracking.cc:435-466) and GT poses of data/groundtruth.txt for %d frames; "
                    "synthetic 3-D object clouds / tracked map points (%.0f per frame) / line segments around "
                    "them; procedurally rendered 640x480 extraction frames (TUM images absent)"
                    % (int(nb.sum()), F, np.mean([len(f["ids"]) for f in assoc_frames])),
            "config": {"workload": cfg["workload"] + ", %d frames/rank/step, %d ORB features, 8 levels, assoc flag "
                                                     "%s" % (F, NFEAT, cfg["flag"]),
                       "frames_per_step": F, "features": NFEAT, "levels": NLEV, "assoc_flag": cfg["flag"],
                       "parallelism": "streams%d" % world,
                       "frame_work_cus_per_xcd": args.frame_cus or "all"},
            "roofline": {"bound": "hbm", "kernel": KERNELS[dom_name], "achieved": ach, "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": ach / PEAK_HBM_GBS, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": dom_bytes * F, "avg_launch_ms": float(stage[dom])},
            "stages_ms_per_step": {n: float(v) for n, v in zip(STAGES, stage)},
            # the pyramid's own line (HBM-bound: every level read once and written once; its launches
            # are timed together, so no per-launch traffic here -- the per-level PMC passes are in
            # profiles/r05_pmc_fetch.txt / r05_pmc_write.txt)
            "roofline_pyramid": {"bound": "hbm", "kernel": KERNELS["pyramid"],
                                 "achieved": ab["pyramid"] * F / (float(stage[0]) * 1e-3) / 1e9,
                                 "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                 "frac": ab["pyramid"] * F / (float(stage[0]) * 1e-3) / 1e9 / PEAK_HBM_GBS,
                                 "algorithmic_bytes_per_step": ab["pyramid"] * F, "ms_per_step": float(stage[0])},
            # host time of the step's parts (ms): enqueueing the frame work, tearing down the last
            # replay and creating this one, eao_replay_run
            "step_split_ms": dict(zip(("front_enqueue", "replay_setup", "replay_run"),
                                      (float(v) * 1e3 for v in np.mean(np.array(rec["split"]), 0)))),
            "roofline_valu": valu_roof(KERNELS[dom_name], F, float(stage[dom])),
            "extract_ms_per_step": ext_ms,
            "extract_fps": F / (ext_ms * 1e-3),
            "extract_gbs": ab["extract"] * F / (ext_ms * 1e-3) / 1e9,
            "match_ms_per_step": match_ms,
            "searches": searches,
            "line_detect": lines_leg,
            "pose_optimization": pose,
            "bag_of_words": bow,
            "frame_input_stage": {"kernel": "k_gray (cvtColor RGB2GRAY, Tracking.cc:349-362)",
                                  "frames": F, "ms": gray_ms, "achieved_gbs": gray_bytes / (gray_ms * 1e-3) / 1e9,
                                  "frac_hbm_peak": gray_bytes / (gray_ms * 1e-3) / 1e9 / PEAK_HBM_GBS,
                                  "note": "a stage of the step: colour frames in HBM -> mImGray for the extraction"},
            "mean_keypoints": n_kps,
            "mean_matches": float(d_nm[1:].float().mean().item()),
            "assoc_detections": int(nb.sum()),
        }
        prof = np.zeros(24)
        ea.lib().eao_replay_profile(out["replay"].h, ea.P(prof))
        result["assoc_profile_us_per_frame"] = {
            "frame": prof[0] / F, "local_mapping": prof[1] / F, "forest_wait": prof[3] / F,
            "frame_start": prof[14] / F, "assoc_loop": prof[15] / F, "forest_launches_per_frame": prof[2] / F}

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"], result["parity"] = cpu_baseline(args, cfg, assoc_frames, d_frames, poses, kps, cnt,
                                                                mpos, has, sc, d_desc, d_match, d_nm, out,
                                                                d_color, d_lines, d_lcnt)
        result["gpu_over_cpu"] = {"all_cores": result["value"] / result["cpu_baseline"]["value"],
                                  "single_thread": result["value"] / result["cpu_baseline"]["single_thread"]["value"]}
    if rank == 0 and world == 1 and not args.no_dropin:
        # the per-frame legs stand for a process that uses the single-frame entry points only: the
        # step's engines (their streams, HSA queues and buffers) are released first, so the legs do
        # not share the device's hardware queues with idle ones
        for h in (last["replay"], assoc, orb, matcher, lines):
            if h is not None:
                h.close()
        last["replay"] = None
        kd = min(args.dropin_frames, F)
        result["dropin_per_frame"] = dropin_leg(ea, gpu, assoc_frames[:kd], d_color[:kd].cpu().numpy(),
                                                d_frames[:kd].cpu().numpy(), poses[:kd], cfg["flag"],
                                                check=not args.no_cpu_baseline)
    if rank == 0 and world == 1 and not args.no_dropin and args.chain_frames > 0:
        result["chained_per_frame"] = chained_leg(ea, args.chain_frames, check=not args.no_cpu_baseline)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result, default=float), flush=True)
    return 0


def chained_leg(ea, n, check=True):
    """The hot path chained on its own data, one frame at a time (tools/chain.py, as Tracking
    chains it: src/Tracking.cc:1266-1281, 2434-2468): frame t's ORB extraction -> the motion
    search against frame t-1's tracked map points -> the matched keypoints, with the map points
    they carry, into frame t's object association (LocalMapping's object pass at keyframes). The
    batched step above replays recorded fr3 observations; here the association consumes what the
    same frames' extraction and matching produced. Host clock per call; every stage's outputs
    checked against the oracle running the same chain (check)."""
    from tools import chain

    class Timed(chain.EngineBackend):
        def __init__(self):
            super().__init__(ea)
            self.ms = {"extract": [], "match": [], "assoc": []}

        def _t(self, k, f, *a):
            t0 = time.perf_counter()
            r = f(*a)
            self.ms[k].append((time.perf_counter() - t0) * 1e3)
            return r

        def extract(self, g):
            return self._t("extract", super().extract, g)

        def match(self, *a):
            return self._t("match", super().match, *a)

        def replay_frame(self, *a):
            return self._t("assoc", super().replay_frame, *a)

        def local_mapping(self):
            return self._t("assoc", super().local_mapping)

    chain.run(chain.EngineBackend(ea), 3)  # warm every entry point
    be = Timed()
    g = chain.run(be, n)
    call_s = sum(float(np.sum(v)) for v in be.ms.values()) * 1e-3
    res = {"frames": n, "frames_per_s": n / call_s,
           "ms_per_frame": {k: float(np.sum(v)) / n for k, v in be.ms.items()},
           "matches_per_frame": float(np.mean([f["nmatch"] for f in g[1:]])),
           "data": "tools/chain.py: synth's textured plane along synth.camera_path, map points back-projected "
                   "at keyframes, boxes projected from object regions; host buffers, one frame per call; "
                   "frames_per_s over the calls' time (the caller's frame rendering and map bookkeeping "
                   "excluded)"}
    if check:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle as orc  # checker only
        o = chain.run(chain.OracleBackend(orc), n)
        bad = [t for t, (a, b) in enumerate(zip(g, o))
               if not (np.array_equal(a["kps"], b["kps"]) and np.array_equal(a["desc"], b["desc"])
                       and a["nmatch"] == b["nmatch"] and np.array_equal(a["match"], b["match"])
                       and np.array_equal(a["ids"], b["ids"]) and np.array_equal(a["det"], b["det"]))]
        res["parity"] = {"frames_checked": n, "frames_differing": bad[:10], "all_equal": not bad}
    return res


def bow_leg(ea, torch, stream, F, cap, gpu, d_kps, d_desc, d_cnt, kps, cnt, with_cpu=True, reps=3):
    """Bag of words beside the step: Frame::ComputeBoW (DBoW2 transform,
    levelsup 4, Frame.cc:516-523) of the step's F extracted frames and SearchByBoW
    (ORBmatcher.cc:159-288) of every frame against its predecessor as the keyframe (F-1
    searches, 80 % of the keyframe features holding a valid map point), batched and
    HBM-resident, timed with HIP events; the vocabulary is a synthetic ORB-shaped tree (K=10,
    L=6, 1.1M nodes: the reference's ORBvoc blob is missing). The CPU restatement
    (oracle/bow_ref.cpp, one thread) is timed on a sample and checked bit-exact."""
    from tools import synth
    dev = torch.device("cuda", gpu)
    voc = synth.vocabulary(K=10, L=6, seed=0xB0)
    V = ea.Vocab(voc, max_kps=cap, max_batch=F, device=gpu)
    rng = np.random.default_rng(0xB1)
    valid = (rng.random((F, cap)) < 0.8).astype(np.uint8)
    d_valid = torch.from_numpy(valid).to(dev)
    z = lambda *s, dt=torch.int32: torch.zeros(s, dtype=dt, device=dev)
    wid, ww, nw = z(F, cap), z(F, cap, dt=torch.float64), z(F)
    nid, ns, nf, nn = z(F, cap), z(F, cap + 1), z(F, cap), z(F)
    S = F - 1
    match, nm = z(S, cap), z(S)
    sp = stream.cuda_stream
    stream.wait_stream(torch.cuda.current_stream())

    def transform():
        V.transform_batch_device(F, cap, d_cnt.data_ptr(), d_desc.data_ptr(), 4, wid.data_ptr(), ww.data_ptr(),
                                 nw.data_ptr(), nid.data_ptr(), ns.data_ptr(), nf.data_ptr(), nn.data_ptr(), sp)

    i32 = 4
    def search():  # keyframe slot s = frame s, frame slot = frame s + 1 (pointer offsets, no copies)
        kf = (d_kps.data_ptr(), d_desc.data_ptr(), d_valid.data_ptr(), nn.data_ptr(), nid.data_ptr(), ns.data_ptr(),
              nf.data_ptr())
        fr = (d_cnt.data_ptr() + i32, d_kps.data_ptr() + cap * 28, d_desc.data_ptr() + cap * 32,
              nn.data_ptr() + i32, nid.data_ptr() + cap * i32, ns.data_ptr() + (cap + 1) * i32,
              nf.data_ptr() + cap * i32)
        V.search_batch_device(0.75, 1, S, cap, kf, fr, match.data_ptr(), nm.data_ptr(), sp)
    transform()
    search()
    tms, sms = [], []
    for _ in range(reps):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record(stream)
        transform()
        e[1].record(stream)
        search()
        e[2].record(stream)
        e[2].synchronize()
        tms.append(e[0].elapsed_time(e[1]))
        sms.append(e[1].elapsed_time(e[2]))
    h = [x.cpu().numpy() for x in (nid, ns, nf, nn, match, nm)]
    hd = d_desc.cpu().numpy()
    res = {"frames": F, "searches": S, "vocabulary": "synthetic K=10 L=6 (%d nodes)" % len(voc["parent"]),
           "transform_ms_per_batch": float(np.mean(tms)), "search_ms_per_batch": float(np.mean(sms)),
           "transform_frames_per_s": F / (np.mean(tms) * 1e-3), "searches_per_s": S / (np.mean(sms) * 1e-3),
           "mean_matches": float(h[5].mean()), "kernels": "k_bow_words + k_bow_build; k_bow_search + k_bow_rot"}
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle as orc  # checker / CPU baseline only
        orc.use_native()
        OV = orc.Vocab(voc)
        k = 16
        t0 = time.perf_counter()
        fv = [orc.bow_transform(OV, hd[f, :cnt[f]], 4) for f in range(k + 1)]
        t_ms = (time.perf_counter() - t0) * 1e3 / (k + 1)
        t0 = time.perf_counter()
        sr = [orc.search_by_bow(0.75, 1, kps[s, :cnt[s]], hd[s, :cnt[s]], valid[s, :cnt[s]], fv[s][2:],
                                kps[s + 1, :cnt[s + 1]], hd[s + 1, :cnt[s + 1]], fv[s + 1][2:]) for s in range(k)]
        s_ms = (time.perf_counter() - t0) * 1e3 / k
        ok = True
        for f in range(k + 1):
            q = h[3][f]
            ok &= bool(np.array_equal(h[0][f, :q], fv[f][2]) and np.array_equal(h[1][f, :q + 1], fv[f][3]) and
                       np.array_equal(h[2][f, :h[1][f, q]], fv[f][4]))
        for s_ in range(k):
            ok &= bool(h[5][s_] == sr[s_][0] and np.array_equal(h[4][s_, :cnt[s_ + 1]], sr[s_][1]))
        res.update({"cpu_transform_ms_per_frame": t_ms, "cpu_search_ms": s_ms,
                    "cpu_kind": "port (oracle/bow_ref.cpp, 1 thread)", "parity_frames": k + 1,
                    "parity_bitexact": bool(ok),
                    "gpu_over_cpu_transform": (F / (np.mean(tms) * 1e-3)) / (1e3 / t_ms),
                    "gpu_over_cpu_search": (S / (np.mean(sms) * 1e-3)) / (1e3 / s_ms)})
    V.close()
    return res


def pose_leg(ea, torch, stream, F, cap, gpu, with_cpu=True, reps=3, distinct=64):
    """Pose-only optimisation (Optimizer::PoseOptimization, Optimizer.cc:243-457; called per
    frame at Tracking.cc:1106,1699,1741) beside the step: F frames of NFEAT keypoints, 70 %
    holding a map point, 10 % gross outliers, a perturbed motion-model prior
    (tools/synth.pose_problem, `distinct` problems cycled), HBM-resident and batched, timed with
    HIP events; the single-frame host call (the tracker's pattern) timed for its latency; the
    CPU restatement (oracle/pose_ref.cpp, one thread) timed on a sample and checked."""
    from tools import synth
    dev = torch.device("cuda", gpu)
    probs = [synth.pose_problem(2000 + i, NFEAT) for i in range(min(F, distinct))]
    idx = pingpong(F, len(probs))
    T = np.stack([probs[i][0].reshape(16) for i in idx])
    kp = np.zeros((F, cap), dtype=ea.KP_DTYPE)
    has = np.zeros((F, cap), np.uint8)
    pos = np.zeros((F, cap, 3), np.float32)
    for f, i in enumerate(idx):
        kp[f, :NFEAT], has[f, :NFEAT], pos[f, :NFEAT] = probs[i][1], probs[i][2], probs[i][3]
    inv = probs[0][4]
    cnt = torch.full((F,), NFEAT, dtype=torch.int32, device=dev)
    d_T = torch.from_numpy(T).to(dev)
    d_kp = torch.from_numpy(kp.view(np.uint8).reshape(F, cap, 28)).to(dev)
    d_has, d_pos = torch.from_numpy(has).to(dev), torch.from_numpy(pos).to(dev)
    d_To = torch.zeros((F, 16), dtype=torch.float32, device=dev)
    d_out = torch.zeros((F, cap), dtype=torch.uint8, device=dev)
    d_ni = torch.zeros(F, dtype=torch.int32, device=dev)
    P = ea.Pose(max_kps=cap, max_batch=F, device=gpu)
    sp = stream.cuda_stream
    stream.wait_stream(torch.cuda.current_stream())

    def run():
        P.optimize_batch_device(ea.camera(), F, cap, d_T.data_ptr(), cnt.data_ptr(), d_kp.data_ptr(),
                                d_has.data_ptr(), d_pos.data_ptr(), inv, d_To.data_ptr(), d_out.data_ptr(),
                                d_ni.data_ptr(), sp)
    run()
    ms = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        run()
        e1.record(stream)
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    Tp, k1, h1, X1, _, _ = probs[0]
    P.optimize(ea.camera(), Tp, k1, h1, X1, inv)
    t0 = time.perf_counter()
    nlat = 20
    for _ in range(nlat):
        P.optimize(ea.camera(), Tp, k1, h1, X1, inv)
    lat_ms = (time.perf_counter() - t0) * 1e3 / nlat
    To, out, ni = d_To.cpu().numpy(), d_out.cpu().numpy(), d_ni.cpu().numpy()
    res = {"frames": F, "keypoints": NFEAT, "edges_mean": float(has.sum(1).mean()), "ms_per_batch": float(np.mean(ms)),
           "frames_per_s": F / (np.mean(ms) * 1e-3), "single_frame_latency_ms": lat_ms,
           "kernel": "k_pose_opt (one workgroup per frame)",
           "data": "tools/synth.pose_problem (%d problems cycled)" % len(probs)}
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle as orc  # checker / CPU baseline only
        orc.use_native()
        k = min(32, len(probs))
        t0 = time.perf_counter()
        ref = [orc.pose_optimization(orc.cam(), p[0], p[1], p[2], p[3], inv) for p in probs[:k]]
        cpu_ms = (time.perf_counter() - t0) * 1e3 / k
        ok = True
        for f in range(k):
            h = probs[f][2]
            ok &= ref[f][0] == int(ni[f]) and np.array_equal(ref[f][2] * h, out[f, :NFEAT] * h)
            ok &= float(np.abs(ref[f][1] - To[f].reshape(4, 4)).max()) < 1e-5
        res.update({"cpu_ms_per_frame": cpu_ms, "cpu_kind": "port (oracle/pose_ref.cpp, 1 thread)",
                    "gpu_over_cpu": (F / (np.mean(ms) * 1e-3)) / (1e3 / cpu_ms), "parity_frames": k,
                    "parity": bool(ok), "parity_bar": "inliers and outlier flags identical, pose within 1e-5"})
    P.close()
    return res


def dropin_leg(ea, gpu, assoc_frames, color_h, gray_h, poses, flag, check=True):
    """The drop-in as mono_tum drives it: ONE frame at a time through the single-frame C-ABI entry
    points the INTEGRATION.md shims bind, host buffers in and out (PCIe copies included), in the
    reference's per-frame order:
      lines    eao_lines_detect_color(rawImage)  -- the EAO Frame ctor (Frame.cc:324-326)
      extract  eao_orb_extract(mImGray)          -- Frame::ExtractORB (Frame.cc:368-374)
      match    eao_match_motion(Cur, Last)       -- TrackWithMotionModel (Tracking.cc:1266-1273)
      assoc    eao_replay_frame (+ eao_replay_local_mapping at keyframes) -- the object section
               (Tracking.cc:1241-1696, ObjectDataAssociation at :1576; LocalMapping.cc:772-882)
    Pass "sequential" makes the calls one after the other as the reference does; pass
    "overlapped" issues the frame's line detection from a second host thread while the same
    frame's extraction and motion search run (a shim's std::async: the two handles own separate
    HIP streams), joining it before the association. Each call is timed on the host clock. The
    outputs of every frame are checked against the oracle (CPU restatement; thread pool)."""
    from concurrent.futures import ThreadPoolExecutor
    from tools import synth
    F = len(assoc_frames)
    orb1 = ea.Orb(NFEAT, SCALE, NLEV, 20, 7, W, H, max_batch=1, device=gpu)
    sc1 = orb1.scale_tables()[0]
    mt1 = ea.Matcher(max_kps=orb1.cap, max_batch=2, device=gpu)
    ln1 = ea.Lines(W, H, max_batch=1, device=gpu)
    as1 = ea.Assoc(device=gpu)
    cam = ea.camera()
    # warm every entry point once (a throwaway replay: the timed one starts from an empty map)
    ln1.detect_color(color_h[0])
    k0, d0 = orb1.extract(gray_h[0])
    mt1.motion(cam, poses[0], MOTION_TH, 1, k0, np.ones(len(k0), np.uint8),
               synth.backproject(poses[0], k0["x"], k0["y"]), d0, k0, d0, sc1)
    w = ea.Replay(as1, flag)
    f0 = assoc_frames[0]
    w.frame(1, f0["T"], f0["boxes"], f0["ids"], f0["pos"], f0["uv"], f0["bad"], lines=f0.get("lines"))
    w.close()

    def one_pass(overlap, keep):
        rp = ea.Replay(as1, flag)
        st = np.zeros((F, 5))  # lines, extract, match, assoc, frame (ms)
        outs = []
        last = None
        # overlap "thread": the line call on a second host thread; "async": its two halves on this
        # thread (eao_lines_detect_color_start before the extraction, _finish after frame_begin)
        pool = ThreadPoolExecutor(1) if overlap == "thread" else None
        for t in range(F):
            prep = 0.0
            t0 = time.perf_counter()
            if overlap == "thread":
                fut = pool.submit(lambda c: (ln1.detect_color(c), time.perf_counter()), color_h[t])
                t1 = t0
            elif overlap:
                ln1.detect_color_start(color_h[t])
                t1 = time.perf_counter()
            else:
                lines = ln1.detect_color(color_h[t])
                t1 = time.perf_counter()
            kps, desc = orb1.extract(gray_h[t])
            t2 = time.perf_counter()
            nm, cm, t_match = 0, None, 0.0
            if last is not None:
                lk, ld = last
                pos = synth.backproject(poses[t - 1], lk["x"], lk["y"])  # the tracked map: the caller's state
                tp = time.perf_counter()
                prep = tp - t2
                nm, cm = mt1.motion(cam, poses[t], MOTION_TH, 1, lk, np.ones(len(lk), np.uint8), pos, ld, kps, desc,
                                    sc1)
                t_match = time.perf_counter() - tp
            f = assoc_frames[t]
            if overlap:
                # the association runs up to its line-dependent tail while the lines are detected
                # (eao_replay_frame_begin), then takes them (eao_replay_frame_end)
                t3 = time.perf_counter()
                rp.frame_begin(t + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"])
                t3b = time.perf_counter()
                if overlap == "thread":
                    lines, tl = fut.result()
                else:
                    lines = ln1.detect_finish()
                    tl = time.perf_counter()
                t3e = time.perf_counter()
                det = rp.frame_end(lines=f.get("lines"))
                t_assoc = (t3b - t3) + (time.perf_counter() - t3e)
            else:
                t3 = time.perf_counter()
                det = rp.frame(t + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"], lines=f.get("lines"))
                t_assoc = time.perf_counter() - t3
            if f["kf"]:
                t5 = time.perf_counter()
                rp.local_mapping()
                t_assoc += time.perf_counter() - t5
            t4 = time.perf_counter()
            st[t] = [((tl if overlap else t1) - t0) * 1e3, (t2 - t1) * 1e3, t_match * 1e3, t_assoc * 1e3,
                     (t4 - t0 - prep) * 1e3]
            if keep:
                outs.append((lines, kps, desc, nm, cm, det))
            last = (kps, desc)
        if pool:
            pool.shutdown()
        objs = rp.objects() if keep else None
        rp.close()
        return st, outs, objs

    seq, outs, gobjs = one_pass(False, True)
    ovt, outs_t, objs_t = one_pass("thread", True)
    ovl, outs_o, objs_o = one_pass("async", True)

    def same(outs_o, objs_o):
        return (all(np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2]) and
                      a[3] == b[3] and np.array_equal(a[5], b[5]) for a, b in zip(outs, outs_o)) and
                  all(np.array_equal(x, y) for x, y in zip(gobjs[0], objs_o[0])) and
                  np.array_equal(np.nan_to_num(gobjs[1]), np.nan_to_num(objs_o[1])))
    # both overlapped passes (split association calls, lines beside them) give the same outputs
    split_same = same(outs_o, objs_o) and same(outs_t, objs_t)
    for h in (orb1, mt1, ln1):
        h.close()

    def stats(a):
        return {"mean": float(np.nanmean(a)), "p50": float(np.nanmedian(a)), "p90": float(np.nanpercentile(a, 90))}
    res = {"frames": F, "entry_points": "eao_lines_detect_color (overlapped: eao_lines_detect_color_start / eao_lines_detect_finish), eao_orb_extract, eao_match_motion, eao_replay_frame "
                                        "(+ eao_replay_local_mapping), host buffers, one frame per call",
           "sequential": {"frames_per_s": F / (seq[:, 4].sum() * 1e-3),
                          "ms_per_frame": {n: stats(seq[:, k]) for k, n in
                                           enumerate(["lines", "extract", "match", "assoc", "frame"])}},
           "overlapped": {"frames_per_s": F / (ovl[:, 4].sum() * 1e-3),
                          "ms_per_frame": {n: stats(ovl[:, k]) for k, n in
                                           enumerate(["lines", "extract", "match", "assoc", "frame"])},
                          "note": "one host thread: the line detection enqueued first "
                                  "(eao_lines_detect_color_start), extract + match and the association's first "
                                  "call (eao_replay_frame_begin) while it runs, its lines taken "
                                  "(eao_lines_detect_finish) for eao_replay_frame_end; 'lines' is the span from "
                                  "_start to _finish's return, 'assoc' the two calls, 'frame' the frame's wall time",
                          "second_thread_form": {
                              "frames_per_s": F / (ovt[:, 4].sum() * 1e-3),
                              "note": "eao_lines_detect_color on a second host thread instead of the two halves"},
                          "outputs_identical_to_sequential": bool(split_same)}}
    if check:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle as orc  # checker only
        oc = orc.cam()
        sco = orc.orb_params()["scale"]
        threads = max(1, min(16, len(os.sched_getaffinity(0))))
        with ThreadPoolExecutor(threads) as pool:
            ol = list(pool.map(orc.edlines_color, color_h))
            oe = list(pool.map(lambda g: orc.extract(g, NFEAT, SCALE, NLEV), gray_h))
        bad_l = [t for t in range(F) if not np.array_equal(outs[t][0], ol[t])]
        bad_e = [t for t in range(F) if not (np.array_equal(outs[t][1], oe[t][0]) and np.array_equal(outs[t][2], oe[t][1]))]
        bad_m = []
        for t in range(1, F):
            lk, ld = oe[t - 1]
            n, m = orc.match_motion(oc, poses[t], MOTION_TH, 1, lk, np.ones(len(lk), np.uint8),
                                    synth.backproject(poses[t - 1], lk["x"], lk["y"]), ld, oe[t][0], oe[t][1], sco)
            if not (n == outs[t][3] and np.array_equal(m, outs[t][4])):
                bad_m.append(t)
        o = orc.Replay(flag)
        bad_a = []
        for t, f in enumerate(assoc_frames):
            d = o.frame(t + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"], lines=f.get("lines"))
            if not np.array_equal(d, outs[t][5]):
                bad_a.append(t)
            if f["kf"]:
                o.local_mapping()
        oi, of, _ = o.objects()
        gi, gf, _ = gobjs
        ok_obj = bool(np.array_equal(oi, gi) and np.allclose(of, gf, rtol=1e-5, atol=1e-5, equal_nan=True))
        res["parity"] = {"frames_checked": F, "lines_bitexact": not bad_l, "keypoints_descriptors_bitexact": not bad_e,
                         "match_ids_bitexact": not bad_m, "assoc_ids_identical": not bad_a,
                         "object_stats_1e-5": ok_obj,
                         "mismatch_frames": {"lines": bad_l[:5], "extract": bad_e[:5], "match": bad_m[:5],
                                             "assoc": bad_a[:5]}}
    return res


def valu_roof(kernel, frames, ms):
    """The dominant extraction kernel against the VALU issue roofline: lane-ops per launch
    (the committed SQ_INSTS_VALU pass, PMC_FILES["sq"]) over this run's launch time."""
    ops = pmc_valu(kernel, frames)
    if ops is None:
        return None
    ach = ops / (ms * 1e-3)
    return {"bound": "valu", "kernel": kernel, "achieved": ach / 1e12, "peak": PEAK_VALU_LANE_OPS / 1e12,
            "unit": "T lane-ops/s", "frac": ach / PEAK_VALU_LANE_OPS, "lane_ops_per_launch": ops,
            "source": "rocprofv3 --pmc SQ_INSTS_VALU x 64 (profiles/%s), same 405-frame launch" % PMC_FILES["sq"]}


def search_legs(ea, torch, matcher, cam, stream, F, cap, poses, kps, cnt, mpos, has, sc, d_kps, d_desc, d_cnt,
                d_has, d_mpos, motion_ms, reps=5):
    """The single-frame searches beside the step, batched over the stream's F-1 frame
    pairs (search t: frame t's map points / keypoints against frame t+1), HBM-resident,
    each timed with HIP events on the bench stream (ms per batch of F-1 searches):
      local    -- SearchByProjection(Frame&, vector<MapPoint*>, th=1) (TrackLocalMap,
                  ORBmatcher.cc:45-129), map points projected by the next pose;
      keyframe -- SearchByProjection(Frame&, KeyFrame*, sFound, 10, 100) (relocalisation,
                  ORBmatcher.cc:1472-1599), frame t as the candidate keyframe;
      init     -- SearchForInitialization(F1, F2, ..., 100) (ORBmatcher.cc:405-520).
    Parity of these kernels is the -m gpu tests' job (tests/test_gpu_match.py)."""
    dev = d_kps.device
    S = F - 1
    kp_sz = d_kps.shape[2]
    fx, fy, cx, cy = cam.fx, cam.fy, cam.cx, cam.cy
    inv = np.zeros((S, cap), np.uint8)
    proj = np.zeros((S, cap, 2), np.float32)
    lvl = np.zeros((S, cap), np.int32)
    mind = np.zeros((S, cap), np.float32)
    maxd = np.zeros((S, cap), np.float32)
    sc_np = np.asarray(sc, np.float32)
    for t in range(S):
        n = int(cnt[t])
        P = mpos[t, :n].astype(np.float64)
        T = poses[t + 1].astype(np.float64)
        Pc = P @ T[:3, :3].T + T[:3, 3]
        z = np.where(Pc[:, 2] > 0, Pc[:, 2], 1.0)
        u, v = fx * Pc[:, 0] / z + cx, fy * Pc[:, 1] / z + cy
        inv[t, :n] = (Pc[:, 2] > 0) & (u >= 0) & (u <= cam.img_w) & (v >= 0) & (v <= cam.img_h)
        proj[t, :n, 0], proj[t, :n, 1] = u, v
        lvl[t, :n] = kps[t, :n]["octave"]
        Tt = poses[t].astype(np.float64)
        Ow = -Tt[:3, :3].T @ Tt[:3, 3]
        dist = np.linalg.norm(P - Ow[None, :], axis=1)
        maxd[t, :n] = dist * sc_np[kps[t, :n]["octave"]]
        mind[t, :n] = maxd[t, :n] / sc_np[-1]
    up = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d_inv, d_proj, d_lvl = up(inv), up(proj), up(lvl)
    d_vc = torch.ones((S, cap), dtype=torch.float32, device=dev)
    d_mind, d_maxd = up(mind), up(maxd)
    d_T1 = up(poses[1:].reshape(S, 16).astype(np.float32))
    prev0 = torch.zeros((S, cap, 2), dtype=torch.float32, device=dev)
    for t in range(S):
        n = int(cnt[t])
        prev0[t, :n, 0] = torch.from_numpy(kps[t, :n]["x"].astype(np.float32))
        prev0[t, :n, 1] = torch.from_numpy(kps[t, :n]["y"].astype(np.float32))
    d_prev = prev0.clone()
    out = torch.full((S, cap), -1, dtype=torch.int32, device=dev)
    nm = torch.zeros(S, dtype=torch.int32, device=dev)
    q_kps, c_kps = d_kps.data_ptr(), d_kps.data_ptr() + cap * kp_sz
    q_desc, c_desc = d_desc.data_ptr(), d_desc.data_ptr() + cap * 32
    q_n, c_n = d_cnt.data_ptr(), d_cnt.data_ptr() + 4
    sp = stream.cuda_stream
    logsf = float(np.log(np.float32(SCALE)))

    def local():
        matcher.local_batch_device(cam, S, 1.0, 0.8, cap, q_n, d_inv.data_ptr(), d_proj.data_ptr(),
                                   d_lvl.data_ptr(), d_vc.data_ptr(), q_desc, cap, c_n, c_kps, c_desc, None, sc,
                                   out.data_ptr(), nm.data_ptr(), sp)

    def keyframe():
        matcher.keyframe_batch_device(cam, S, d_T1.data_ptr(), 10, 100, 1, cap, q_n, q_kps, d_has.data_ptr(),
                                      d_mpos.data_ptr(), q_desc, d_mind.data_ptr(), d_maxd.data_ptr(), logsf, cap,
                                      c_n, c_kps, c_desc, None, sc, out.data_ptr(), nm.data_ptr(), sp)

    def init():
        matcher.init_batch_device(cam, S, 0.9, 1, cap, q_n, q_kps, q_desc, cap, c_n, c_kps, c_desc,
                                  d_prev.data_ptr(), 100, out.data_ptr(), nm.data_ptr(), sp)

    res = {"searches_per_batch": S, "motion_ms": motion_ms, "motion_us_per_search": motion_ms * 1e3 / S}
    for name, fn in (("local", local), ("keyframe", keyframe), ("init", init)):
        fn()  # warm
        ms = []
        for _ in range(reps):
            if name == "init":
                d_prev.copy_(prev0)  # updated in place (vbPrevMatched), restored outside the timed region
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            e1.synchronize()
            ms.append(e0.elapsed_time(e1))
        res[name + "_ms"] = float(np.mean(ms))
        res[name + "_us_per_search"] = float(np.mean(ms)) * 1e3 / S
        res[name + "_mean_matches"] = float(nm.float().mean().item())
    return res


def cpu_model():
    try:
        for l in open("/proc/cpuinfo"):
            if l.startswith("model name"):
                return l.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args, cfg, assoc_frames, d_frames, poses, kps, cnt, mpos, has, sc, d_desc, d_match, d_nm, gpu_out,
                 d_color, d_lines, d_lcnt):
    """Time the oracle (CPU restatement, -O3 -march=native built here) on a bounded sample
    and check the GPU outputs of the same sample against it."""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as orc  # checker / CPU baseline only
    orc.use_native()
    F = len(assoc_frames)
    nb = np.cumsum([0] + [len(f["boxes"]) for f in assoc_frames])
    det = gpu_out["det"]
    # the job's CPU share: the GPU box grants 16 CPUs per job (OMP_NUM_THREADS / MAX_JOBS = 16) while
    # nproc reports the whole machine, so the all-cores leg runs on min(16, affinity) threads
    threads = max(1, min(16, len(os.sched_getaffinity(0))))

    # (a) the reference's shape: one thread -- per frame cvtColor (mImGray), ORB extraction, the line
    # detector on the colour frame (EAO Frame ctor), the motion search, the association
    k = min(args.cpu_frames, F)
    color_k = d_color[:k].cpu().numpy()
    gpu_gray = d_frames[:k].cpu().numpy()
    desc = d_desc.cpu().numpy()
    match = d_match.cpu().numpy()
    nm = d_nm.cpu().numpy()
    t0 = time.perf_counter()
    frames_k = [orc.color_to_gray(color_k[t], rgb=True) for t in range(k)]
    t_gray = (time.perf_counter() - t0) / k
    bad_gray = [t for t in range(k) if not np.array_equal(frames_k[t], gpu_gray[t])]
    t0 = time.perf_counter()
    olines = [orc.edlines_color(color_k[t]) for t in range(k)]
    t_lines = (time.perf_counter() - t0) / k
    gl, gn = d_lines[:k].cpu().numpy(), d_lcnt[:k].cpu().numpy()
    bad_lines = [t for t in range(k) if not (int(gn[t]) == len(olines[t]) and np.array_equal(gl[t, :gn[t]], olines[t]))]
    t0 = time.perf_counter()
    okps, odesc = [], []
    for t in range(k):
        a, b = orc.extract(frames_k[t], NFEAT, SCALE, NLEV)
        okps.append(a)
        odesc.append(b)
    t_ext = (time.perf_counter() - t0) / k
    bad_kp = [t for t in range(k) if not (int(cnt[t]) == len(okps[t]) and np.array_equal(kps[t, :int(cnt[t])], okps[t])
                                          and np.array_equal(desc[t, :int(cnt[t])], odesc[t]))]
    c = orc.cam()
    t0 = time.perf_counter()
    omatch = []
    for t in range(1, k):
        n0 = len(okps[t - 1])
        omatch.append(orc.match_motion(c, poses[t], MOTION_TH, 1, okps[t - 1], has[t - 1, :n0],
                                       mpos[t - 1, :n0], odesc[t - 1], okps[t], odesc[t], sc))
    t_match = (time.perf_counter() - t0) / max(1, k - 1)
    bad_match = [t for t in range(1, k) if not (omatch[t - 1][0] == int(nm[t])
                                                and np.array_equal(match[t, :int(cnt[t])], omatch[t - 1][1]))]
    ka = min(cfg["cpu_assoc"], F)
    t0 = time.perf_counter()
    rp = orc.Replay(cfg["flag"])
    ok_assoc = True
    for t in range(ka):
        f = assoc_frames[t]
        ids = rp.frame(t + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"], lines=f.get("lines"))
        ok_assoc &= bool(np.array_equal(ids, det[nb[t]:nb[t + 1]]))
        if f["kf"]:
            rp.local_mapping()
    t_assoc = (time.perf_counter() - t0) / ka
    ok_obj = None
    if ka == F:
        oi, of, _ = rp.objects()
        gi, gf, _ = gpu_out["replay"].objects()
        ok_obj = bool(np.array_equal(oi, gi) and np.allclose(of, gf, rtol=1e-5, atol=1e-5, equal_nan=True))

    # (b) all cores: the frame work frame-parallel (cvtColor and the line detector on a thread pool --
    # ctypes releases the GIL --, extraction + matching on std::threads), association on one thread beside
    km = min(args.cpu_mt_frames, F)
    color_m = d_color[:km].cpu().numpy()
    with ThreadPoolExecutor(threads) as pool:
        t0 = time.perf_counter()
        frames_m = np.stack(list(pool.map(lambda c: orc.color_to_gray(c, rgb=True), color_m)))
        t_gray_mt = time.perf_counter() - t0
        t0 = time.perf_counter()
        lines_m = list(pool.map(orc.edlines_color, color_m))
        t_lines_mt = time.perf_counter() - t0
    sec, mk, md, mn, mm, mnm = orc.extract_match_mt(frames_m, poses[:km].reshape(km, 16), has[:km], mpos[:km], sc,
                                                    threads)
    bad_mt = [t for t in range(km) if not (int(mn[t]) == int(cnt[t]) and np.array_equal(mk[t, :mn[t]], kps[t, :mn[t]])
                                           and (t == 0 or np.array_equal(mm[t, :mn[t]], match[t, :mn[t]])))]
    bad_mt += [t for t in range(min(km, k)) if not np.array_equal(lines_m[t], olines[t])]
    t_em_mt = (sec + t_gray_mt + t_lines_mt) / km
    single = 1.0 / (t_gray + t_ext + t_lines + t_match + t_assoc)
    allc = 1.0 / max(t_em_mt, t_assoc)  # pipelined: the association thread is the bound
    base = {"value": allc, "unit": "frames/s", "cores": threads, "kind": "port",
            "cpu": cpu_model(), "nproc": os.cpu_count(),
            "sample": "oracle/ CPU restatement (g++ -O3 -march=native -ffp-contract=off, built on this host): "
                      "cvtColor + line detection + extract + match of %d frames frame-parallel on %d threads (the "
                      "job's CPU share; %.2f ms/frame), association replay (%s flag, one thread) over the first %d "
                      "of %d frames (%.2f ms/frame); frames/s = 1/max of the two (pipelined)"
                      % (km, threads, 1e3 * t_em_mt, cfg["flag"], ka, F, 1e3 * t_assoc),
            "single_thread": {"value": single, "cores": 1,
                              "sample": "one thread: cvtColor %d frames (%.2f ms/frame), extract (%.2f ms/frame), "
                                        "line detection (%.2f ms/frame), motion-match %d pairs (%.2f ms/pair), "
                                        "association %d frames (%.2f ms/frame)"
                                        % (k, 1e3 * t_gray, 1e3 * t_ext, 1e3 * t_lines, k - 1, 1e3 * t_match, ka,
                                           1e3 * t_assoc)}}
    parity = {"frames_checked_extract": k, "gray_bitexact": not bad_gray, "lines_bitexact": not bad_lines,
              "keypoints_descriptors_bitexact": not bad_kp,
              "match_ids_bitexact": not bad_match, "mismatch_frames": (bad_kp[:5], bad_match[:5]),
              "frames_checked_all_cores_leg": km, "all_cores_leg_identical": not bad_mt,
              "all_cores_leg_mismatch_frames": bad_mt[:5],
              "frames_checked_assoc": ka, "assoc_ids_identical": bool(ok_assoc), "object_stats_1e-5": ok_obj}
    return base, parity


def run_config_c(args, rank, world, gpu):
    """BASELINE configs[3] / SURVEY §8d input 4 + §8e: the object-sharded association of a
    synthetic stream, 64 objects x 2000 map points (16 classes), 8 detections per frame
    observing m in [50, 300] points each. Every rank replays the same stream; object o's GPU
    work (NP pairs, projected rect, isolation forest) runs on rank o.id % world and the result
    records are all-gathered over RCCL (eao_replay_shard_rccl), or over a gloo callback with
    EAO_SHARD_EXCHANGE=gloo (a rehearsal of several ranks on one device)."""
    import torch.distributed as dist
    import eao_accel as ea
    import eao_dist
    from tools import synth
    nfr = args.frames or 1000
    exch = os.environ.get("EAO_SHARD_EXCHANGE", "rccl")
    if world > 1:
        dist.init_process_group("gloo")  # control plane only (id broadcast, barrier, timing)
    if not ea.device_ok(gpu):
        raise RuntimeError("no gfx950 device: the engine has no CPU fallback")
    frames = synth.assoc_stream_config_c(nfr)
    packed = ea.Replay.pack(frames)
    assoc = ea.Assoc(device=gpu)

    # --shard: the sharded path at any world size, world 1 included (a one-rank RCCL
    # communicator: every record is written, gathered and read back through the exchange)
    sharded = world > 1 or args.shard

    def make():
        rp = ea.Replay(assoc, "EAO")
        if sharded:
            if exch == "gloo" and world > 1:
                rp.shard(rank, world, allgather=eao_dist.allgather_bytes_gloo())
            else:
                uid = ea.rccl_unique_id() if world == 1 else \
                    eao_dist.broadcast_bytes(ea.rccl_unique_id() if rank == 0 else None)
                rp.shard(rank, world, unique_id=uid)
        return rp

    for _ in range(args.warmup):
        w = make()
        w.run(packed)
        w.close()
    # one replay per timed step, built (communicators included) before its timed run and closed after
    # it, outside the timer: only the K runs are timed, each bracketed by barriers, and only one
    # replay is alive at a time
    det, rp, elapsed = None, None, 0.0
    for k in range(args.steps):
        if rp is not None:
            rp.close()
        rp = make()
        eao_dist.barrier()
        t0 = time.perf_counter()
        det = rp.run(packed)
        eao_dist.barrier()
        elapsed += time.perf_counter() - t0
    elapsed = eao_dist.max_over_ranks(elapsed)
    st = rp.shard_stats() if sharded else {"exchanges": 0, "bytes_per_rank": 0.0, "exchange_us": 0.0}
    prof = np.zeros(24, np.float64)
    ea.lib().eao_replay_profile(rp.h, ea.P(prof))
    result = None
    if rank == 0:
        nb = [len(f["boxes"]) for f in frames]
        result = {
            "metric": "frames/sec (EAO association, Config C: 64 objects x 2k points, sharded by object)",
            "value": nfr * args.steps / elapsed, "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (SURVEY.md §8d input 4: 64 Gaussian object clouds x 2000 points + 5%% outliers, "
                    "16 classes, %.1f boxes and %.0f map points per frame)"
                    % (np.mean(nb), np.mean([len(f["ids"]) for f in frames])),
            "config": {"workload": "Config C association (BASELINE configs[3]), %d frames" % nfr,
                       "parallelism": "objects%d" % world,
                       "timed": "the K replay runs only; each replay's setup (RCCL communicator, forest "
                                "tables) is built before and closed after its run, outside the timer",
                       "exchange": (exch if world > 1 else "rccl") if sharded else None},
            "exchange": {"count": st["exchanges"], "bytes_per_rank_per_exchange":
                         st["bytes_per_rank"] / max(1, st["exchanges"]),
                         "us_per_exchange": st["exchange_us"] / max(1, st["exchanges"]),
                         "exchanges_per_frame": st["exchanges"] / nfr},
            "replay_profile_us_per_frame": {"iforest_wait": prof[3] / nfr, "np": prof[5] / nfr,
                                            "frame_start": prof[7] / nfr},
        }
        if not args.no_cpu_baseline and args.cpu_frames > 0:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import pyoracle as orc  # checker / CPU baseline only
            orc.use_native()
            k = min(max(args.cpu_frames, 200), nfr)
            o = orc.Replay("EAO")
            off = np.cumsum([0] + nb)
            ok = True
            t0 = time.perf_counter()
            for t in range(k):
                f = frames[t]
                ids = o.frame(t + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"])
                ok &= bool(np.array_equal(ids, det[off[t]:off[t + 1]]))
                if f["kf"]:
                    o.local_mapping()
            dt = time.perf_counter() - t0
            result["cpu_baseline"] = {"value": k / dt, "unit": "frames/s", "cores": 1, "kind": "port",
                                      "cpu": cpu_model(),
                                      "sample": "oracle/ CPU restatement (-O3 -march=native, 1 thread: the "
                                                "association is one decision chain), first %d frames" % k}
            result["parity"] = {"frames_checked": k, "assoc_ids_identical": ok}
    rp.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result, default=float), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
