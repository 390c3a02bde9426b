"""bench.py -- frames/s of the EAO-SLAM hot path (ORB extract + motion-model
match + EAO ensemble association) on a synthetic TUM-fr3-shaped 640x480 stream.

Workload (BASELINE.json configs[1], SURVEY.md §8d input 2): "mono_tum EAO
fr3_long_office 640x480, 1xMI355X".  One *step* is one pass of the hot path
over the whole 405-frame stream, everything resident in HBM before timing:

  1. ORBextractor::operator() for all 405 frames (eao_orb_extract_batch_device,
     src/ORBextractor.cc:1060-1135)          -- 10 kernel launches,
  2. SearchByProjection(CurrentFrame, LastFrame, 15, mono) for the 404
     consecutive pairs (eao_match_motion_batch_device, src/ORBmatcher.cc:1328)
                                              -- 2 launches,
  3. the object-association replay of Tracking.cc:1199-1530 + LocalMapping
     object maintenance over the 405 frames' YOLO boxes (eao_replay_run: frame
     by frame, NP test / isolation forest / projected rects on the GPU,
     decisions on the host).
     It runs on its own host thread + HIP stream, overlapped with 1-2 the way
     the reference's Tracking thread overlaps the next frame's extraction.

The EAO flag is the full ensemble: IoU / NP / projected IoU / t-test
association, isolation forests, and the object-line association + yaw sampling
(Tracking.cc:2472-2527, 2624-2871) over each frame's synthetic line segments
(projected ground-truth cuboid edges, +-2 deg noise, broken edges, clutter).

Multi-GPU: frames are independent units, so each rank processes
its own 405-frame stream shard with no data-path collective ("scaling":
"weak"); value = all ranks' frames / max-over-ranks time.

cpu_baseline: the CPU restatement under oracle/ (kind "port", 1 core) timed on
rank 0 only on a bounded sample -- extraction + matching on the first
--cpu-frames frames and the association replay over the full stream -- and
the sample's outputs are checked against the GPU's (parity block).
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "eao-slam_amd", "python")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402  (device memory, streams, torch.distributed: plumbing)
import torch.distributed as dist  # noqa: E402

import eao_accel as ea  # noqa: E402
import eao_dist  # noqa: E402
from tools import synth  # noqa: E402

W, H = 640, 480
NFEAT, NLEV, SCALE = 1000, 8, 1.2
MOTION_TH = 15            # Tracking::TrackWithMotionModel, monocular (th=15)
PEAK_HBM_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E peak


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
        # resize: read level l-1, write level l (l = 1..7)
        "pyramid": sum(lv[:-1]) + upper,
        # FAST: every level plane read once
        "fast": l0 + upper,
        # blur: every level read once and its blurred copy written once
        "blur": 2 * (l0 + upper),
        # orient (raw level) + describe (blurred level), outputs 28 B kp + 32 B desc
        "describe": 2 * (l0 + upper) + n_kps * 60,
        # SURVEY §8d per-frame figure for the whole extraction
        "extract": l0 + 2 * upper + n_kps * 60,
    }


def stage_names():
    return ["pyramid", "fast", "distribute", "blur", "describe"]


class Stream:
    """All inputs of one rank's step, resident in HBM."""

    def __init__(self, nframes, seed, dev):
        frames, poses = synth.frame_stream(nframes, seed=seed)
        self.poses = np.stack(poses).astype(np.float32)
        self.host_frames = frames
        self.d_frames = torch.from_numpy(np.stack(frames)).to(dev)
        self.assoc = synth.assoc_stream_fr3(nframes, seed=0xEA1 + (seed - 0xEA0))
        self.n = nframes



def pmc_traffic(kernel, frames):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc passes
    (FETCH_SIZE and WRITE_SIZE in separate runs of tools/pmc_extract.py over the same
    405-frame stream; FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950 note).
    A counter run cannot sit inside the timed region, so this is the profiled figure
    for the same launch shape; None when the summaries are absent or for another size."""
    if frames != 405:
        return None
    tot = 0.0
    for f in ("r01_pmc_fetch_final.txt", "r01_pmc_write_final.txt"):
        p = os.path.join(ROOT, "profiles", f)
        if not os.path.exists(p):
            return None
        hit = [l.split() for l in open(p) if l.split()[:1] == ["eao::" + kernel.split()[0]]]
        if not hit:
            return None
        tot += float(hit[0][-1])
    return tot

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--frames", type=int, default=405)
    ap.add_argument("--cpu-frames", type=int, default=60, help="extract+match CPU sample size")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-overlap", action="store_true", help="run association after extract+match")
    args = ap.parse_args()

    rank, world, local = eao_dist.env_rank()
    # one process per GPU; ranks beyond the visible devices (a rehearsal of
    # several ranks on one card) share devices round-robin
    ndev = torch.cuda.device_count()
    if ndev < 1:
        raise RuntimeError("no GPU visible: the engine has no CPU fallback")
    gpu = local % ndev
    if world > 1:
        backend = os.environ.get("EAO_DIST_BACKEND", "nccl")  # nccl == RCCL on ROCm
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    local = gpu
    if not ea.device_ok(local):
        raise RuntimeError("no gfx950 device: the engine has no CPU fallback")

    F = args.frames
    data = Stream(F, 0xEA0 + rank, dev)

    orb = ea.Orb(NFEAT, SCALE, NLEV, 20, 7, W, H, max_batch=F, device=local)
    cap = orb.cap
    sc = orb.scale_tables()[0]
    cam = ea.camera()
    matcher = ea.Matcher(max_kps=cap, max_batch=F, device=local)
    assoc = ea.Assoc(device=local)

    u8, i32, f32 = torch.uint8, torch.int32, torch.float32
    d_kps = torch.zeros((F, cap, 28), dtype=u8, device=dev)
    d_desc = torch.zeros((F, cap, 32), dtype=u8, device=dev)
    d_cnt = torch.zeros(F, dtype=i32, device=dev)
    d_T = torch.from_numpy(data.poses.reshape(F, 16)).to(dev)
    d_has = torch.zeros((F, cap), dtype=u8, device=dev)
    d_mpos = torch.zeros((F, cap, 3), dtype=f32, device=dev)
    d_mdesc = torch.zeros((F, cap, 32), dtype=u8, device=dev)
    d_match = torch.full((F, cap), -1, dtype=i32, device=dev)
    d_nm = torch.zeros(F, dtype=i32, device=dev)
    # a dedicated stream: the engine launches on it (a NULL handle would
    # select the engine's own stream, which torch events do not see)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    assert sptr != 0

    def extract():
        orb.extract_batch_device(d_frames_ptr, F, W, d_kps.data_ptr(), d_desc.data_ptr(), d_cnt.data_ptr(),
                                 cap, sptr)

    d_frames_ptr = data.d_frames.data_ptr()

    def match():
        matcher.motion_batch_device(cam, F, cap, d_T.data_ptr(), MOTION_TH, 1, d_kps.data_ptr(),
                                    d_desc.data_ptr(), d_cnt.data_ptr(), d_has.data_ptr(), d_mpos.data_ptr(),
                                    d_mdesc.data_ptr(), sc, d_match.data_ptr(), d_nm.data_ptr(), sptr)

    # -- the map the motion model tracks against: every keypoint of frame t-1
    # holds a map point on the scene plane (backprojected with the GT pose,
    # descriptor = its observation's).  Built once, untimed: it is the map
    # state (an input of SearchByProjection), not an output of the step.
    extract()
    torch.cuda.synchronize()
    cnt = d_cnt.cpu().numpy()
    kps = d_kps.cpu().numpy().view(ea.KP_DTYPE).reshape(F, cap)
    mpos = np.zeros((F, cap, 3), np.float32)
    has = np.zeros((F, cap), np.uint8)
    for t in range(F):
        n = int(cnt[t])
        mpos[t, :n] = synth.backproject(data.poses[t], kps[t, :n]["x"], kps[t, :n]["y"])
        has[t, :n] = 1
    d_mpos.copy_(torch.from_numpy(mpos))
    d_has.copy_(torch.from_numpy(has))
    d_mdesc.copy_(d_desc)

    # the recorded detections / map-point observations of the stream, packed
    # once (host-resident input of the association, like the frames in HBM)
    packed = ea.Replay.pack(data.assoc)

    last = {"replay": None}

    def associate(out):
        # the previous pass's replay is torn down first, so its forest slots,
        # streams and pinned staging pass to this one instead of being
        # allocated afresh (eao_replay_destroy hands them to the engine)
        if last["replay"] is not None:
            last["replay"].close()
        rp = ea.Replay(assoc, "EAO")
        last["replay"] = rp
        det = rp.run(packed)  # eao_replay_run: frame-by-frame association + local mapping
        out["det"] = det
        out["replay"] = rp  # object state read back after the timed region

    orb.set_timing(True)
    ev_m0 = torch.cuda.Event(enable_timing=True)
    ev_m1 = torch.cuda.Event(enable_timing=True)
    ev_done = torch.cuda.Event()

    def step(record):
        out = {}
        th = None
        if args.no_overlap:
            extract()
            ev_m0.record(stream)
            match()
            ev_m1.record(stream)
            associate(out)
        else:
            th = threading.Thread(target=associate, args=(out,))
            th.start()
            extract()
            ev_m0.record(stream)
            match()
            ev_m1.record(stream)
        # wait for the extraction stream only (a device-wide synchronize would
        # also serialise against the association thread's launches), politely:
        # the association thread is the critical path and needs its core
        ev_done.record(stream)
        while not ev_done.query():
            time.sleep(2e-4)
        if th is not None:
            th.join()
        if record is not None:
            record["stage_ms"].append(orb.stage_ms())
            record["match_ms"].append(ev_m0.elapsed_time(ev_m1))
        return out

    for _ in range(args.warmup):
        step(None)

    rec = {"stage_ms": [], "match_ms": []}
    eao_dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step(rec)
    eao_dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = eao_dist.max_over_ranks(time.perf_counter() - t0, dev)

    # frame input stage (measured beside the step, not in it):
    # cvtColor(CV_RGB2GRAY) of the same stream as 3-channel frames resident in HBM
    d_color = data.d_frames.unsqueeze(-1).repeat(1, 1, 1, 3)
    d_gray = torch.empty_like(data.d_frames)
    ev_g0, ev_g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ea.color_to_gray_batch_device(d_color.data_ptr(), F, W, H, 3 * W, 3, True, d_gray.data_ptr(), W, local, sptr)
    reps = 10
    ev_g0.record(stream)
    for _ in range(reps):
        ea.color_to_gray_batch_device(d_color.data_ptr(), F, W, H, 3 * W, 3, True, d_gray.data_ptr(), W, local, sptr)
    ev_g1.record(stream)
    torch.cuda.synchronize(dev)
    gray_ms = ev_g0.elapsed_time(ev_g1) / reps
    gray_bytes = F * W * H * 4  # read 3 B + write 1 B per pixel
    del d_color, d_gray

    total_frames = F * args.steps * world
    ms_per_step = 1000.0 * elapsed / args.steps
    stage = np.mean(np.stack(rec["stage_ms"]), 0)
    match_ms = float(np.mean(rec["match_ms"]))
    n_kps = float(d_cnt.float().mean().item())
    ab = algorithmic_bytes(n_kps)
    names = stage_names()
    dom = int(np.argmax(stage))
    dom_name = names[dom]
    kernels = {"pyramid": "k_resize (x7)", "fast": "k_fast_band", "distribute": "k_distribute", "blur": "k_blur",
               "describe": "k_describe"}

    result = None
    if rank == 0:
        dom_bytes = ab.get(dom_name)
        if dom_bytes is None:  # distribute: candidates + selections, data dependent -> use extract figure
            dom_bytes = ab["extract"]
        ach = dom_bytes * F / (stage[dom] * 1e-3) / 1e9
        ext_ms = float(stage.sum())
        ext_gbs = ab["extract"] * F / (ext_ms * 1e-3) / 1e9
        result = {
            "metric": "frames/sec (extract+match+EAO-assoc) on 640x480; CPU-ref parity on assoc IDs",
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
            "data": "synthetic (procedural textured plane along a smooth camera path; seeded object clouds "
                    "observed as ~8 YOLO-shaped boxes and ~800 tracked map points per frame; SURVEY.md §8d input 2)",
            "config": {"workload": "mono_tum EAO fr3_long_office 640x480 (synthetic, %d frames/rank/step, "
                                   "%d ORB features, 8 levels, assoc flag EAO: iForest + object lines + yaw sampling)" % (F, NFEAT),
                       "frames_per_step": F, "features": NFEAT, "levels": NLEV, "parallelism": "frames%d" % world},
            "roofline": {"bound": "hbm", "kernel": kernels[dom_name], "achieved": ach, "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": ach / PEAK_HBM_GBS,
                         "traffic": pmc_traffic(kernels[dom_name], F),
                         "algorithmic_bytes_per_launch": dom_bytes * F,
                         "avg_launch_ms": float(stage[dom])},
            "stages_ms_per_step": {n: float(v) for n, v in zip(names, stage)},
            "extract_ms_per_step": ext_ms,
            "extract_fps": F / (ext_ms * 1e-3),
            "extract_gbs": ext_gbs,
            "match_ms_per_step": match_ms,
            "frame_input_stage": {"kernel": "k_gray (cvtColor RGB2GRAY, Tracking.cc:349-362)",
                                  "ms_per_405_frames": gray_ms, "achieved_gbs": gray_bytes / (gray_ms * 1e-3) / 1e9,
                                  "frac_hbm_peak": gray_bytes / (gray_ms * 1e-3) / 1e9 / PEAK_HBM_GBS,
                                  "note": "measured beside the step (the bench workload is mono frames)"},
            "mean_keypoints": n_kps,
            "mean_matches": float(d_nm[1:].float().mean().item()),
        }

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"], result["parity"] = cpu_baseline(args, data, kps, cnt, mpos, has, sc, d_desc,
                                                                d_match, d_nm, out)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result, default=float), flush=True)


def cpu_baseline(args, data, kps, cnt, mpos, has, sc, d_desc, d_match, d_nm, gpu_out):
    """Time the oracle (CPU restatement, 1 thread) on a bounded sample and
    check the GPU outputs of the same sample against it."""
    nb = np.cumsum([0] + [len(f["boxes"]) for f in data.assoc])
    gpu_ids = [gpu_out["det"][nb[t]:nb[t + 1]] for t in range(data.n)]
    gpu_objects = gpu_out["replay"].objects()
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as orc  # checker / CPU baseline only

    k = min(args.cpu_frames, data.n)
    desc = d_desc.cpu().numpy()
    match = d_match.cpu().numpy()
    nm = d_nm.cpu().numpy()
    t0 = time.perf_counter()
    okps, odesc = [], []
    for t in range(k):
        a, b = orc.extract(data.host_frames[t], NFEAT, SCALE, NLEV)
        okps.append(a)
        odesc.append(b)
    t_ext = (time.perf_counter() - t0) / k
    bad_kp = [t for t in range(k) if not (int(cnt[t]) == len(okps[t]) and np.array_equal(kps[t, :int(cnt[t])], okps[t])
                                          and np.array_equal(desc[t, :int(cnt[t])], odesc[t]))]
    ok_kp = not bad_kp
    c = orc.cam()
    t0 = time.perf_counter()
    omatch = []
    for t in range(1, k):
        n0 = len(okps[t - 1])
        omatch.append(orc.match_motion(c, data.poses[t], MOTION_TH, 1, okps[t - 1], has[t - 1, :n0],
                                       mpos[t - 1, :n0], odesc[t - 1], okps[t], odesc[t], sc))
    t_match = (time.perf_counter() - t0) / max(1, k - 1)
    bad_match = [t for t in range(1, k) if not (omatch[t - 1][0] == int(nm[t])
                                                and np.array_equal(match[t, :int(cnt[t])], omatch[t - 1][1]))]
    ok_match = not bad_match
    t0 = time.perf_counter()
    rp = orc.Replay("EAO")
    ok_assoc = True
    for t, f in enumerate(data.assoc):
        ids = rp.frame(t + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"], lines=f.get("lines"))
        ok_assoc &= np.array_equal(ids, gpu_ids[t])
        if f["kf"]:
            rp.local_mapping()
    t_assoc = (time.perf_counter() - t0) / data.n
    oi, of, _ = rp.objects()
    gi, gf, _ = gpu_objects
    ok_obj = np.array_equal(oi, gi) and np.allclose(of, gf, rtol=1e-5, atol=1e-5, equal_nan=True)
    per_frame = t_ext + t_match + t_assoc
    base = {"value": 1.0 / per_frame, "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": "oracle/ CPU restatement (g++ -O2, 1 thread): extract %d frames, motion-match %d pairs, "
                      "association replay over all %d frames; per-frame ms extract %.2f match %.2f assoc %.2f"
                      % (k, k - 1, data.n, 1e3 * t_ext, 1e3 * t_match, 1e3 * t_assoc)}
    parity = {"frames_checked_extract": k, "keypoints_descriptors_bitexact": bool(ok_kp),
              "match_ids_bitexact": bool(ok_match), "mismatch_frames": (bad_kp[:5], bad_match[:5]), "assoc_ids_identical": bool(ok_assoc),
              "object_stats_1e-5": bool(ok_obj)}
    return base, parity


if __name__ == "__main__":
    main()
