"""Config B (BASELINE.json configs[4], SURVEY.md §8d input 5): ORB extraction
+ motion-model matching on a synthetic 1920x1080 stream, 8 levels, 4000
features per frame.

One step = eao_orb_extract_batch_device over the whole --frames batch (frames
resident in HBM before timing) + eao_match_motion_batch_device over its
consecutive pairs (SearchByProjection(Cur, Last, 15, mono),
src/ORBmatcher.cc:1328-1470), on one HIP stream. Frames are independent units
(SURVEY §8e): under torchrun every rank runs its own stream shard with no
data-path collective ("scaling": "weak"); value = all ranks' frames / the max
over ranks of the timed region.

  python bench.py --config b [--gpus N] [--frames 256] [--steps 5] [--cpu-frames 3]
  python tools/bench_config_b.py [--frames 256] [--steps 5] [--cpu-frames 3]

The stream is --unique rendered frames (a smooth camera path) repeated to
--frames; the pairs across a repeat boundary are pose jumps that match little.
Rank 0 prints one JSON line: frames/s, the per-stage times (HIP events on the
launch stream, measured in a separate pass after the timed region), the
roofline of the dominant extraction kernel against the 8 TB/s HBM peak
(algorithmic bytes of SURVEY §8d Config B), and the oracle (CPU restatement,
1 core) timed on --cpu-frames frames with its keypoints / descriptors / match
ids compared with the GPU's.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "eao-slam_amd", "python")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import eao_accel as ea  # noqa: E402
import eao_dist  # noqa: E402
from tools import synth  # noqa: E402

W, H = 1920, 1080
NFEAT, NLEV, SCALE = 4000, 8, 1.2
MOTION_TH = 15
PEAK_HBM_GBS = 8000.0


def level_sizes():
    s, out = 1.0, []
    for _ in range(NLEV):
        inv = np.float32(1.0) / np.float32(s)
        out.append((int(np.rint(np.float32(W) * inv)), int(np.rint(np.float32(H) * inv))))
        s = float(np.float32(s) * np.float32(SCALE))
    return out


def algorithmic_bytes(n_kps):
    """Per-frame algorithmic bytes of each stage (bench.py's accounting at 1080p)."""
    lv = [w * h for w, h in level_sizes()]
    l0, upper = lv[0], sum(lv[1:])
    return {"pyramid": sum(lv[:-1]) + upper, "fast": l0 + upper,
            "describe": l0 + upper + n_kps * 60, "extract": l0 + 2 * upper + n_kps * 60}


def parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--unique", type=int, default=64, help="rendered frames (repeated to --frames)")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-frames", type=int, default=3)
    return ap


def main(args=None):
    """One Config B measurement; `args` as parser() makes them (bench.py --config b passes its own)."""
    if args is None:
        args = parser().parse_args()
    rank, world, local = eao_dist.env_rank()
    ndev = torch.cuda.device_count()
    if ndev < 1:
        raise RuntimeError("no GPU visible: the engine has no CPU fallback")
    gpu = local % ndev
    if world > 1:
        backend = os.environ.get("EAO_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if not ea.device_ok(gpu):
        raise RuntimeError("no gfx950 device: the engine has no CPU fallback")

    F = args.frames
    U = min(args.unique, F)
    uf, up = synth.frame_stream(U, w=W, h=H, seed=0xEA4 + rank)
    idx = np.arange(F) % U
    frames = uf[idx]
    poses = np.asarray(up, np.float32)[idx]
    d_frames = torch.from_numpy(frames).to(dev)

    orb = ea.Orb(NFEAT, SCALE, NLEV, 20, 7, W, H, max_batch=F, device=gpu)
    cap = orb.cap
    sc = orb.scale_tables()[0]
    cam = ea.camera(W, H)
    matcher = ea.Matcher(max_kps=cap, max_batch=F, device=gpu)
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
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream

    def extract():
        orb.extract_batch_device(d_frames.data_ptr(), F, W, d_kps.data_ptr(), d_desc.data_ptr(), d_cnt.data_ptr(),
                                 cap, sptr)

    def match():
        matcher.motion_batch_device(cam, F, cap, d_T.data_ptr(), MOTION_TH, 1, d_kps.data_ptr(), d_desc.data_ptr(),
                                    d_cnt.data_ptr(), d_has.data_ptr(), d_mpos.data_ptr(), d_mdesc.data_ptr(), sc,
                                    d_match.data_ptr(), d_nm.data_ptr(), sptr)

    # the map the motion model tracks against (an untimed input of the step):
    # frame t-1's keypoints backprojected onto the scene plane with its pose
    extract()
    torch.cuda.synchronize(dev)
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

    ev_m0, ev_m1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def step():
        extract()
        ev_m0.record(stream)
        match()
        ev_m1.record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    eao_dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    eao_dist.barrier()
    elapsed = eao_dist.max_over_ranks(time.perf_counter() - t0, dev)
    # per-stage times in a separate pass (reading them back between steps
    # would put host syncs inside the timed region)
    orb.set_timing(True)
    stages, mms = [], []
    for _ in range(3):
        step()
        stream.synchronize()
        stages.append(orb.stage_ms())
        mms.append(ev_m0.elapsed_time(ev_m1))
    orb.set_timing(False)

    result = None
    if rank == 0:
        names = ["pyramid", "fast", "distribute", "describe"]  # blur fused into k_describe
        stage = np.mean(np.stack(stages), 0)
        n_kps = float(d_cnt.float().mean().item())
        ab = algorithmic_bytes(n_kps)
        dom = int(np.argmax(stage))
        dom_bytes = ab.get(names[dom], ab["extract"])
        ach = dom_bytes * F / (stage[dom] * 1e-3) / 1e9
        ext_ms = float(stage.sum())
        kern = {"pyramid": "k_resize_tile (x7)", "fast": "k_fast_band", "distribute": "k_distribute",
                "describe": "k_describe"}
        result = {
            "metric": "frames/sec (ORB extract+match) on 1920x1080, 4000 features, 8 levels",
            "value": F * args.steps * world / elapsed, "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (procedural textured plane along a smooth camera path, seed 0xEA4; %d rendered "
                    "frames repeated to %d; SURVEY §8d input 5)" % (U, F),
            "config": {"workload": "Config B: synthetic 1920x1080 stream, %d frames/rank/step, 4000 features, "
                                   "8 levels" % F, "frames_per_step": F, "parallelism": "frames%d" % world},
            "roofline": {"bound": "hbm", "kernel": kern[names[dom]], "achieved": ach, "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": ach / PEAK_HBM_GBS, "traffic": None,
                         "algorithmic_bytes_per_launch": dom_bytes * F, "avg_launch_ms": float(stage[dom])},
            "stages_ms_per_step": {n: float(v) for n, v in zip(names, stage)},
            "extract_ms_per_step": ext_ms, "extract_fps": F / (ext_ms * 1e-3),
            "extract_gbs": ab["extract"] * F / (ext_ms * 1e-3) / 1e9,
            "match_ms_per_step": float(np.mean(mms)),
            "mean_keypoints": n_kps, "mean_matches": float(d_nm[1:].float().mean().item()),
        }
        if world == 1 and args.cpu_frames > 0:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import pyoracle as orc  # checker / CPU baseline only
            k = min(args.cpu_frames, U)
            desc = d_desc.cpu().numpy()
            match = d_match.cpu().numpy()
            nm = d_nm.cpu().numpy()
            t0 = time.perf_counter()
            okk, okd = [], []
            for t in range(k):
                a, b = orc.extract(frames[t], NFEAT, SCALE, NLEV)
                okk.append(a)
                okd.append(b)
            t_ext = (time.perf_counter() - t0) / k
            bad_kp = [t for t in range(k) if not (int(cnt[t]) == len(okk[t]) and np.array_equal(
                kps[t, :int(cnt[t])], okk[t]) and np.array_equal(desc[t, :int(cnt[t])], okd[t]))]
            c = orc.cam(W, H)
            t0 = time.perf_counter()
            bad_m = []
            for t in range(1, k):
                n0 = len(okk[t - 1])
                no, mo = orc.match_motion(c, poses[t], MOTION_TH, 1, okk[t - 1], has[t - 1, :n0], mpos[t - 1, :n0],
                                          okd[t - 1], okk[t], okd[t], sc)
                if not (no == int(nm[t]) and np.array_equal(match[t, :int(cnt[t])], mo)):
                    bad_m.append(t)
            t_match = (time.perf_counter() - t0) / max(1, k - 1)
            result["cpu_baseline"] = {"value": 1.0 / (t_ext + t_match), "unit": "frames/s", "cores": 1,
                                      "kind": "port",
                                      "sample": "oracle/ CPU restatement (1 thread): extract %d frames, motion-match "
                                                "%d pairs; per-frame ms extract %.1f match %.2f"
                                                % (k, k - 1, 1e3 * t_ext, 1e3 * t_match)}
            result["parity"] = {"frames_checked": k, "keypoints_descriptors_bitexact": not bad_kp,
                                "match_ids_bitexact": not bad_m, "mismatch_frames": [bad_kp, bad_m]}
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result, default=float), flush=True)


if __name__ == "__main__":
    main()
