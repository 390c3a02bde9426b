"""Config C (SURVEY.md §8d input 4, §8e): the object-sharded association.

64 objects x 2000 map points (16 classes), 8 detections per frame observing
m in [50, 300] points each, 1000 frames. Every rank replays the same stream;
object o's GPU work (NP pairs, projected rect, isolation forest) runs on rank
o.id % world and the result records are all-gathered over RCCL
(eao_replay_shard_rccl) -- "scaling": "strong" (total work fixed).

  python tools/bench_config_c.py [--frames 1000] [--cpu-frames 60]
  torchrun --nproc-per-node N tools/bench_config_c.py ...   (one rank per GPU)

EAO_SHARD_EXCHANGE=gloo selects the gloo callback exchanger instead (a
rehearsal of several ranks on one device). Rank 0 prints one JSON line; the
CPU restatement (oracle, 1 core) is timed on the first --cpu-frames frames and
its ids are compared with the GPU's on that prefix.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-frames", type=int, default=60)
    args = ap.parse_args()

    rank, world, local = eao_dist.env_rank()
    ndev = torch.cuda.device_count()
    if ndev < 1:
        raise RuntimeError("no GPU visible: the engine has no CPU fallback")
    gpu = local % ndev
    exch = os.environ.get("EAO_SHARD_EXCHANGE", "rccl")
    if world > 1:
        dist.init_process_group("gloo")  # control plane only (id broadcast, barrier, timing)
    if not ea.device_ok(gpu):
        raise RuntimeError("no gfx950 device: the engine has no CPU fallback")

    frames = synth.assoc_stream_config_c(args.frames)
    packed = ea.Replay.pack(frames)
    assoc = ea.Assoc(device=gpu)

    def make():
        rp = ea.Replay(assoc, "EAO")
        if world > 1:
            if exch == "gloo":
                rp.shard(rank, world, allgather=eao_dist.allgather_bytes_gloo())
            else:
                uid = eao_dist.broadcast_bytes(ea.rccl_unique_id() if rank == 0 else None)
                rp.shard(rank, world, unique_id=uid)
        return rp

    for _ in range(args.warmup):
        make().run(packed)
    times, det, st, rp = [], None, None, None
    for _ in range(args.steps):
        rp = make()
        eao_dist.barrier()
        t0 = time.perf_counter()
        det = rp.run(packed)
        eao_dist.barrier()
        times.append(eao_dist.max_over_ranks(time.perf_counter() - t0))
    st = rp.shard_stats() if world > 1 else {"exchanges": 0, "bytes_per_rank": 0.0, "exchange_us": 0.0}
    prof = np.zeros(24, np.float64)
    ea.lib().eao_replay_profile(rp.h, ea.P(prof))
    elapsed = float(np.sum(times))

    result = None
    if rank == 0:
        nb = [len(f["boxes"]) for f in frames]
        result = {
            "metric": "frames/sec (EAO association, Config C: 64 objects x 2k points, sharded by object)",
            "value": args.frames * args.steps / elapsed, "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (SURVEY.md §8d input 4: 64 Gaussian object clouds x 2000 points + 5%% outliers, "
                    "16 classes, %.1f boxes and %.0f map points per frame)"
                    % (np.mean(nb), np.mean([len(f["ids"]) for f in frames])),
            "config": {"workload": "Config C association, %d frames" % args.frames,
                       "parallelism": "objects%d" % world, "exchange": exch if world > 1 else None},
            "exchange": {"count": st["exchanges"], "bytes_per_rank_per_exchange":
                         st["bytes_per_rank"] / max(1, st["exchanges"]),
                         "us_per_exchange": st["exchange_us"] / max(1, st["exchanges"]),
                         "exchanges_per_frame": st["exchanges"] / args.frames},
            "replay_profile_us": {"iforest_wait": prof[3] / args.frames, "np": prof[5] / args.frames,
                                  "frame_start": prof[7] / args.frames},
        }
        if args.cpu_frames > 0:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import pyoracle as orc  # checker / CPU baseline only
            k = min(args.cpu_frames, args.frames)
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
                                      "sample": "oracle/ CPU restatement (1 thread), first %d frames" % k}
            result["parity"] = {"frames_checked": k, "assoc_ids_identical": ok}
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result, default=float), flush=True)


if __name__ == "__main__":
    main()
