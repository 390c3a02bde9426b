"""Single-frame extraction and motion search latency (the drop-in's per-frame eao_orb_extract and
eao_match_motion calls, Frame.cc:368-374 / Tracking.cc:1266-1273): host frames in, keypoints /
matches out, one call per frame over the bench's rendered frames; prints the mean / median ms per
call. Run under rocprofv3 --kernel-trace --stats for the per-kernel split. Development aid."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "eao-slam_amd", "python")]
import eao_accel as ea  # noqa: E402
from tools import synth  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 64
fr, poses = synth.frame_stream(F, seed=0xEA0, structure=True)
orb = ea.Orb(1000, 1.2, 8, 20, 7, 640, 480, max_batch=1)
sc = orb.scale_tables()[0]
mt = ea.Matcher(max_kps=orb.cap, max_batch=2)
cam = ea.camera()
k0, d0 = orb.extract(fr[0])
mt.motion(cam, poses[0], 15, 1, k0, np.ones(len(k0), np.uint8), synth.backproject(poses[0], k0["x"], k0["y"]), d0,
          k0, d0, sc)
te, tm, nms = [], [], []
last = None
for t in range(F):
    t0 = time.perf_counter()
    k, d = orb.extract(fr[t])
    te.append((time.perf_counter() - t0) * 1e3)
    if last is not None:
        lk, ld = last
        pos = synth.backproject(poses[t - 1], lk["x"], lk["y"])
        t1 = time.perf_counter()
        nm, _ = mt.motion(cam, poses[t], 15, 1, lk, np.ones(len(lk), np.uint8), pos, ld, k, d, sc)
        tm.append((time.perf_counter() - t1) * 1e3)
        nms.append(nm)
    last = (k, d)
print("single-frame extract: %.3f ms mean, %.3f median | motion search: %.3f ms mean, %.3f median, %.0f matches"
      % (np.mean(te), np.median(te), np.mean(tm), np.median(tm), np.mean(nms)), flush=True)
