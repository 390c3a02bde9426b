"""The association as the drop-in drives it: one eao_replay_frame (+ eao_replay_local_mapping at
keyframes) call per frame over the fr3 stream, nothing else on the GPU; per-call wall time and the
engine's profile counters (development aid).  python tools/micro/assoc_single.py [gap_us]
gap_us: a host pause between calls (the caller's other work: lines, extraction, matching)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "eao-slam_amd", "python"), os.path.join(ROOT, "tools")]
import eao_accel as ea  # noqa: E402
from tools import synth  # noqa: E402
from replay_probe_names import NAMES  # noqa: E402

gap = float(sys.argv[1]) * 1e-6 if len(sys.argv) > 1 else 0.0
frames = synth.assoc_stream_fr3_real()
a = ea.Assoc()
for rep in range(2):
    rp = ea.Replay(a, "EAO")
    ts = []
    for i, f in enumerate(frames):
        if gap:
            t_end = time.perf_counter() + gap
            while time.perf_counter() < t_end:
                pass
        t0 = time.perf_counter()
        rp.frame(i + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"], lines=f.get("lines"))
        if f["kf"]:
            rp.local_mapping()
        ts.append((time.perf_counter() - t0) * 1e6)
    pr = np.zeros(60)
    ea.lib().eao_replay_profile_n(rp.h, ea.P(pr), 60)
    nf = len(frames)
    ts = np.array(ts)
    print("pass %d (gap %.0f us): per call mean %.0f us, median %.0f, p90 %.0f" % (rep, gap * 1e6, ts.mean(),
                                                                                  np.median(ts), np.percentile(ts, 90)))
    print("   " + "  ".join("%s=%.0f%s" % (NAMES[k], pr[k] / (1 if NAMES[k][0] == "#" else nf),
                                          "" if NAMES[k][0] == "#" else "us/f") for k in sorted(NAMES)))
    rp.close()
