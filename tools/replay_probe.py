"""Wall-clock breakdown of the association replay on the engine."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "eao-slam_amd", "python"))
import eao_accel as ea  # noqa: E402
from tools import synth  # noqa: E402

frames = synth.assoc_stream_fr3(405) if "dense" not in sys.argv else synth.assoc_stream(405)
a = ea.Assoc()
for rep in range(2):
    rp = ea.Replay(a, "EAO")
    t0 = time.perf_counter()
    for t, f in enumerate(frames):
        rp.frame(t + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"])
        if f["kf"]:
            rp.local_mapping()
    dt = time.perf_counter() - t0
    pr = np.zeros(24)
    ea.lib().eao_replay_profile(rp.h, ea.P(pr))
    print("wall %.1f ms (%.0f us/frame): frame %.0f lm %.0f | iforest %d %.0f | np %d %.0f | rects %d %.0f (us)"
          % (dt * 1e3, dt * 1e6 / len(frames), pr[0], pr[1], pr[2], pr[3], pr[4], pr[5], pr[6], pr[7]))
    rp.close()
