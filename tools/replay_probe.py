"""Wall-clock breakdown of the association replay on the engine (development aid).

python tools/replay_probe.py [synth] [full]   -- prints eao_replay_profile's counters per pass."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "eao-slam_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import eao_accel as ea  # noqa: E402
from tools import synth  # noqa: E402

# eao_replay_profile slots (replay.cpp prof[]): times in us, counts marked #
from replay_probe_names import NAMES  # noqa: E402

if "full" in sys.argv:  # BASELINE configs[2]: the Full list, real detections
    frames, flag = synth.assoc_stream_fr3_real(0, 2582), "Full"
elif "synth" in sys.argv:  # round-1 synthetic stream
    frames, flag = synth.assoc_stream_fr3(405), "EAO"
else:  # BASELINE configs[1]: the demo list, real detections
    frames, flag = synth.assoc_stream_fr3_real(), "EAO"
packed = ea.Replay.pack(frames)
a = ea.Assoc()
for rep in range(int(os.environ.get("EAO_PROBE_PASSES", "3"))):
    rp = ea.Replay(a, flag)
    t0 = time.perf_counter()
    rp.run(packed)
    dt = time.perf_counter() - t0
    pr = np.zeros(60)
    ea.lib().eao_replay_profile_n(rp.h, ea.P(pr), 60)
    nf = len(frames)
    print("pass %d: wall %.1f ms (%.0f us/frame)" % (rep, dt * 1e3, dt * 1e6 / nf))
    print("   " + "  ".join("%s=%.0f%s" % (NAMES[k], pr[k] / (1 if NAMES[k][0] == "#" else nf),
                                          "" if NAMES[k][0] == "#" else "us/f") for k in sorted(NAMES)))
    rp.close()
