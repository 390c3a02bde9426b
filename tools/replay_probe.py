"""Wall-clock breakdown of the association replay on the engine (development aid).

python tools/replay_probe.py [synth] [full]   -- prints eao_replay_profile's counters per pass."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "eao-slam_amd", "python"))
import eao_accel as ea  # noqa: E402
from tools import synth  # noqa: E402

# eao_replay_profile slots (replay.cpp prof[]): times in us, counts marked #
NAMES = {0: "frame", 1: "local_mapping", 2: "#forest_launch", 3: "forest_complete", 4: "#np_launch",
         5: "np_relaunch", 6: "#frame_start", 7: "frame_start_rt", 8: "#frames", 9: "#spec_np", 10: "#lm_forests", 11: "lm_forest",
         12: "steps1-3", 13: "steps4-9", 14: "frame_start_total", 15: "assoc_loop", 16: "same_cls_flush",
         17: "pending_flush", 18: "kick", 19: "launch", 20: "#retire", 21: "retire", 22: "kick_scan",
         23: "pack", 24: "lm_flush", 25: "lm_stats", 26: "lm_merge_overlap", 28: "update", 29: "lm_overlap", 30: "frame_end",
         32: "ms_pass12", 33: "ms_pose", 34: "ms_pass3", 35: "ms_corners", 36: "#ms_pts", 37: "big_to_small", 38: "bts_filter",
         39: "forest_spin", 40: "forest_erase", 41: "fs_spin", 42: "spin_fs", 43: "spin_loop", 44: "spin_end", 45: "spin_lm", 46: "spin_steps1-9", 47: "spin_samecls", 48: "spin_np", 49: "spin_pro", 50: "spin_t", 51: "spin_update", 52: "lookahead", 53: "#lookahead"}

if "full" in sys.argv:  # BASELINE configs[2]: the Full list, real detections
    frames, flag = synth.assoc_stream_fr3_real(0, 2582), "Full"
elif "synth" in sys.argv:  # round-1 synthetic stream
    frames, flag = synth.assoc_stream_fr3(405), "EAO"
else:  # BASELINE configs[1]: the demo list, real detections
    frames, flag = synth.assoc_stream_fr3_real(), "EAO"
packed = ea.Replay.pack(frames)
a = ea.Assoc()
for rep in range(3):
    rp = ea.Replay(a, flag)
    t0 = time.perf_counter()
    rp.run(packed)
    dt = time.perf_counter() - t0
    pr = np.zeros(56)
    ea.lib().eao_replay_profile_n(rp.h, ea.P(pr), 56)
    nf = len(frames)
    print("pass %d: wall %.1f ms (%.0f us/frame)" % (rep, dt * 1e3, dt * 1e6 / nf))
    print("   " + "  ".join("%s=%.0f%s" % (NAMES[k], pr[k] / (1 if NAMES[k][0] == "#" else nf),
                                          "" if NAMES[k][0] == "#" else "us/f") for k in sorted(NAMES)))
    rp.close()
