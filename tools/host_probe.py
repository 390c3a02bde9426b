"""Host-side profile of the association orchestration on the CPU harness (tests/native: replay.cpp
with the GPU primitives served by the oracle): the replay's wall-clock counters for the host loops
(update, ComputeMeanAndStandard passes, LocalMapping merge / overlap, BigToSmall), so host work can
be tuned without a device. Development aid. python tools/host_probe.py [full]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "eao-slam_amd", "python")]
import eao_accel as ea  # noqa: E402
import pyoracle as orc  # noqa: E402
import test_replay_host as T  # noqa: E402
from replay_probe_names import NAMES  # noqa: E402
from tools import synth  # noqa: E402

orc.lib()
H = ctypes.CDLL(os.environ.get("EAO_HARNESS_SO") or os.path.join(ROOT, "tests", "native", "_build", "libreplay_host.so"))
H.harness_assoc_create.restype = ctypes.c_void_p
frames, flag = (synth.assoc_stream_fr3_real(0, 2582), "Full") if "full" in sys.argv else (synth.assoc_stream_fr3_real(), "EAO")
packed = ea.Replay.pack(frames)
keys = [28, 32, 33, 34, 35, 36, 25, 26, 29, 37, 38, 13, 12]
for rep in range(3):
    g = T._HostReplay(H, flag)
    g._with(ea.Replay.run, g, packed)
    pr = np.zeros(60)
    H.eao_replay_profile_n(g.h, ea.P(pr), 60)
    nf = len(frames)
    print("pass %d: " % rep + "  ".join("%s=%.1f%s" % (NAMES[k], pr[k] / (1 if NAMES[k][0] == "#" else nf),
                                                      "" if NAMES[k][0] == "#" else "us/f") for k in keys), flush=True)
    g.close()
