"""Host-phase timing of the association replay's orchestration on the CPU (development aid).

The engine's replay.cpp built -O3 -march=native against the host-only HIP stand-in of
tests/native (GPU primitives served synchronously by the oracle), run over the fr3 EAO stream
(or Full with `full`): the eao_replay_profile slots of the host-only phases -- DataAssociateUpdate,
ComputeMeanAndStandard, LocalMapping's merges / overlap / BigToSmall, steps 1-9 -- are the
same code the GPU replay runs on its critical path, without the GPU waits.
  python tools/micro/host_prof.py [full] [passes]"""
import ctypes
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "eao-slam_amd", "python"),
                os.path.join(ROOT, "tools")]
import eao_accel as ea  # noqa: E402
import pyoracle as orc  # noqa: E402
from tools import synth  # noqa: E402
from replay_probe_names import NAMES  # noqa: E402

NATIVE = os.path.join(ROOT, "tests", "native")
orc.lib()
subprocess.check_call(["make", "-s", "-C", NATIVE, "_build/libreplay_host_o3.so"])
H = ctypes.CDLL(os.path.join(NATIVE, "_build", "libreplay_host_o3.so"))
H.harness_assoc_create.restype = ctypes.c_void_p
full = "full" in sys.argv
passes = int(([a for a in sys.argv[1:] if a.isdigit()] or ["2"])[0])
frames, flag = (synth.assoc_stream_fr3_real(0, 2582), "Full") if full else (synth.assoc_stream_fr3_real(), "EAO")
packed = ea.Replay.pack(frames)
HOST = ["#ms_skip", "update", "ms_pass12", "ms_pass3", "ms_pose", "ms_corners", "lm_stats", "lm_merge_overlap", "lm_overlap",
        "big_to_small", "bts_filter", "#bts_scan", "lm_forest", "#lm_forests", "lm_flush", "steps1-3", "steps4-9", "local_mapping", "assoc_loop", "frame"]


class A:
    pass


for rep in range(passes):
    a = A()
    a.h = ctypes.c_void_p(H.harness_assoc_create())
    saved = ea._lib
    ea._lib = H
    try:
        rp = ea.Replay(a, flag)
        t0 = time.perf_counter()
        rp.run(packed)
        dt = time.perf_counter() - t0
        pr = np.zeros(60)
        H.eao_replay_profile_n(rp.h, ea.P(pr), 60)
        H.eao_replay_destroy(rp.h)
        rp.h = ctypes.c_void_p()
    finally:
        ea._lib = saved
    inv = {v: k for k, v in NAMES.items()}
    nf = len(frames)
    print("pass %d: %d frames, wall %.2f s (oracle primitives included)" % (rep, nf, dt))
    print("   " + "  ".join("%s=%.1f" % (n, pr[inv[n]] / nf) for n in HOST) + "  (us/frame)")
