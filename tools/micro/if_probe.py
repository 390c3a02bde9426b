"""Isolation-forest latency probe (development aid): wall time per
eao_iforest_scores_batch call and the in-kernel phase stamps of workgroup
(0,0) for a range of cloud sizes."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "eao-slam_amd", "python"))
import eao_accel as ea  # noqa: E402

a = ea.Assoc()
rng = np.random.default_rng(0)
st = np.zeros(32, np.uint64)
prev = np.zeros(20, np.int64)
names = ["load", "shufdraw", "writers", "resolve", "gather", "build", "score"]
for n in (40, 80, 160, 320, 640, 1280, 2560):
    c = rng.normal([0, 0, 2], [0.1, 0.2, 0.05], (n, 3)).astype(np.float32)
    for _ in range(3):
        a.iforest([c])
    t0 = time.perf_counter()
    R = 20
    for _ in range(R):
        a.iforest([c])
    dt = (time.perf_counter() - t0) / R * 1e6
    ea.lib().eao_debug_iforest_stamps(st.ctypes.data_as(ctypes.c_void_p))
    ph = [int(st[k + 1]) - int(st[k]) for k in range(7)]
    print("n=%5d call %7.1f us | nodes %4d | " % (n, dt, int(st[10])) +
          " ".join("%s %d" % (nm, p) for nm, p in zip(names, ph)), flush=True)
    acc = st[12:32].astype(np.int64) - prev
    prev = st[12:32].astype(np.int64).copy()
    if acc.any():  # EAO_IF_PROF builds: register-path sub-steps, cycles summed over this size's calls
        print("   per register-path step (cycles): lemire %.0f minmax %.0f uniform %.0f ballot %.0f push %.0f "
              "leaf/pop %.0f | big-node path %.0f cycles/node over %d nodes, %d register steps"
              % (tuple(acc[:6] / max(1, acc[8])) + (acc[6] / max(1, acc[7]), acc[7], acc[8])), flush=True)
        print("   rank subtrees: %d calls, %.0f cycles/call, %d nodes, %.0f cycles/node"
              % (acc[10], acc[9] / max(1, acc[10]), acc[11], acc[9] / max(1, acc[11])), flush=True)
        nb_ = max(1, acc[7])
        print("   big nodes (cycles/node): dim %.0f minmax-loop %.0f reduce %.0f split %.0f partition+push %.0f "
              "| mean items %.0f" % (acc[12] / nb_, acc[13] / nb_, acc[14] / nb_, acc[15] / nb_, acc[17] / nb_,
                                     acc[16] / nb_), flush=True)
