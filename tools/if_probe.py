"""Phase stamps of the isolation-forest tree kernel on a few cloud sizes."""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "eao-slam_amd", "python"))
import eao_accel as ea  # noqa: E402

a = ea.Assoc()
rng = np.random.default_rng(0)
names = ["seed", "shuffle", "lists", "resolve", "gather", "build", "score"]
for n in (100, 300, 600, 1000, 2000):
    cloud = rng.normal([0, 0, 2], 0.05, (n, 3)).astype(np.float32)
    for _ in range(3):
        a.iforest([cloud])
    t0 = time.perf_counter()
    for _ in range(20):
        a.iforest([cloud])
    dt = (time.perf_counter() - t0) / 20
    st = np.zeros(24, np.uint64)
    ea.lib().eao_debug_iforest_stamps(ea.P(st))
    d = np.diff(st[:8].astype(np.int64))
    print("n=%5d call %.1f us  nodes %d  " % (n, dt * 1e6, st[10]) + " ".join("%s %d" % (k, v) for k, v in zip(names, d)),
          flush=True)
    if st[12:18].any():
        print("   register path (cycles, cumulative over calls): lemire %d minmax %d uniform %d ballot %d push %d leaf/pop %d"
              % tuple(int(v) for v in st[12:18]))
        print("   big-node path cycles %d over %d nodes; register-path steps %d" % tuple(int(v) for v in st[18:21]))
