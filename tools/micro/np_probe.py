"""NoParaDataAssociation kernel latency by pair size (development aid): wall time of
eao_np_test_batch calls (upload + k_np_pairs + download) for a few (m, n)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "eao-slam_amd", "python"))
import eao_accel as ea  # noqa: E402

a = ea.Assoc()
rng = np.random.default_rng(0)
SIZES = ((30, 100), (60, 300), (120, 500), (200, 1200), (300, 2500), (30, 8000), (100, 5000), (300, 7000),
         (60, 2000))
if len(sys.argv) > 1:  # "m,n m,n ..." (e.g. the fr3 frame-start pairs: 74,1162 175,1162 300,1162)
    SIZES = tuple(tuple(int(x) for x in a.split(",")) for a in sys.argv[1:])
for m, n in SIZES:
    pairs = []
    for _ in range(4):
        f = rng.normal(0, 0.1, (m, 3)).astype(np.float32)
        o = rng.normal(0, 0.1, (n, 3)).astype(np.float32)
        pairs.append(((f, np.ones(m, np.uint8)), (o, np.ones(n, np.uint8))))
    fs, os_ = [p[0] for p in pairs], [p[1] for p in pairs]
    for _ in range(3):
        a.np_batch(fs, os_)
    t0 = time.perf_counter()
    for _ in range(20):
        a.np_batch(fs, os_)
    st = np.zeros(32, np.uint64)
    ea.lib().eao_debug_iforest_stamps(ea.P(st))
    ph = np.diff(st[:6].astype(np.int64))  # EAO_NP_PROF builds (make -C eao-slam_amd prof)
    print("m=%4d n=%5d 4 pairs: %.1f us/call | cycles count %d frame/pad %d sort %d counts %d sums %d"
          % ((m, n, (time.perf_counter() - t0) / 20 * 1e6) + tuple(int(v) for v in ph)), flush=True)
    if int(st[6]) > int(st[3]) and int(st[7]) >= int(st[6]):  # the rank path's searches + atomics, barrier
        print("   rank path: searches+atomics %d, barrier wait %d, fold+prefix+final %d"
              % (int(st[6]) - int(st[3]), int(st[7]) - int(st[6]), int(st[4]) - int(st[7])), flush=True)
