"""NoParaDataAssociation: the direct-count path against the sort / rank paths by pair size
(development aid): wall time of one-pair eao_np_test_batch calls at the frame-start pair sizes of the
fr3 stream (the host harness's EAO_HARNESS_DUMP): run once with EAO_NP_DIRECT=0 (never direct)
and once with EAO_NP_DIRECT=100000000 (always direct)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "eao-slam_amd", "python"))
import eao_accel as ea  # noqa: E402

a = ea.Assoc()
rng = np.random.default_rng(0)
tag = os.environ.get("EAO_NP_DIRECT", "default")
for m, n in ((74, 182), (74, 1162), (120, 1162), (175, 1162), (250, 1162), (300, 1162), (463, 1276), (172, 1059),
             (100, 3000), (40, 3000)):
    f = rng.normal(0, 0.1, (m, 3)).astype(np.float32)
    o = rng.normal(0, 0.1, (n, 3)).astype(np.float32)
    fs, os_ = [(f, np.ones(m, np.uint8))], [(o, np.ones(n, np.uint8))]
    for _ in range(5):
        a.np_batch(fs, os_)
    ts = []
    for _ in range(40):
        t0 = time.perf_counter()
        a.np_batch(fs, os_)
        ts.append(time.perf_counter() - t0)
    print("direct_max=%s m=%4d n=%5d m*n=%7d: %.1f us/call (median of 40)" % (tag, m, n, m * n, np.median(ts) * 1e6),
          flush=True)
