"""Single-frame line detection latency (the drop-in's per-frame call, Frame.cc:324-326): host colour
frame in, lines out, one eao_lines_detect_color call per frame over the bench's rendered frames; prints
the mean / median ms per call and a digest of every frame's lines (A/B across builds or switches).
Run under rocprofv3 --kernel-trace --stats for the per-kernel split. Development aid."""
import hashlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "eao-slam_amd", "python")]
import eao_accel as ea  # noqa: E402
from tools import synth  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 64
W, H = 640, 480
rendered, _ = synth.frame_stream(F, seed=0xEA0, structure=True)
yy, xx = np.mgrid[0:H, 0:W]
tb = np.rint(14 * np.sin(xx / 37.0)).astype(np.int16)
tr = np.rint(11 * np.cos(yy / 29.0 + xx / 83.0)).astype(np.int16)
color = []
for g in rendered:
    g16 = g.astype(np.int16)
    color.append(np.ascontiguousarray(np.stack([np.clip(g16 + tb, 0, 255), g16, np.clip(g16 - tr, 0, 255)], -1)
                                      .astype(np.uint8)))
L = ea.Lines(W, H)
L.detect_color(color[0])
ms, h = [], hashlib.sha256()
for c in color:
    t0 = time.perf_counter()
    out = L.detect_color(c)
    ms.append((time.perf_counter() - t0) * 1e3)
    h.update(out.tobytes())
print("single-frame lines: %.3f ms mean, %.3f median, %.3f min over %d frames, digest %s"
      % (np.mean(ms), np.median(ms), np.min(ms), F, h.hexdigest()[:16]), flush=True)
if "--check" in sys.argv:
    from oracle import pyoracle as orc  # the checker (development aid only)
    bad = [i for i, c in enumerate(color) if not np.array_equal(L.detect_color(c), orc.edlines_color(c))]
    print("oracle check of %d frames: %s" % (len(color), "ok" if not bad else "MISMATCH %s" % bad), flush=True)

L.close()  # EAO_LINES_PROF=1: the merge counters are printed at destroy
