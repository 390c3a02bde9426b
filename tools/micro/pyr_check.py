"""Pyramid levels of the engine against the oracle on a few frames / sizes: prints, per level, the
number of differing pixels and the first few (row, col, engine, oracle). Development check for the
resize kernels (EAO_RESIZE=0 selects k_resize_tile)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "eao-slam_amd", "python"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import eao_accel as ea  # noqa: E402
import pyoracle as orc  # noqa: E402
from tools import synth  # noqa: E402


def check(name, img, orb):
    g = orb.pyramid(img)
    o = orc.pyramid(img)
    bad = 0
    for l, (a, b) in enumerate(zip(g, o)):
        d = np.argwhere(a != b)
        if len(d):
            bad += 1
            ex = [(int(r), int(c), int(a[r, c]), int(b[r, c])) for r, c in d[:6]]
            print("%s level %d %s: %d px differ, first %s" % (name, l, a.shape, len(d), ex))
    print("%s: %s" % (name, "ok" if not bad else "%d levels differ" % bad))
    return bad


if __name__ == "__main__":
    fr, _ = synth.frame_stream(3)
    orb = ea.Orb()
    nb = sum(check("synth%d" % i, f, orb) for i, f in enumerate(fr))
    img = np.random.default_rng(5).integers(0, 256, (480, 640), dtype=np.uint8)
    nb += check("rand640", img, orb)
    sys.exit(1 if nb else 0)
