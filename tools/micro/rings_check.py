"""Dense-rings line parity probe (development aid): maps and lines of the engine against the
oracle on concentric rings, repeated (EAO_ACCEL_LIB selects the library)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "eao-slam_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import eao_accel as ea  # noqa: E402
import pyoracle as orc  # noqa: E402


def rings(period):
    yy, xx = np.mgrid[0:480, 0:640]
    return ((np.hypot(xx - 320, yy - 240) // (period / 2)) % 2 * 255).astype(np.uint8)


L = ea.Lines()
for period in (8, 10, 12):
    img = rings(period)
    o = orc.edlines(img)
    ob, odx, ody, og, odr = orc.line_maps(img)
    for rep in range(3):
        g = L.detect(img)
        blur, dx, dy, code = L.debug_maps()
        bad = {"blur": int((blur != ob).sum()), "dx": int((dx != odx).sum()), "dy": int((dy != ody).sum()),
               "grad": int(((code & 0x7fff).astype(np.int16) != og).sum()),
               "dir": int(((code >> 15).astype(np.uint8) * 255 != odr).sum())}
        same = g.shape == o.shape and np.array_equal(g, o)
        print("period %d rep %d: lines %d / oracle %d, equal %s, map mismatches %s" % (period, rep, len(g), len(o), same, bad))
        if bad["blur"]:
            ys, xs = np.nonzero(blur != ob)
            print("   first blur mismatches:", list(zip(ys[:8].tolist(), xs[:8].tolist())),
                  blur[ys[:8], xs[:8]].tolist(), ob[ys[:8], xs[:8]].tolist())
