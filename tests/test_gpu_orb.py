"""GPU ORB extraction vs the CPU restatement (bit-exact keypoints + descriptors).

Reference: src/ORBextractor.cc:1043-1105. The oracle (oracle/orb_ref.cpp) is the
checker; the product runs through the C ABI in eao-slam_amd/lib/libeao_accel.so.
"""
import numpy as np
import pytest

import eao_accel as ea
import pyoracle as orc
from tools import synth

pytestmark = pytest.mark.gpu


def _cmp_kps(g, o):
    assert len(g) == len(o), (len(g), len(o))
    for f in ("x", "y", "size", "angle", "response", "octave", "class_id"):
        a, b = g[f], o[f]
        if not np.array_equal(a, b):
            bad = np.nonzero(a != b)[0]
            raise AssertionError("field %s differs at %d kps, first %d: %r vs %r" % (f, len(bad), bad[0], a[bad[0]], b[bad[0]]))


def test_pyramid_exact(frames):
    fr, _ = frames
    orb = ea.Orb()
    g = orb.pyramid(fr[0])
    o = orc.pyramid(fr[0])
    for l, (a, b) in enumerate(zip(g, o)):
        assert a.shape == b.shape
        assert np.array_equal(a, b), "level %d differs at %d px" % (l, int((a != b).sum()))


def test_scale_tables_and_quotas():
    orb = ea.Orb()
    p = orc.orb_params()
    sc, inv, s2, is2 = orb.scale_tables()
    assert np.array_equal(sc, p["scale"]) and np.array_equal(inv, p["inv_scale"])
    assert np.array_equal(s2, p["sigma2"]) and np.array_equal(is2, p["inv_sigma2"])
    assert list(orb.quotas()) == [217, 181, 151, 126, 105, 87, 73, 60]


@pytest.mark.parametrize("idx", [0, 1, 2, 3])
def test_extract_exact(frames, idx):
    fr, _ = frames
    orb = ea.Orb()
    gk, gd = orb.extract(fr[idx])
    ok, od = orc.extract(fr[idx])
    _cmp_kps(gk, ok)
    assert np.array_equal(gd, od), "descriptor rows differ: %d" % int((gd != od).any(1).sum())


def test_extract_init_extractor(frames):
    fr, _ = frames
    orb = ea.Orb(nfeatures=2000)
    gk, gd = orb.extract(fr[1])
    ok, od = orc.extract(fr[1], nfeatures=2000)
    _cmp_kps(gk, ok)
    assert np.array_equal(gd, od)


def test_extract_flat_and_noise():
    # edge cases: a flat image (no corners -> 0 keypoints) and pure noise (dense corners)
    orb = ea.Orb()
    flat = np.full((480, 640), 128, np.uint8)
    gk, gd = orb.extract(flat)
    ok, od = orc.extract(flat)
    assert len(gk) == len(ok) == 0
    rng = np.random.default_rng(5)
    noise = rng.integers(0, 256, (480, 640), dtype=np.uint8)
    gk, gd = orb.extract(noise)
    ok, od = orc.extract(noise)
    _cmp_kps(gk, ok)
    assert np.array_equal(gd, od)


def test_extract_1080p():
    tex = synth.texture(0xEA4, 4096)
    poses = synth.camera_path(1, 0xEA4)
    img = synth.render(tex, poses[0], 1920, 1080, K=(1600.0, 1600.0, 960.0, 540.0))
    orb = ea.Orb(nfeatures=4000, width=1920, height=1080)
    gk, gd = orb.extract(img)
    ok, od = orc.extract(img, nfeatures=4000)
    _cmp_kps(gk, ok)
    assert np.array_equal(gd, od)
