"""GPU ORB matching vs the CPU restatement (bit-exact match indices).

Reference: src/ORBmatcher.cc:45-129 (local map), :405-520 (initialization),
:1328-1470 (motion model), :1647-1663 (Hamming); src/Frame.cc:390-513 (grid,
frustum).
"""
import numpy as np
import pytest

import eao_accel as ea
import pyoracle as orc
from tools import synth

pytestmark = pytest.mark.gpu

SC = orc.orb_params()["scale"]


def _scene(frames, a, b, frac=0.9, seed=1):
    fr, poses = frames
    k0, d0 = orc.extract(fr[a])
    k1, d1 = orc.extract(fr[b])
    rng = np.random.default_rng(seed)
    has = (rng.random(len(k0)) < frac).astype(np.uint8)
    pos = synth.backproject(poses[a], k0["x"], k0["y"])
    return k0, d0, k1, d1, has, pos, poses[b]


@pytest.mark.parametrize("th,ori", [(15, 1), (30, 1), (15, 0)])
def test_motion_exact(frames, th, ori):
    k0, d0, k1, d1, has, pos, T = _scene(frames, 0, 1)
    cam_g, cam_o = ea.camera(), orc.cam()
    m = ea.Matcher()
    ng, mg = m.motion(cam_g, T, th, ori, k0, has, pos, d0, k1, d1, SC)
    no, mo = orc.match_motion(cam_o, T, th, ori, k0, has, pos, d0, k1, d1, SC)
    assert ng == no
    assert np.array_equal(mg, mo), int((mg != mo).sum())
    assert no > 50  # the synthetic stream is trackable


def test_motion_perturbed_descriptors(frames):
    # flip bits so distances tie and exceed TH_HIGH: exercises first-wins ties
    k0, d0, k1, d1, has, pos, T = _scene(frames, 0, 2, seed=3)
    rng = np.random.default_rng(7)
    d0 = d0.copy()
    d0[::3] ^= rng.integers(0, 256, d0[::3].shape, dtype=np.uint8) & 0x11
    m = ea.Matcher()
    ng, mg = m.motion(ea.camera(), T, 15, 1, k0, has, pos, d0, k1, d1, SC)
    no, mo = orc.match_motion(orc.cam(), T, 15, 1, k0, has, pos, d0, k1, d1, SC)
    assert ng == no and np.array_equal(mg, mo)


def test_hamming_pairs():
    rng = np.random.default_rng(11)
    q = rng.integers(0, 256, (300, 32), dtype=np.uint8)
    t = rng.integers(0, 256, (200, 32), dtype=np.uint8)
    qi = rng.integers(0, 300, 1000).astype(np.int32)
    ti = rng.integers(0, 200, 1000).astype(np.int32)
    g = ea.Matcher().hamming(q, t, qi, ti)
    o = np.array([orc.hamming(q[a], t[b]) for a, b in zip(qi, ti)])
    assert np.array_equal(g, o)


def test_frustum_and_local(frames):
    fr, poses = frames
    k0, d0 = orc.extract(fr[0])
    k2, d2 = orc.extract(fr[2])
    pos = synth.backproject(poses[0], k0["x"], k0["y"])
    n = len(pos)
    rng = np.random.default_rng(2)
    normal = np.tile(np.array([0, 0, -1], np.float32), (n, 1))
    Rwc = poses[0][:3, :3].T
    twc = -Rwc @ poses[0][:3, 3]
    dist = np.linalg.norm(pos - twc[None, :], axis=1).astype(np.float32)
    sc = SC[k0["octave"]]
    maxd = (dist * sc).astype(np.float32)
    mind = (maxd / SC[7]).astype(np.float32)
    logsf = float(np.log(np.float32(1.2)))
    m = ea.Matcher()
    cg = m.frustum(ea.camera(), poses[2], pos, normal, mind, maxd, 0.5, logsf)
    co = orc.frustum(orc.cam(), poses[2], pos, normal, mind, maxd, 0.5, logsf)
    assert cg[0] == co[0]
    for a, b in zip(cg[1:], co[1:]):
        inv = co[1].astype(bool)
        assert np.array_equal(np.asarray(a)[inv], np.asarray(b)[inv])
    _, inv, proj, lvl, vc = co
    pre = np.full(len(k2), -1, np.int32)
    pre[rng.choice(len(k2), len(k2) // 5, replace=False)] = 0
    for th in (1.0, 3.0, 5.0):
        ng, mg = m.local(ea.camera(), th, 0.8, inv, proj, lvl, vc, d0, k2, d2, pre, SC)
        no, mo = orc.match_local(orc.cam(), th, 0.8, inv, proj, lvl, vc, d0, k2, d2, pre, SC)
        assert ng == no and np.array_equal(mg, mo), (th, ng, no, int((mg != mo).sum()))


def test_initialization(frames):
    fr, _ = frames
    k1, d1 = orc.extract(fr[0], nfeatures=2000)
    k2, d2 = orc.extract(fr[1], nfeatures=2000)
    prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
    m = ea.Matcher()
    ng, mg, pg = m.init(ea.camera(), 0.9, 1, k1, d1, k2, d2, prev, 100)
    no, mo, po = orc.match_init(orc.cam(), 0.9, 1, k1, d1, k2, d2, prev, 100)
    assert ng == no and np.array_equal(mg, mo) and np.array_equal(pg, po)
    assert no > 100
