"""GPU ORB matching vs the CPU restatement (bit-exact match indices).

Reference: src/ORBmatcher.cc:45-129 (local map), :405-520 (initialization),
:1328-1470 (motion model), :1472-1599 (relocalisation),
:1647-1663 (Hamming); src/Frame.cc:390-513 (grid,
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


def _kf_scene(frames, a, b, seed):
    """Keyframe a's map points (back-projected keypoints, distance bounds from
    their octave like MapPoint::UpdateNormalAndDepth, MapPoint.cc:340-370)
    searched in frame b."""
    fr, poses = frames
    k0, d0 = orc.extract(fr[a])
    k1, d1 = orc.extract(fr[b])
    rng = np.random.default_rng(seed)
    pos = synth.backproject(poses[a], k0["x"], k0["y"])
    Rwc = poses[a][:3, :3].T
    twc = -Rwc @ poses[a][:3, 3]
    dist = np.linalg.norm(pos - twc[None, :], axis=1).astype(np.float32)
    maxd = (dist * SC[k0["octave"]]).astype(np.float32)
    mind = (maxd / SC[7]).astype(np.float32)
    valid = (rng.random(len(k0)) < 0.85).astype(np.uint8)
    pre = np.full(len(k1), -1, np.int32)
    pre[rng.choice(len(k1), len(k1) // 6, replace=False)] = 7
    return k0, d0, k1, d1, pos, mind, maxd, valid, pre, poses[b]


@pytest.mark.parametrize("th,orbdist,ori", [(10, 100, 1), (3, 64, 1), (10, 100, 0)])
def test_keyframe_exact(frames, th, orbdist, ori):
    """Relocalisation projection search (ORBmatcher.cc:1472-1599), the two
    call shapes of Tracking::Relocalization (Tracking.cc:2295,2309)."""
    k0, d0, k1, d1, pos, mind, maxd, valid, pre, T = _kf_scene(frames, 0, 2, seed=th)
    logsf = float(np.log(np.float32(1.2)))
    ng, mg = ea.Matcher().keyframe(ea.camera(), T, th, orbdist, ori, k0, valid, pos, d0, mind, maxd, logsf,
                                   k1, d1, pre, SC)
    no, mo = orc.match_keyframe(orc.cam(), T, th, orbdist, ori, k0, valid, pos, d0, mind, maxd, logsf,
                                k1, d1, pre, SC)
    assert ng == no and np.array_equal(mg, mo), (ng, no, int((mg != mo).sum()))
    assert no > 30
    assert np.array_equal(mo[pre >= 0], pre[pre >= 0])  # preassigned keypoints are kept


def test_keyframe_empty_and_no_preassigned(frames):
    k0, d0, k1, d1, pos, mind, maxd, valid, pre, T = _kf_scene(frames, 1, 2, seed=4)
    logsf = float(np.log(np.float32(1.2)))
    m = ea.Matcher()
    n, out = m.keyframe(ea.camera(), T, 10, 100, 1, k0[:0], valid[:0], pos[:0], d0[:0], mind[:0], maxd[:0],
                        logsf, k1, d1, None, SC)
    assert n == 0 and (out == -1).all()
    ng, mg = m.keyframe(ea.camera(), T, 10, 100, 1, k0, valid, pos, d0, mind, maxd, logsf, k1, d1, None, SC)
    no, mo = orc.match_keyframe(orc.cam(), T, 10, 100, 1, k0, valid, pos, d0, mind, maxd, logsf, k1, d1, None, SC)
    assert ng == no and np.array_equal(mg, mo)


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


def test_motion_batch_device_exact():
    """Batched HBM-resident extraction + motion matching (the bench path) vs the
    oracle frame by frame: keypoints, descriptors and match ids bit-exact."""
    import torch
    F = 6
    fr, poses = synth.frame_stream(F, seed=0xEA7)
    dev = torch.device("cuda", 0)
    orb = ea.Orb(max_batch=F)
    cap = orb.cap
    d_fr = torch.from_numpy(np.stack(fr)).to(dev)
    kps = torch.zeros((F, cap, 28), dtype=torch.uint8, device=dev)
    desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(F, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(dev)
    orb.extract_batch_device(d_fr.data_ptr(), F, 640, kps.data_ptr(), desc.data_ptr(), cnt.data_ptr(), cap,
                             s.cuda_stream)
    torch.cuda.synchronize()
    n = cnt.cpu().numpy()
    hk = kps.cpu().numpy().view(ea.KP_DTYPE).reshape(F, cap)
    hd = desc.cpu().numpy()
    ok, od = zip(*[orc.extract(f) for f in fr])
    for t in range(F):
        assert n[t] == len(ok[t]) and np.array_equal(hk[t, :n[t]], ok[t]) and np.array_equal(hd[t, :n[t]], od[t])
    rng = np.random.default_rng(5)
    has = np.zeros((F, cap), np.uint8)
    pos = np.zeros((F, cap, 3), np.float32)
    for t in range(F):
        has[t, :n[t]] = rng.random(n[t]) < 0.9
        pos[t, :n[t]] = synth.backproject(poses[t], ok[t]["x"], ok[t]["y"])
    T = torch.from_numpy(np.stack(poses).astype(np.float32).reshape(F, 16)).to(dev)
    d_has = torch.from_numpy(has).to(dev)
    d_pos = torch.from_numpy(pos).to(dev)
    match = torch.full((F, cap), -1, dtype=torch.int32, device=dev)
    nm = torch.zeros(F, dtype=torch.int32, device=dev)
    ea.Matcher(max_kps=cap, max_batch=F).motion_batch_device(
        ea.camera(), F, cap, T.data_ptr(), 15, 1, kps.data_ptr(), desc.data_ptr(), cnt.data_ptr(), d_has.data_ptr(),
        d_pos.data_ptr(), desc.data_ptr(), SC, match.data_ptr(), nm.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    hm, hn = match.cpu().numpy(), nm.cpu().numpy()
    for t in range(1, F):
        no, mo = orc.match_motion(orc.cam(), poses[t], 15, 1, ok[t - 1], has[t - 1, :n[t - 1]],
                                  pos[t - 1, :n[t - 1]], od[t - 1], ok[t], od[t], SC)
        assert hn[t] == no and np.array_equal(hm[t, :n[t]], mo), t
