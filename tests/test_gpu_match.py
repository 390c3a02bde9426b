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


def test_motion_single_call_full_capacity(frames):
    """A single call packs both frames with a slot stride of their keypoint count rounded up to 64,
    clamped to the matcher's max_kps: a matcher whose max_kps is no multiple of 64, called with
    frames that fill it (the round-up alone would overrun the [2][max_kps] candidate, grid and
    result buffers) and with frames of different sizes, matches the oracle."""
    k0, d0, k1, d1, has, pos, T = _scene(frames, 0, 1)
    n = min(len(k0), len(k1))
    cap = n - 3 if (n - 3) % 64 else n - 4  # no multiple of 64
    for a, b in ((cap, cap), (cap, cap - 100), (cap - 200, cap)):
        m = ea.Matcher(max_kps=cap, max_batch=2)
        ng, mg = m.motion(ea.camera(), T, 15, 1, k0[:a], has[:a], pos[:a], d0[:a], k1[:b], d1[:b], SC)
        no, mo = orc.match_motion(orc.cam(), T, 15, 1, k0[:a], has[:a], pos[:a], d0[:a], k1[:b], d1[:b], SC)
        assert ng == no and np.array_equal(mg, mo), (a, b)


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


@pytest.mark.parametrize("window", [100, 10])
def test_initialization(frames, window):
    """window 100 leaves most queries with more candidates than the stored keys (the
    sequential phase rescans them); window 10 settles nearly all from the stored keys."""
    fr, _ = frames
    k1, d1 = orc.extract(fr[0], nfeatures=2000)
    k2, d2 = orc.extract(fr[1], nfeatures=2000)
    prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
    m = ea.Matcher()
    ng, mg, pg = m.init(ea.camera(), 0.9, 1, k1, d1, k2, d2, prev, window)
    no, mo, po = orc.match_init(orc.cam(), 0.9, 1, k1, d1, k2, d2, prev, window)
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


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")


def _pad(arrs, cap, dtype=None):
    """[n][...] arrays into one [len(arrs)][cap][...] zero-padded slot array."""
    a0 = np.asarray(arrs[0])
    out = np.zeros((len(arrs), cap) + a0.shape[1:], dtype or a0.dtype)
    for f, a in enumerate(arrs):
        out[f, :len(a)] = a
    return out


def test_local_batch_device(frames):
    """eao_match_local_batch_device: 4 searches (map of frame a in frame b) in one
    launch pair, each equal to the oracle's SearchByProjection(local)."""
    import torch
    fr, poses = frames
    logsf = float(np.log(np.float32(1.2)))
    pairs = [(0, 1), (0, 2), (1, 2), (2, 1)]
    rng = np.random.default_rng(9)
    Q, C, exp = [], [], []
    for a, b in pairs:
        k0, d0 = orc.extract(fr[a])
        kb, db = orc.extract(fr[b])
        pos = synth.backproject(poses[a], k0["x"], k0["y"])
        n = len(pos)
        normal = np.tile(np.array([0, 0, -1], np.float32), (n, 1))
        Rwc = poses[a][:3, :3].T
        twc = -Rwc @ poses[a][:3, 3]
        dist = np.linalg.norm(pos - twc[None, :], axis=1).astype(np.float32)
        maxd = (dist * SC[k0["octave"]]).astype(np.float32)
        mind = (maxd / SC[7]).astype(np.float32)
        _, inv, proj, lvl, vc = orc.frustum(orc.cam(), poses[b], pos, normal, mind, maxd, 0.5, logsf)
        pre = np.full(len(kb), -1, np.int32)
        pre[rng.choice(len(kb), len(kb) // 5, replace=False)] = 0
        Q.append((inv, proj, lvl, vc, d0))
        C.append((kb, db, pre))
        exp.append(orc.match_local(orc.cam(), 3.0, 0.8, inv, proj, lvl, vc, d0, kb, db, pre, SC))
    qcap = max(len(q[0]) for q in Q)
    cap = max(len(c[0]) for c in C)
    m = ea.Matcher(max_kps=max(qcap, cap), max_batch=len(pairs))
    t = {k: _dev(_pad([q[i] for q in Q], qcap)) for i, k in enumerate(["inv", "proj", "lvl", "vc", "desc"])}
    kc = _dev(_pad([c[0] for c in C], cap).view(np.uint8))
    dc = _dev(_pad([c[1] for c in C], cap))
    pc = _dev(_pad([c[2] for c in C], cap))
    nq = _dev(np.array([len(q[0]) for q in Q], np.int32))
    nc = _dev(np.array([len(c[0]) for c in C], np.int32))
    out = torch.full((len(pairs), cap), -7, dtype=torch.int32, device="cuda:0")
    nm = torch.zeros(len(pairs), dtype=torch.int32, device="cuda:0")
    m.local_batch_device(ea.camera(), len(pairs), 3.0, 0.8, qcap, nq.data_ptr(), t["inv"].data_ptr(),
                         t["proj"].data_ptr(), t["lvl"].data_ptr(), t["vc"].data_ptr(), t["desc"].data_ptr(), cap,
                         nc.data_ptr(), kc.data_ptr(), dc.data_ptr(), pc.data_ptr(), SC, out.data_ptr(),
                         nm.data_ptr())
    torch.cuda.synchronize()
    ho, hn = out.cpu().numpy(), nm.cpu().numpy()
    for f, (no, mo) in enumerate(exp):
        assert hn[f] == no and np.array_equal(ho[f, :len(mo)], mo), (f, hn[f], no)


def test_keyframe_batch_device(frames):
    import torch
    pairs = [(0, 2, 10, 100, 1), (1, 2, 10, 100, 1)]  # th / ORBdist are per call: one batch shares them
    logsf = float(np.log(np.float32(1.2)))
    S, exp = [], []
    for a, b, th, od, ori in pairs:
        k0, d0, k1, d1, pos, mind, maxd, valid, pre, T = _kf_scene(frames, a, b, seed=a + b)
        S.append((k0, d0, k1, d1, pos, mind, maxd, valid, pre, T))
        exp.append(orc.match_keyframe(orc.cam(), T, th, od, ori, k0, valid, pos, d0, mind, maxd, logsf, k1, d1, pre,
                                      SC))
    qcap = max(len(s[0]) for s in S)
    cap = max(len(s[2]) for s in S)
    m = ea.Matcher(max_kps=max(qcap, cap), max_batch=2)
    sub = S
    kk = _dev(_pad([s[0] for s in sub], qcap).view(np.uint8))
    kd = _dev(_pad([s[1] for s in sub], qcap))
    ck = _dev(_pad([s[2] for s in sub], cap).view(np.uint8))
    cdsc = _dev(_pad([s[3] for s in sub], cap))
    pos = _dev(_pad([s[4] for s in sub], qcap))
    mind = _dev(_pad([s[5] for s in sub], qcap))
    maxd = _dev(_pad([s[6] for s in sub], qcap))
    val = _dev(_pad([s[7] for s in sub], qcap))
    pre = _dev(_pad([s[8] for s in sub], cap))
    T = _dev(np.stack([s[9] for s in sub]).astype(np.float32))
    nq = _dev(np.array([len(s[0]) for s in sub], np.int32))
    nc = _dev(np.array([len(s[2]) for s in sub], np.int32))
    out = torch.full((2, cap), -7, dtype=torch.int32, device="cuda:0")
    nm = torch.zeros(2, dtype=torch.int32, device="cuda:0")
    m.keyframe_batch_device(ea.camera(), 2, T.data_ptr(), 10, 100, 1, qcap, nq.data_ptr(), kk.data_ptr(),
                            val.data_ptr(), pos.data_ptr(), kd.data_ptr(), mind.data_ptr(), maxd.data_ptr(), logsf,
                            cap, nc.data_ptr(), ck.data_ptr(), cdsc.data_ptr(), pre.data_ptr(), SC, out.data_ptr(),
                            nm.data_ptr())
    torch.cuda.synchronize()
    ho, hn = out.cpu().numpy(), nm.cpu().numpy()
    for f in range(2):
        no, mo = exp[f]
        assert hn[f] == no and np.array_equal(ho[f, :len(mo)], mo), (f, hn[f], no)


@pytest.mark.parametrize("window", [100, 20])
def test_init_batch_device(frames, window):
    import torch
    fr, _ = frames
    pairs = [(0, 1), (1, 2), (0, 2)]
    ex = {i: orc.extract(fr[i], nfeatures=2000) for i in range(3)}
    exp = []
    for a, b in pairs:
        k1, d1 = ex[a]
        k2, d2 = ex[b]
        prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
        exp.append(orc.match_init(orc.cam(), 0.9, 1, k1, d1, k2, d2, prev, window))
    cap1 = max(len(ex[a][0]) for a, _ in pairs)
    cap2 = max(len(ex[b][0]) for _, b in pairs)
    m = ea.Matcher(max_kps=max(cap1, cap2), max_batch=len(pairs))
    k1 = _dev(_pad([ex[a][0] for a, _ in pairs], cap1).view(np.uint8))
    d1 = _dev(_pad([ex[a][1] for a, _ in pairs], cap1))
    k2 = _dev(_pad([ex[b][0] for _, b in pairs], cap2).view(np.uint8))
    d2 = _dev(_pad([ex[b][1] for _, b in pairs], cap2))
    prev = _dev(_pad([np.stack([ex[a][0]["x"], ex[a][0]["y"]], 1).astype(np.float32) for a, _ in pairs], cap1))
    n1 = _dev(np.array([len(ex[a][0]) for a, _ in pairs], np.int32))
    n2 = _dev(np.array([len(ex[b][0]) for _, b in pairs], np.int32))
    m12 = torch.full((len(pairs), cap1), -7, dtype=torch.int32, device="cuda:0")
    nm = torch.zeros(len(pairs), dtype=torch.int32, device="cuda:0")
    m.init_batch_device(ea.camera(), len(pairs), 0.9, 1, cap1, n1.data_ptr(), k1.data_ptr(), d1.data_ptr(), cap2,
                        n2.data_ptr(), k2.data_ptr(), d2.data_ptr(), prev.data_ptr(), window, m12.data_ptr(),
                        nm.data_ptr())
    torch.cuda.synchronize()
    hm, hn, hp = m12.cpu().numpy(), nm.cpu().numpy(), prev.cpu().numpy()
    for f, (no, mo, po) in enumerate(exp):
        n = len(mo)
        assert hn[f] == no and np.array_equal(hm[f, :n], mo) and np.array_equal(hp[f, :n], po), (f, hn[f], no)
