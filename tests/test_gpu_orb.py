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

SC = orc.orb_params()["scale"]


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


@pytest.mark.parametrize("w,h", [(641, 481), (320, 240), (800, 600), (1000, 700), (1280, 720), (1920, 1080), (3840, 2160)])
def test_pyramid_exact_sizes(w, h):
    # k_resize_lds: unaligned rows (odd widths: byte staging of level 0), a partial last column
    # group / row tile, wide levels with one 4-row segment per 1024-thread tile (4K); k_pyr_tail:
    # levels 2-7 (320x240), 5-7 (641x481), 6-7 (800x600), 7 (1000x700), none (1280x720 and up); the
    # debug pyramid takes the batch form (k_pyr_tail) also for one image
    img = np.random.default_rng(w + h).integers(0, 256, (h, w), dtype=np.uint8)
    orb = ea.Orb(width=w, height=h, nfeatures=2000)
    g = orb.pyramid(img)
    o = orc.pyramid(img)
    for l, (a, b) in enumerate(zip(g, o)):
        assert a.shape == b.shape
        assert np.array_equal(a, b), "%dx%d level %d differs at %d px" % (w, h, l, int((a != b).sum()))


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


@pytest.mark.parametrize("w,h", [(641, 481), (333, 257)])
def test_extract_single_call_odd_sizes(w, h):
    # the single call moves its image in 16-byte units by kernel (OrbEngine::image_in): w*h not a
    # multiple of 16, and the outputs back by kernel (count, keypoints, descriptors), twice in a row
    img = synth.render(synth.texture(w * h, 2048), synth.camera_path(1, w)[0], w, h,
                       K=(0.8 * w, 0.8 * w, 0.5 * w, 0.5 * h))
    orb = ea.Orb(width=w, height=h, nfeatures=1000)
    ok, od = orc.extract(img)
    for _ in range(2):
        gk, gd = orb.extract(img)
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


def _batch_extract(fr, nfeat, w, h):
    import torch
    F = len(fr)
    dev = torch.device("cuda", 0)
    orb = ea.Orb(nfeat, 1.2, 8, 20, 7, w, h, max_batch=F)
    cap = orb.cap
    d_fr = torch.from_numpy(np.stack(fr)).to(dev)
    kps = torch.zeros((F, cap, 28), dtype=torch.uint8, device=dev)
    desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(F, dtype=torch.int32, device=dev)
    orb.extract_batch_device(d_fr.data_ptr(), F, w, kps.data_ptr(), desc.data_ptr(), cnt.data_ptr(), cap, None)
    torch.cuda.synchronize()
    return cnt.cpu().numpy(), kps.cpu().numpy().view(ea.KP_DTYPE).reshape(F, cap), desc.cpu().numpy()


def test_batch_full_bench_stream_exact():
    """The bench's whole 405-frame batch in one launch group: every frame
    bit-exact, then the 404 motion-model searches of the batch (two-phase
    kernels) against the oracle pair by pair. A full batch keeps thousands of
    workgroups in flight at once, which is what exposes cross-workgroup
    buffer overlap."""
    import torch
    fr, poses = synth.frame_stream(405)
    n, hk, hd = _batch_extract(fr, 1000, 640, 480)
    bad = []
    okps, odesc = [], []
    for t in range(len(fr)):
        ok, od = orc.extract(fr[t])
        okps.append(ok)
        odesc.append(od)
        if not (n[t] == len(ok) and np.array_equal(hk[t, :n[t]], ok) and np.array_equal(hd[t, :n[t]], od)):
            bad.append(t)
    assert not bad, "frames differing: %s" % bad[:20]
    F, cap = len(fr), hk.shape[1]
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(9)
    has = np.zeros((F, cap), np.uint8)
    pos = np.zeros((F, cap, 3), np.float32)
    for t in range(F):
        has[t, :n[t]] = rng.random(n[t]) < 0.9
        pos[t, :n[t]] = synth.backproject(poses[t], okps[t]["x"], okps[t]["y"])
    kps = torch.from_numpy(hk.view(np.uint8).reshape(F, cap, 28)).to(dev)
    desc = torch.from_numpy(hd).to(dev)
    cnt = torch.from_numpy(n.astype(np.int32)).to(dev)
    T = torch.from_numpy(np.stack(poses).astype(np.float32).reshape(F, 16)).to(dev)
    d_has, d_pos = torch.from_numpy(has).to(dev), torch.from_numpy(pos).to(dev)
    match = torch.full((F, cap), -1, dtype=torch.int32, device=dev)
    nm = torch.zeros(F, dtype=torch.int32, device=dev)
    ea.Matcher(max_kps=cap, max_batch=F).motion_batch_device(
        ea.camera(), F, cap, T.data_ptr(), 15, 1, kps.data_ptr(), desc.data_ptr(), cnt.data_ptr(), d_has.data_ptr(),
        d_pos.data_ptr(), desc.data_ptr(), SC, match.data_ptr(), nm.data_ptr(), None)
    torch.cuda.synchronize()
    hm, hn = match.cpu().numpy(), nm.cpu().numpy()
    badm = []
    for t in range(1, F):
        no, mo = orc.match_motion(orc.cam(), poses[t], 15, 1, okps[t - 1], has[t - 1, :n[t - 1]],
                                  pos[t - 1, :n[t - 1]], odesc[t - 1], okps[t], odesc[t], SC)
        if not (hn[t] == no and np.array_equal(hm[t, :n[t]], mo)):
            badm.append(t)
    assert not badm, "pairs differing: %s" % badm[:20]


def test_batch_1080p_4000_features_exact():
    """Config B shape (1920x1080, 4000 features): the largest quadtree
    capacity instantiation, batched."""
    fr, _ = synth.frame_stream(12, w=1920, h=1080, seed=0xEA4)
    n, hk, hd = _batch_extract(fr, 4000, 1920, 1080)
    for t in range(len(fr)):
        ok, od = orc.extract(fr[t], 4000)
        assert n[t] == len(ok) and np.array_equal(hk[t, :n[t]], ok) and np.array_equal(hd[t, :n[t]], od), t


@pytest.mark.parametrize("w,h,cn,rgb", [(640, 480, 3, True), (640, 480, 3, False), (533, 37, 4, True), (640, 7, 4, False),
                                        (61, 9, 3, True)])
def test_color_to_gray_batch(w, h, cn, rgb):
    """Frame input stage (src/Tracking.cc:349-362) vs the oracle, vector and
    ragged-width scalar paths."""
    import torch
    rng = np.random.default_rng(w + cn)
    col = rng.integers(0, 256, (3, h, w, cn), dtype=np.uint8)
    dev = torch.device("cuda", 0)
    d_col = torch.from_numpy(col).to(dev)
    d_g = torch.zeros((3, h, w), dtype=torch.uint8, device=dev)
    ea.color_to_gray_batch_device(d_col.data_ptr(), 3, w, h, w * cn, cn, rgb, d_g.data_ptr(), w)
    torch.cuda.synchronize()
    g = d_g.cpu().numpy()
    for f in range(3):
        assert np.array_equal(g[f], orc.color_to_gray(col[f], rgb)), f


def test_color_frames_through_extraction():
    """Colour frames -> GPU gray -> batched extraction equals the oracle's
    cvtColor + ORBextractor on the same frames."""
    import torch
    fr, _ = synth.frame_stream(3)
    rng = np.random.default_rng(4)
    col = np.stack([np.stack([np.clip(f.astype(np.int16) + rng.integers(-6, 7, f.shape), 0, 255).astype(np.uint8)
                              for _ in range(3)], -1) for f in fr])
    dev = torch.device("cuda", 0)
    d_col = torch.from_numpy(col).to(dev)
    d_g = torch.zeros((3, 480, 640), dtype=torch.uint8, device=dev)
    ea.color_to_gray_batch_device(d_col.data_ptr(), 3, 640, 480, 640 * 3, 3, True, d_g.data_ptr(), 640)
    torch.cuda.synchronize()
    gray = list(d_g.cpu().numpy())
    n, hk, hd = _batch_extract(gray, 1000, 640, 480)
    for t in range(3):
        og = orc.color_to_gray(col[t], True)
        assert np.array_equal(gray[t], og)
        ok, od = orc.extract(og)
        assert n[t] == len(ok) and np.array_equal(hk[t, :n[t]], ok) and np.array_equal(hd[t, :n[t]], od)
