"""GPU bag of words (k_bow_words / k_bow_build / k_bow_search / k_bow_rot) vs oracle/bow_ref.cpp.

Reference: src/Frame.cc:516-523 (ComputeBoW -> DBoW2 transform, levelsup 4),
Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1139-1271, src/ORBmatcher.cc:159-288 (SearchByBoW).
Bar: bit-exact (word ids, weights, FeatureVector CSR, match indices and counts). Vocabularies are
synthetic (the ORBvoc blob is missing): the ORB shape K=10, L=6 (1.1M nodes) and small trees.
"""
import numpy as np
import pytest

import eao_accel as ea
import pyoracle as orc
from tools import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def orbvoc():
    return synth.vocabulary(K=10, L=6, seed=0xB0)


def _eq_tf(g, o):
    for a, b in zip(g, o):
        assert a.shape == b.shape and np.array_equal(a, b)


@pytest.mark.parametrize("n", [1000, 0, 1, 64, 4096])
def test_transform_orb_shape(orbvoc, n):
    d = synth.bow_features(orbvoc, n, seed=n)
    g = ea.Vocab(orbvoc).transform(d, 4)
    o = orc.bow_transform(orbvoc, d, 4)
    _eq_tf(g, o)


@pytest.mark.parametrize("K,L,levelsup", [(6, 4, 2), (3, 5, 6), (10, 3, 1)])
def test_transform_small(K, L, levelsup):
    voc = synth.vocabulary(K=K, L=L, seed=K * 10 + L, stop_frac=0.2)
    d = synth.bow_features(voc, 700, seed=1)
    _eq_tf(ea.Vocab(voc).transform(d, levelsup), orc.bow_transform(voc, d, levelsup))


@pytest.mark.parametrize("check_ori,nnratio", [(1, 0.75), (0, 0.75), (1, 0.6), (1, 1.0)])
def test_search_orb_shape(orbvoc, check_ori, nnratio):
    kk, kd, kv, fk, fd = synth.bow_pair(orbvoc, 1000, 1000, seed=11)
    V = ea.Vocab(orbvoc)
    kfv, ffv = V.transform(kd)[2:], V.transform(fd)[2:]
    ng, mg = V.search(nnratio, check_ori, kk, kd, kv, kfv, fk, fd, ffv)
    no, mo = orc.search_by_bow(nnratio, check_ori, kk, kd, kv, kfv, fk, fd, ffv)
    assert ng == no and np.array_equal(mg, mo), int((mg != mo).sum())
    assert no > 100


def test_search_dense_nodes():
    """coarse FeatureVector nodes (levelsup = L - 1: K nodes of ~100 features each)."""
    voc = synth.vocabulary(K=10, L=4, seed=9)
    kk, kd, kv, fk, fd = synth.bow_pair(voc, 1200, 900, seed=3)
    V = ea.Vocab(voc)
    kfv, ffv = V.transform(kd, 3)[2:], V.transform(fd, 3)[2:]
    ng, mg = V.search(0.75, 1, kk, kd, kv, kfv, fk, fd, ffv)
    no, mo = orc.search_by_bow(0.75, 1, kk, kd, kv, kfv, fk, fd, ffv)
    assert ng == no and np.array_equal(mg, mo)


def test_search_edges(orbvoc):
    kk, kd, kv, fk, fd = synth.bow_pair(orbvoc, 300, 200, seed=4)
    V = ea.Vocab(orbvoc)
    kfv, ffv = V.transform(kd)[2:], V.transform(fd)[2:]
    none = np.zeros_like(kv)
    assert V.search(0.75, 1, kk, kd, none, kfv, fk, fd, ffv)[0] == 0  # no valid map point
    e = (np.zeros(0, np.int32), np.zeros(1, np.int32), np.zeros(0, np.int32))
    assert V.search(0.75, 1, kk, kd, kv, e, fk, fd, ffv)[0] == 0  # empty FeatureVector


def test_batch_device(orbvoc):
    import torch
    dev = torch.device("cuda", 0)
    F, cap = 12, 1024
    sizes = [1000, 0, 5, 1024, 700, 333, 1000, 64, 999, 1, 512, 800]
    desc = np.zeros((F, cap, 32), np.uint8)
    kps = np.zeros((F, cap), ea.KP_DTYPE)
    valid = np.zeros((F, cap), np.uint8)
    pairs = []
    for f, n in enumerate(sizes):
        kk, kd, kv, fk, fd = synth.bow_pair(orbvoc, max(n, 1), max(n, 1), seed=100 + f)
        pairs.append((kk[:n], kd[:n], kv[:n]))
        desc[f, :n], kps[f, :n], valid[f, :n] = kd[:n], kk[:n], kv[:n]
    V = ea.Vocab(orbvoc, max_kps=cap, max_batch=F)
    t = lambda a, dt=None: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    d_desc, d_cnt = t(desc), t(np.array(sizes, np.int32))
    z = lambda *s, dt=torch.int32: torch.zeros(s, dtype=dt, device=dev)
    wid, ww, nw = z(F, cap), z(F, cap, dt=torch.float64), z(F)
    nid, ns, nf, nn = z(F, cap), z(F, cap + 1), z(F, cap), z(F)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream())
    V.transform_batch_device(F, cap, d_cnt.data_ptr(), d_desc.data_ptr(), 4, wid.data_ptr(), ww.data_ptr(),
                             nw.data_ptr(), nid.data_ptr(), ns.data_ptr(), nf.data_ptr(), nn.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    h = [x.cpu().numpy() for x in (wid, ww, nw, nid, ns, nf, nn)]
    fvs = []
    for f, n in enumerate(sizes):
        o = orc.bow_transform(orbvoc, desc[f, :n], 4)
        k = h[6][f]
        g = (h[0][f, :h[2][f]], h[1][f, :h[2][f]], h[3][f, :k], h[4][f, :k + 1], h[5][f, :h[4][f, k]])
        _eq_tf(g, o)
        fvs.append(o[2:])
    # search f: keyframe slot f against frame slot (f + 1) % F, all HBM-resident
    nxt = [(f + 1) % F for f in range(F)]
    fr = lambda a: t(a[nxt])
    d_kps, d_valid = t(kps.view(np.uint8).reshape(F, cap, 28)), t(valid)
    match, nm = torch.full((F, cap), -7, dtype=torch.int32, device=dev), z(F)
    # the frame-side tensors are kept referenced until the launch has finished
    fside = [fr(np.array(sizes, np.int32)), fr(kps.view(np.uint8).reshape(F, cap, 28)), fr(desc), fr(h[6]),
             fr(h[3]), fr(h[4]), fr(h[5])]
    V.search_batch_device(0.75, 1, F, cap,
                          (d_kps.data_ptr(), d_desc.data_ptr(), d_valid.data_ptr(), nn.data_ptr(), nid.data_ptr(),
                           ns.data_ptr(), nf.data_ptr()),
                          tuple(x.data_ptr() for x in fside), match.data_ptr(), nm.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    hm, hn = match.cpu().numpy(), nm.cpu().numpy()
    for f in range(F):
        g2 = nxt[f]
        n2 = sizes[g2]
        kk, kd, kv = pairs[f]
        fk2, fd2 = kps[g2, :n2], desc[g2, :n2]
        no, mo = orc.search_by_bow(0.75, 1, kk, kd, kv, fvs[f], fk2, fd2, fvs[g2])
        assert hn[f] == no and np.array_equal(hm[f, :n2], mo), f


def test_search_node_capacity():
    """a vocabulary node with more than 1024 frame features is reported (EAO_E_CAPACITY),
    not silently truncated"""
    voc = synth.vocabulary(K=2, L=2, seed=5, stop_frac=0.0)
    kk, kd, kv, fk, fd = synth.bow_pair(voc, 3000, 3000, seed=6)
    V = ea.Vocab(voc, max_kps=4096)
    kfv, ffv = V.transform(kd, 1)[2:], V.transform(fd, 1)[2:]
    assert np.diff(ffv[1]).max() > 1024
    with pytest.raises(ea.EaoError, match="1024"):
        V.search(0.75, 1, kk, kd, kv, kfv, fk, fd, ffv)


# ---- SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2) (src/ORBmatcher.cc:522-655)
@pytest.mark.parametrize("check_ori,nnratio", [(1, 0.75), (0, 0.75), (1, 0.9)])
def test_search_kf_orb_shape(orbvoc, check_ori, nnratio):
    k1, d1, v1, k2, d2 = synth.bow_pair(orbvoc, 1000, 1000, seed=21)
    v2 = (np.random.default_rng(22).random(len(k2)) < 0.8).astype(np.uint8)
    V = ea.Vocab(orbvoc)
    fv1, fv2 = V.transform(d1)[2:], V.transform(d2)[2:]
    ng, mg = V.search_kf(nnratio, check_ori, k1, d1, v1, fv1, k2, d2, v2, fv2)
    no, mo = orc.search_by_bow_kf(nnratio, check_ori, k1, d1, v1, fv1, k2, d2, v2, fv2)
    assert ng == no and np.array_equal(mg, mo), int((mg != mo).sum())
    assert no > 100


def test_search_kf_dense_nodes_and_edges():
    voc = synth.vocabulary(K=10, L=4, seed=9)
    k1, d1, v1, k2, d2 = synth.bow_pair(voc, 1200, 900, seed=23)
    v2 = (np.random.default_rng(24).random(len(k2)) < 0.7).astype(np.uint8)
    V = ea.Vocab(voc)
    fv1, fv2 = V.transform(d1, 3)[2:], V.transform(d2, 3)[2:]
    g = V.search_kf(0.75, 1, k1, d1, v1, fv1, k2, d2, v2, fv2)
    o = orc.search_by_bow_kf(0.75, 1, k1, d1, v1, fv1, k2, d2, v2, fv2)
    assert g[0] == o[0] and np.array_equal(g[1], o[1])
    assert V.search_kf(0.75, 1, k1, d1, v1, fv1, k2, d2, np.zeros_like(v2), fv2)[0] == 0  # no valid KF2 point
    e = (np.zeros(0, np.int32), np.zeros(1, np.int32), np.zeros(0, np.int32))
    assert V.search_kf(0.75, 1, k1, d1, v1, e, k2, d2, v2, fv2)[0] == 0


def test_search_kf_batch_device(orbvoc):
    import torch
    dev = torch.device("cuda", 0)
    F, cap = 6, 1024
    sizes = [1000, 0, 700, 1024, 1, 333]
    desc = np.zeros((F, cap, 32), np.uint8)
    kps = np.zeros((F, cap), ea.KP_DTYPE)
    valid = np.zeros((F, cap), np.uint8)
    rng = np.random.default_rng(31)
    for f, n in enumerate(sizes):
        kk, kd, _, _, _ = synth.bow_pair(orbvoc, max(n, 1), 1, seed=200 + f)
        desc[f, :n], kps[f, :n], valid[f, :n] = kd[:n], kk[:n], (rng.random(n) < 0.85)
    # KF2 of search f = KF1 slot f re-observed (bits flipped, angles rotated): share many words
    desc2, kps2 = desc.copy(), kps.copy()
    for f, n in enumerate(sizes):
        desc2[f, :n] = synth._flip_bits(desc[f, :n].copy(), 6, rng)
        kps2[f, :n]["angle"] = np.mod(kps[f, :n]["angle"] - 40 + rng.normal(0, 3, n), 360).astype(np.float32)
    valid2 = (rng.random((F, cap)) < 0.85).astype(np.uint8)
    V = ea.Vocab(orbvoc, max_kps=cap, max_batch=F)
    fv1 = [orc.bow_transform(orbvoc, desc[f, :n], 4)[2:] for f, n in enumerate(sizes)]
    fv2 = [orc.bow_transform(orbvoc, desc2[f, :n], 4)[2:] for f, n in enumerate(sizes)]

    def csr(fvs):
        ids, st, ft, nn = np.zeros((F, cap), np.int32), np.zeros((F, cap + 1), np.int32), \
            np.zeros((F, cap), np.int32), np.zeros(F, np.int32)
        for f, (a, b, c) in enumerate(fvs):
            nn[f] = len(a)
            ids[f, :len(a)], st[f, :len(b)], ft[f, :len(c)] = a, b, c
        return ids, st, ft, nn
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    i1, s1, f1, n1 = csr(fv1)
    i2, s2, f2, n2 = csr(fv2)
    keep = [t(np.array(sizes, np.int32)), t(kps.view(np.uint8).reshape(F, cap, 28)), t(desc), t(valid), t(n1), t(i1),
            t(s1), t(f1), t(kps2.view(np.uint8).reshape(F, cap, 28)), t(desc2), t(valid2), t(n2), t(i2), t(s2), t(f2)]
    match = torch.full((F, cap), -7, dtype=torch.int32, device=dev)
    nm = torch.zeros(F, dtype=torch.int32, device=dev)
    V.search_kf_batch_device(0.75, 1, F, cap, keep[0].data_ptr(), tuple(x.data_ptr() for x in keep[1:8]),
                             tuple(x.data_ptr() for x in keep[8:]), match.data_ptr(), nm.data_ptr())
    torch.cuda.synchronize()
    hm, hn = match.cpu().numpy(), nm.cpu().numpy()
    for f, n in enumerate(sizes):
        no, mo = orc.search_by_bow_kf(0.75, 1, kps[f, :n], desc[f, :n], valid[f, :n], fv1[f], kps2[f, :n],
                                      desc2[f, :n], valid2[f, :n], fv2[f])
        assert hn[f] == no and np.array_equal(hm[f, :n], mo), f
    assert hn.max() > 100
