"""BoW oracle (oracle/bow_ref.cpp) against an independent pure-Python restatement.

Reference: Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1139-1206,1230-1271 (transform, TF_IDF,
L1 normalisation), src/ORBmatcher.cc:159-288 (SearchByBoW(KeyFrame*, Frame&)), :522-655
(SearchByBoW(KeyFrame*, KeyFrame*)) and ComputeThreeMaxima (:1601-1642).
The reference's Vocabulary/ORBvoc.bin is a missing blob: vocabularies are synthetic
(tools/synth.vocabulary), so parity against the original vocabulary is unpinned.
"""
import numpy as np
import pytest

import pyoracle as orc
from tools import synth

POP = np.array([bin(i).count("1") for i in range(256)], np.int32)


def _ham(a, B):
    return POP[np.bitwise_xor(a[None, :], B)].sum(1)


def transform_py(voc, desc, levelsup):
    ch = {}
    for i, p in enumerate(voc["parent"]):
        if p >= 0:
            ch.setdefault(int(p), []).append(i)
    nid_level = voc["L"] - levelsup
    bow, fv = {}, {}
    for i, d in enumerate(desc):
        fid, lvl, nid = 0, 0, 0
        while True:
            lvl += 1
            c = ch[fid]
            dist = _ham(d, voc["desc"][c])
            fid = c[int(np.argmin(dist))]  # first minimum
            if lvl == nid_level:
                nid = fid
            if fid not in ch:
                break
        w = voc["weight"][fid]
        if w > 0:
            wid = int(voc["word"][fid])
            bow[wid] = bow[wid] + w if wid in bow else w
            fv.setdefault(nid, []).append(i)
    norm = 0.0
    for k in sorted(bow):
        norm += abs(bow[k])
    words = sorted(bow)
    ww = [bow[k] / norm for k in words] if norm > 0 else [bow[k] for k in words]
    nodes = sorted(fv)
    start = np.cumsum([0] + [len(fv[k]) for k in nodes])
    feats = [f for k in nodes for f in fv[k]]
    return np.array(words), np.array(ww), np.array(nodes), start, np.array(feats)


def search_py(nnratio, check_ori, kk, kd, kv, kfv, fk, fd, ffv):
    match = np.full(len(fk), -1)
    hist = [[] for _ in range(30)]
    fpos = {int(n): j for j, n in enumerate(ffv[0])}
    for a, node in enumerate(kfv[0]):
        b = fpos.get(int(node))
        if b is None:
            continue
        fl = list(ffv[2][ffv[1][b]:ffv[1][b + 1]])
        for ikf in kfv[2][kfv[1][a]:kfv[1][a + 1]]:
            if not kv[ikf]:
                continue
            free = [i for i in fl if match[i] < 0]
            if not free:
                continue
            d = _ham(kd[ikf], fd[free])
            order = np.argsort(d, kind="stable")
            b1 = int(d[order[0]])
            b2 = int(d[order[1]]) if len(free) > 1 else 256
            if b1 <= 50 and np.float32(b1) < np.float32(nnratio) * np.float32(b2):
                idx = free[order[0]]
                match[idx] = ikf
                rot = np.float32(kk["angle"][ikf]) - np.float32(fk["angle"][idx])
                if rot < 0:
                    rot = np.float32(rot + np.float32(360))
                bn = int(np.round(np.float32(rot * np.float32(1 / 30))))
                hist[0 if bn == 30 else bn].append(idx)
    if check_ori:
        sizes = [len(h) for h in hist]
        top = []
        m1 = m2 = m3 = 0
        i1 = i2 = i3 = -1
        for i, s in enumerate(sizes):
            if s > m1:
                m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, i
            elif s > m2:
                m3, m2, i3, i2 = m2, s, i2, i
            elif s > m3:
                m3, i3 = s, i
        if m2 < 0.1 * m1:
            i2 = i3 = -1
        elif m3 < 0.1 * m1:
            i3 = -1
        for i in range(30):
            if i not in (i1, i2, i3):
                for j in hist[i]:
                    match[j] = -1
    return int((match >= 0).sum()), match


def three_maxima_keep(hist):
    sizes = [len(h) for h in hist]
    m1 = m2 = m3 = 0
    i1 = i2 = i3 = -1
    for i, sz in enumerate(sizes):
        if sz > m1:
            m3, m2, m1, i3, i2, i1 = m2, m1, sz, i2, i1, i
        elif sz > m2:
            m3, m2, i3, i2 = m2, sz, i2, i
        elif sz > m3:
            m3, i3 = sz, i
    if m2 < 0.1 * m1:
        i2 = i3 = -1
    elif m3 < 0.1 * m1:
        i3 = -1
    return (i1, i2, i3)


def search_kf_py(nnratio, check_ori, k1, d1, v1, fv1, k2, d2, v2, fv2):
    """SearchByBoW(KeyFrame*, KeyFrame*) restated from ORBmatcher.cc:522-655 in pure Python: both
    sides' map points checked, vbMatched2 first-wins, bestDist1 < TH_LOW (strict), ratio test,
    the histogram over idx1 with rot = angle1 - angle2."""
    match = np.full(len(k1), -1)
    matched2 = np.zeros(len(k2), bool)
    hist = [[] for _ in range(30)]
    pos2 = {int(n): j for j, n in enumerate(fv2[0])}
    for a, node in enumerate(fv1[0]):
        b = pos2.get(int(node))
        if b is None:
            continue
        cand = [int(i) for i in fv2[2][fv2[1][b]:fv2[1][b + 1]]]
        for i1 in fv1[2][fv1[1][a]:fv1[1][a + 1]]:
            if not v1[i1]:
                continue
            best1, best2, bi = 256, 256, -1
            for i2 in cand:  # the reference's scan: first minimum kept
                if matched2[i2] or not v2[i2]:
                    continue
                dd = int(_ham(d1[i1], d2[i2:i2 + 1])[0])
                if dd < best1:
                    best2, best1, bi = best1, dd, i2
                elif dd < best2:
                    best2 = dd
            if best1 < 50 and np.float32(best1) < np.float32(nnratio) * np.float32(best2):
                match[i1] = bi
                matched2[bi] = True
                rot = np.float32(k1["angle"][i1]) - np.float32(k2["angle"][bi])
                if rot < 0:
                    rot = np.float32(rot + np.float32(360))
                bn = int(np.round(np.float32(rot * np.float32(1 / 30))))
                hist[0 if bn == 30 else bn].append(int(i1))
    if check_ori:
        keep = three_maxima_keep(hist)
        for i in range(30):
            if i not in keep:
                for j in hist[i]:
                    match[j] = -1
    return int((match >= 0).sum()), match


@pytest.fixture(scope="module")
def voc():
    return synth.vocabulary(K=6, L=4, seed=3)


@pytest.mark.parametrize("levelsup", [2, 3, 4])
def test_transform_vs_python(voc, levelsup):
    d = synth.bow_features(voc, 300, seed=levelsup)
    o = orc.bow_transform(voc, d, levelsup)
    p = transform_py(voc, d, levelsup)
    for a, b in zip(o[:1] + o[2:], p[:1] + p[2:]):
        assert np.array_equal(a, b)
    assert np.allclose(o[1], p[1], rtol=0, atol=1e-15)
    assert abs(o[1].sum() - 1) < 1e-12


@pytest.mark.parametrize("check_ori", [1, 0])
def test_search_vs_python(voc, check_ori):
    kk, kd, kv, fk, fd = synth.bow_pair(voc, 500, 450, seed=5)
    V = orc.Vocab(voc)
    kfv = orc.bow_transform(V, kd, 2)[2:]
    ffv = orc.bow_transform(V, fd, 2)[2:]
    n, m = orc.search_by_bow(0.75, check_ori, kk, kd, kv, kfv, fk, fd, ffv)
    n2, m2 = search_py(0.75, check_ori, kk, kd, kv, kfv, fk, fd, ffv)
    assert n == n2 and np.array_equal(m, m2)
    assert n > 50


def test_empty_vocabulary():
    voc = {"desc": np.zeros((1, 32), np.uint8), "parent": np.array([-1], np.int32),
           "word": np.array([-1], np.int32), "weight": np.zeros(1), "L": 0}
    o = orc.bow_transform(voc, np.zeros((5, 32), np.uint8))
    assert len(o[0]) == 0 and len(o[2]) == 0


@pytest.mark.parametrize("check_ori", [1, 0])
def test_search_kf_vs_python(voc, check_ori):
    """SearchByBoW(KF1, KF2) (ORBmatcher.cc:522-655): oracle == the pure-Python restatement; both
    sides carry invalid map points, and a distance exactly TH_LOW (50) is rejected (strict bar)."""
    k1, d1, v1, k2, d2 = synth.bow_pair(voc, 500, 450, seed=9)
    v2 = (np.random.default_rng(10).random(len(k2)) < 0.85).astype(np.uint8)
    V = orc.Vocab(voc)
    fv1 = orc.bow_transform(V, d1, 2)[2:]
    fv2 = orc.bow_transform(V, d2, 2)[2:]
    n, m = orc.search_by_bow_kf(0.75, check_ori, k1, d1, v1, fv1, k2, d2, v2, fv2)
    n2, m2 = search_kf_py(0.75, check_ori, k1, d1, v1, fv1, k2, d2, v2, fv2)
    assert n == n2 and np.array_equal(m, m2)
    assert n > 50
    assert all(v2[j] for j in m[m >= 0]) and all(v1[i] for i in np.nonzero(m >= 0)[0])
    assert len(set(m[m >= 0].tolist())) == n  # vbMatched2: one KF1 feature per KF2 feature


def test_search_kf_strict_th_low():
    """bestDist1 < TH_LOW (ORBmatcher.cc:594) in the keyframe-keyframe search, <= in the keyframe-frame
    one (:217): a single pair at Hamming distance exactly 50 matches only in the latter."""
    d1 = np.zeros((1, 32), np.uint8)
    d2 = np.zeros((1, 32), np.uint8)
    bits = np.unpackbits(d2[0])
    bits[:50] = 1
    d2[0] = np.packbits(bits)
    dt = orc.KP_DTYPE
    k = np.zeros(1, dt)
    fv = (np.array([5], np.int32), np.array([0, 1], np.int32), np.array([0], np.int32))
    one = np.ones(1, np.uint8)
    n, m = orc.search_by_bow_kf(0.9, 0, k, d1, one, fv, k, d2, one, fv)
    assert n == 0 and m[0] == -1
    assert orc.search_by_bow(0.9, 0, k, d1, one, fv, k, d2, fv)[0] == 1
    bits[49] = 0
    d2[0] = np.packbits(bits)  # distance 49: both match
    assert orc.search_by_bow_kf(0.9, 0, k, d1, one, fv, k, d2, one, fv)[0] == 1
