"""BoW oracle (oracle/bow_ref.cpp) against an independent pure-Python restatement.

Reference: Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1139-1206,1230-1271 (transform, TF_IDF,
L1 normalisation) and src/ORBmatcher.cc:159-288 (SearchByBoW, ComputeThreeMaxima :1601-1642).
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
