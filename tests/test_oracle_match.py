"""CPU pinning of the oracle's relocalisation projection search
(SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist),
reference src/ORBmatcher.cc:1472-1599) against an independent pure-Python
restatement written from the reference text, on a small seeded scene with
ties, pre-assigned keypoints and the rotation-consistency filter.
"""
import math

import numpy as np
import pytest

import pyoracle as orc

f32 = np.float32
GRID_COLS, GRID_ROWS, HISTO = 64, 48, 30
SC = orc.orb_params()["scale"]


def _popcount(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def _grid(kps, w, h):
    """Frame::AssignFeaturesToGrid + PosInGrid (Frame.cc:351-366, 503-513)."""
    invW, invH = f32(GRID_COLS) / f32(w), f32(GRID_ROWS) / f32(h)
    cells = {}
    for i, k in enumerate(kps):
        px = int(np.round(f32(k["x"]) * invW))
        py = int(np.round(f32(k["y"]) * invH))
        if 0 <= px < GRID_COLS and 0 <= py < GRID_ROWS:
            cells.setdefault((px, py), []).append(i)
    return cells, invW, invH


def _in_area(cells, invW, invH, kps, x, y, r, minL, maxL):
    """Frame::GetFeaturesInArea (Frame.cc:448-501): ix, iy, cell order."""
    x0 = max(0, math.floor(f32(f32(x) - f32(r)) * invW))
    if x0 >= GRID_COLS:
        return []
    x1 = min(GRID_COLS - 1, math.ceil(f32(f32(x) + f32(r)) * invW))
    if x1 < 0:
        return []
    y0 = max(0, math.floor(f32(f32(y) - f32(r)) * invH))
    if y0 >= GRID_ROWS:
        return []
    y1 = min(GRID_ROWS - 1, math.ceil(f32(f32(y) + f32(r)) * invH))
    if y1 < 0:
        return []
    check = minL > 0 or maxL >= 0
    out = []
    for ix in range(x0, x1 + 1):
        for iy in range(y0, y1 + 1):
            for i in cells.get((ix, iy), []):
                k = kps[i]
                if check and (k["octave"] < minL or (maxL >= 0 and k["octave"] > maxL)):
                    continue
                if abs(f32(k["x"]) - f32(x)) < r and abs(f32(k["y"]) - f32(y)) < r:
                    out.append(i)
    return out


def _three_maxima(h):
    m1 = m2 = m3 = 0
    i1 = i2 = i3 = -1
    for i, s in enumerate(h):
        if s > m1:
            m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, i
        elif s > m2:
            m3, m2, i3, i2 = m2, s, i2, i
        elif s > m3:
            m3, i3 = s, i
    if m2 < f32(0.1) * f32(m1):
        i2 = i3 = -1
    elif m3 < f32(0.1) * f32(m1):
        i3 = -1
    return i1, i2, i3


def _reference_search(cam, T, th, orbdist, ori, kf, valid, pos, desc, mind, maxd, logsf, cur, cdesc, pre):
    w, h = cam.img_w, cam.img_h
    cells, invW, invH = _grid(cur, w, h)
    match = pre.copy()
    R, t = T[:3, :3].astype(np.float64), T[:3, 3].astype(np.float64)
    Ow = (-(R.T @ t)).astype(f32)
    hist = [[] for _ in range(HISTO)]
    n = 0
    for i in range(len(kf)):
        if not valid[i]:
            continue
        P = pos[i]
        pc = []
        for r_ in range(3):  # float dot, then (float)(t + c) in double (oracle transform_point)
            d = f32(f32(f32(T[r_, 0]) * P[0]) + f32(T[r_, 1]) * P[1]) + f32(T[r_, 2]) * P[2]
            pc.append(f32(float(d) + float(T[r_, 3])))
        invz = f32(1.0 / float(pc[2]))
        u = f32(f32(f32(cam.fx) * pc[0]) * invz) + f32(cam.cx)
        v = f32(f32(f32(cam.fy) * pc[1]) * invz) + f32(cam.cy)
        if u < 0 or u > w or v < 0 or v > h:
            continue
        PO = (P - Ow).astype(f32)
        dist = f32(math.sqrt(sum(float(x) * float(x) for x in PO)))
        if dist < f32(0.8) * mind[i] or dist > f32(1.2) * maxd[i]:
            continue
        lvl = math.ceil(f32(f32(math.log(float(f32(maxd[i] / dist)))) / f32(logsf)))
        lvl = min(max(lvl, 0), len(SC) - 1)
        cand = _in_area(cells, invW, invH, cur, u, v, f32(th) * SC[lvl], lvl - 1, lvl + 1)
        best, bi = 256, -1
        for i2 in cand:
            if match[i2] >= 0:
                continue
            d = _popcount(desc[i], cdesc[i2])
            if d < best:
                best, bi = d, i2
        if best <= orbdist:
            match[bi] = i
            n += 1
            if ori:
                rot = f32(kf[i]["angle"]) - f32(cur[bi]["angle"])
                if rot < 0:
                    rot = f32(rot + f32(360))
                b = int(np.round(f32(rot * f32(1.0 / HISTO))))
                hist[0 if b == HISTO else b].append(bi)
    if ori:
        keep = _three_maxima([len(x) for x in hist])
        for b in range(HISTO):
            if b not in keep:
                for i2 in hist[b]:
                    match[i2] = -1
                    n -= 1
    return n, match


@pytest.mark.parametrize("seed,ori", [(1, 1), (2, 0), (3, 1)])
def test_keyframe_search_matches_restatement(seed, ori):
    rng = np.random.default_rng(seed)
    cam = orc.cam()
    nk, nc = 160, 240
    kdt = np.dtype([("x", f32), ("y", f32), ("size", f32), ("angle", f32), ("response", f32),
                    ("octave", np.int32), ("class_id", np.int32)])
    cur = np.zeros(nc, kdt)
    cur["x"] = rng.uniform(0, 640, nc)
    cur["y"] = rng.uniform(0, 480, nc)
    cur["octave"] = rng.integers(0, 4, nc)
    cur["angle"] = rng.uniform(0, 360, nc)
    kf = np.zeros(nk, kdt)
    kf["angle"] = rng.uniform(0, 360, nk)
    # map points in front of an identity-ish camera: project near current keypoints
    T = np.eye(4, dtype=f32)
    T[:3, 3] = [0.01, -0.02, 0.03]
    z = rng.uniform(1.5, 3.0, nk).astype(f32)
    src = rng.integers(0, nc, nk)
    u = cur["x"][src] + rng.normal(0, 3, nk)
    v = cur["y"][src] + rng.normal(0, 3, nk)
    pos = np.stack([(u - cam.cx) / cam.fx * z, (v - cam.cy) / cam.fy * z, z], 1).astype(f32)
    d = np.linalg.norm(pos, axis=1).astype(f32)
    maxd = (d * SC[rng.integers(0, 4, nk)]).astype(f32)
    mind = (maxd / SC[7]).astype(f32)
    cdesc = rng.integers(0, 256, (nc, 32), dtype=np.uint8)
    desc = cdesc[src].copy()
    desc ^= (rng.integers(0, 256, desc.shape, dtype=np.uint8) & rng.choice([0, 1, 3, 0x11], desc.shape).astype(np.uint8))
    valid = (rng.random(nk) < 0.9).astype(np.uint8)
    pre = np.full(nc, -1, np.int32)
    pre[rng.choice(nc, 20, replace=False)] = 3
    logsf = float(np.log(f32(1.2)))
    no, mo = orc.match_keyframe(cam, T, 10, 100, ori, kf, valid, pos, desc, mind, maxd, logsf, cur, cdesc, pre, SC)
    nr, mr = _reference_search(cam, T, 10, 100, ori, kf, valid, pos, desc, mind, maxd, logsf, cur, cdesc, pre)
    assert no == nr and np.array_equal(mo, mr)
    assert no > 20
