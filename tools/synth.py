"""Deterministic synthetic TUM-shaped inputs.

There is no network and no TUM dataset in this pipeline, so every workload is
generated procedurally from fixed seeds:

* ``texture(seed)``      -- a large u8 texture: value-noise octaves + random
                            rectangles, smoothed lightly; dense FAST corners.
* ``render(...)``        -- a 640x480 (or any) view of a textured plane Z=depth
                            seen from a camera pose (pinhole, TUM3 intrinsics),
                            so consecutive frames overlap like a real sequence
                            and every pixel has a known 3-D point.
* ``camera_path(n)``     -- smooth poses Tcw (4x4 float32) along a short arc.
* ``frame_stream(...)``  -- a (n, h, w) u8 stack of rendered frames.

All arithmetic is numpy with explicit seeds (PCG64), so results are identical
here and on the GPU box.
"""
import os

import numpy as np

TUM3_K = (535.4, 539.2, 320.1, 247.6)  # Examples/Monocular/TUM3.yaml:8-11


def _smooth(a, passes=1):
    for _ in range(passes):
        a = (a + np.roll(a, 1, 0) + np.roll(a, -1, 0) + np.roll(a, 1, 1) + np.roll(a, -1, 1)) / 5.0
    return a


def texture(seed=0xEA0, size=2048, structure=False):
    """structure=True adds office-like straight structure (posters, screens, shelf and desk edges:
    large flat rectangles and long bars with sharp edges, own seeded stream) so that views carry
    the long straight edges the line detector finds; the default texture, which
    the committed fixtures were made from, is unchanged."""
    rng = np.random.Generator(np.random.PCG64(seed))
    img = np.zeros((size, size), np.float64)
    for octave, amp in ((8, 60.0), (32, 40.0), (128, 25.0)):
        g = rng.random((size // octave + 2, size // octave + 2))
        idx = np.arange(size) / octave
        i0 = idx.astype(np.int64)
        f = idx - i0
        rows = g[i0][:, i0] * (1 - f)[None, :] + g[i0][:, i0 + 1] * f[None, :]
        rows2 = g[i0 + 1][:, i0] * (1 - f)[None, :] + g[i0 + 1][:, i0 + 1] * f[None, :]
        img += amp * (rows * (1 - f)[:, None] + rows2 * f[:, None])
    n_rect = size * size // 900
    xs = rng.integers(0, size, n_rect)
    ys = rng.integers(0, size, n_rect)
    ws = rng.integers(3, 24, n_rect)
    hs = rng.integers(3, 24, n_rect)
    vs = rng.uniform(-70, 70, n_rect)
    for x, y, w, h, v in zip(xs, ys, ws, hs, vs):
        img[y:y + h, x:x + w] += v
    img = _smooth(img, 1)
    img = img - img.min()
    img = img * (235.0 / max(img.max(), 1e-9)) + 10.0
    if structure:  # sharp-edged, painted over the smoothed texture: 50-70 EDLine segments per view
        srng = np.random.Generator(np.random.PCG64(seed + 0x5157))
        for _ in range(size * size // 8000):
            x, y = int(srng.integers(0, size)), int(srng.integers(0, size))
            if srng.random() < 0.3:  # a long thin bar (shelf / desk / frame edge)
                w, h = (int(srng.integers(120, 500)), int(srng.integers(4, 10)))
                if srng.random() < 0.5:
                    w, h = h, w
            else:  # a flat panel
                w, h = int(srng.integers(60, 260)), int(srng.integers(60, 260))
            img[y:y + h, x:x + w] = srng.uniform(0, 255) + 0.15 * img[y:y + h, x:x + w]
    return np.clip(img, 0, 255).astype(np.uint8)


def camera_path(n, seed=0xEA0, step=0.004):
    """Poses Tcw looking down +Z at the plane; slow translation + small yaw."""
    rng = np.random.Generator(np.random.PCG64(seed + 17))
    phase = rng.uniform(0, 2 * np.pi)
    poses = np.zeros((n, 4, 4), np.float32)
    for i in range(n):
        t = i * step
        yaw = 0.05 * np.sin(0.7 * t * 40 + phase)
        c, s = np.cos(yaw), np.sin(yaw)
        Rwc = np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]], np.float64)
        twc = np.array([0.6 * np.sin(t * 3.0 + phase), 0.4 * np.cos(t * 2.0), 0.05 * np.sin(t * 5.0)])
        Rcw = Rwc.T
        tcw = -Rcw @ twc
        poses[i, :3, :3] = Rcw
        poses[i, :3, 3] = tcw
        poses[i, 3, 3] = 1
    return poses


def render(tex, Tcw, w=640, h=480, depth=2.0, K=TUM3_K, px_per_m=600.0):
    """Render the plane Z=depth (world) textured with ``tex`` from pose Tcw."""
    fx, fy, cx, cy = K
    Rcw = Tcw[:3, :3].astype(np.float64)
    tcw = Tcw[:3, 3].astype(np.float64)
    Rwc = Rcw.T
    twc = -Rwc @ tcw
    u, v = np.meshgrid(np.arange(w, dtype=np.float64), np.arange(h, dtype=np.float64))
    d = np.stack([(u - cx) / fx, (v - cy) / fy, np.ones_like(u)], -1) @ Rwc.T
    lam = (depth - twc[2]) / d[..., 2]
    X = twc[0] + lam * d[..., 0]
    Y = twc[1] + lam * d[..., 1]
    ts = tex.shape[0]
    tx = X * px_per_m + ts / 2
    ty = Y * px_per_m + ts / 2
    x0 = np.clip(np.floor(tx).astype(np.int64), 0, ts - 2)
    y0 = np.clip(np.floor(ty).astype(np.int64), 0, ts - 2)
    fx_ = np.clip(tx - x0, 0, 1)
    fy_ = np.clip(ty - y0, 0, 1)
    t = tex.astype(np.float64)
    val = (t[y0, x0] * (1 - fx_) * (1 - fy_) + t[y0, x0 + 1] * fx_ * (1 - fy_) +
           t[y0 + 1, x0] * (1 - fx_) * fy_ + t[y0 + 1, x0 + 1] * fx_ * fy_)
    return np.clip(np.rint(val), 0, 255).astype(np.uint8)


def backproject(Tcw, u, v, depth=2.0, K=TUM3_K):
    """World points on the plane Z=depth under pixels (u, v) (float32 (n,3))."""
    fx, fy, cx, cy = K
    Rcw = Tcw[:3, :3].astype(np.float64)
    tcw = Tcw[:3, 3].astype(np.float64)
    Rwc = Rcw.T
    twc = -Rwc @ tcw
    d = np.stack([(np.asarray(u, np.float64) - cx) / fx, (np.asarray(v, np.float64) - cy) / fy,
                  np.ones(len(u))], -1) @ Rwc.T
    lam = (depth - twc[2]) / d[:, 2]
    return (twc[None, :] + lam[:, None] * d).astype(np.float32)


def frame_stream(n, w=640, h=480, seed=0xEA0, step=0.004, structure=False):
    tex = texture(seed, 2048 if max(w, h) <= 640 else 4096, structure)
    poses = camera_path(n, seed, step)
    frames = np.stack([render(tex, poses[i], w, h) for i in range(n)])
    return frames, poses


# ----------------------------------------------------------------------------
# Association workload: objects with point clouds
# seen along a camera path, YOLO-like boxes, tracked map points per frame.
# Class mix follows the reference's data/yolo_txts (39 bottle, 56 chair,
# 73 book, 62 tv, 41 cup, 66 keyboard, 64 mouse, 77 teddy bear, 0 person).
OFFICE_CLASSES = [39, 39, 39, 56, 56, 73, 73, 62, 41, 66, 64, 77, 0, 72]
# the fr3_long_office shape of SURVEY.md §8d input 2: about 7 boxes per frame
# (17,181 YOLO boxes over 2,585 frames), m = 5-300 points per box, about a
# thousand tracked map points per frame (1000 ORB features)
FR3_CLASSES = [39, 39, 56, 56, 73, 62, 41, 66, 64]
CLASS_EXTENT = {39: (0.07, 0.07, 0.22), 56: (0.45, 0.45, 0.8), 73: (0.2, 0.05, 0.25),
                62: (0.5, 0.08, 0.35), 41: (0.08, 0.08, 0.1), 66: (0.45, 0.15, 0.03),
                64: (0.06, 0.1, 0.04), 77: (0.25, 0.2, 0.3), 0: (0.5, 0.3, 1.6), 72: (0.4, 0.3, 0.6)}


def _look_at(eye, target):
    z = target - eye
    z = z / np.linalg.norm(z)
    up = np.array([0.0, 0.0, 1.0])
    x = np.cross(z, up)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    Rwc = np.stack([x, y, z], 1)  # columns = camera axes in world
    Rcw = Rwc.T
    T = np.eye(4)
    T[:3, :3] = Rcw
    T[:3, 3] = -Rcw @ eye
    return T.astype(np.float32)


def assoc_scene(seed=0xEA1, classes=None, pts_range=(150, 600), n_background=800):
    rng = np.random.Generator(np.random.PCG64(seed))
    classes = OFFICE_CLASSES if classes is None else classes
    objs = []
    mp_pos = []
    mp_obj = []
    for k, c in enumerate(classes):
        ang = 2 * np.pi * k / len(classes) + rng.uniform(-0.2, 0.2)
        rad = rng.uniform(0.2, 0.9)
        center = np.array([rad * np.cos(ang), rad * np.sin(ang), 0.0])
        ext = np.array(CLASS_EXTENT.get(c, (0.2, 0.2, 0.2)))
        center[2] = ext[2] / 2 + rng.uniform(0, 0.3)
        n = int(rng.integers(*pts_range))
        p = rng.normal(0, 1, (n, 3)) * (ext / 4)
        p = np.clip(p, -ext / 2, ext / 2) + center
        n_out = max(1, n // 20)
        p[:n_out] = center + rng.uniform(-1, 1, (n_out, 3)) * (ext / 2 + 0.25)
        objs.append(dict(cls=c, center=center, ext=ext, first=len(mp_pos), n=n))
        mp_pos.extend(p.tolist())
        mp_obj.extend([k] * n)
    bg = rng.uniform([-2.5, -2.5, 0], [2.5, 2.5, 2.0], (n_background, 3))
    mp_pos.extend(bg.tolist())
    mp_obj.extend([-1] * n_background)
    return objs, np.asarray(mp_pos, np.float32), np.asarray(mp_obj, np.int32)


# cuboid corner numbering of Object_Map::mCuboid3D (corner_1..8: z-min face
# counter-clockwise from (x_min, y_min), then the z-max face), Object.cc:1040-1080
_CORNERS = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0], [0, 0, 1], [1, 0, 1], [1, 1, 1], [0, 1, 1]], float)
_EDGES = [(0, 1), (1, 2), (2, 3), (3, 0), (4, 5), (5, 6), (6, 7), (7, 4), (0, 4), (1, 5), (2, 6), (3, 7)]


def frame_lines(T, objs, rng, K=TUM3_K, w=640, h=480, n_clutter=12):
    """Synthetic Frame::all_lines_eigen (SURVEY §8d input 2: "projected cuboid
    edges +-2 deg noise"): the visible edges of every object's ground-truth box,
    each rotated about its midpoint by N(0, 1 deg) clipped to +-2 deg, about a
    third of the long ones broken in two (so merge_break_lines has work), plus
    random clutter segments; endpoints in random order, float32 (L, 4)."""
    fx, fy, cx, cy = K
    segs = []
    for o in objs:
        c = o["center"] + (_CORNERS - 0.5) * np.asarray(o["ext"])
        Pc = c @ T[:3, :3].T.astype(np.float64) + T[:3, 3]
        if (Pc[:, 2] < 0.1).any():
            continue
        uv = np.stack([fx * Pc[:, 0] / Pc[:, 2] + cx, fy * Pc[:, 1] / Pc[:, 2] + cy], 1)
        for a, b in _EDGES:
            p, q = uv[a], uv[b]
            if not (0 <= p[0] < w and 0 <= p[1] < h and 0 <= q[0] < w and 0 <= q[1] < h):
                continue
            d = q - p
            ln = float(np.hypot(*d))
            if ln < 15:
                continue
            th = np.deg2rad(float(np.clip(rng.normal(0, 1.0), -2, 2)))
            m = (p + q) / 2
            rot = np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
            p, q = m + rot @ (p - m), m + rot @ (q - m)
            if ln > 60 and rng.random() < 0.3:
                t0 = rng.uniform(0.3, 0.7)
                gap = 4.0 / ln
                segs.append(np.concatenate([p, p + (q - p) * (t0 - gap)]))
                segs.append(np.concatenate([p + (q - p) * (t0 + gap), q]))
            else:
                segs.append(np.concatenate([p, q]))
    for _ in range(n_clutter):
        m = rng.uniform([0, 0], [w, h])
        ang, ln = rng.uniform(0, np.pi), rng.uniform(10, 80)
        d = 0.5 * ln * np.array([np.cos(ang), np.sin(ang)])
        segs.append(np.concatenate([m - d, m + d]))
    L = np.asarray(segs, np.float64).reshape(-1, 4)
    flip = rng.random(len(L)) < 0.5
    L[flip] = L[flip][:, [2, 3, 0, 1]]
    return L[rng.permutation(len(L))].astype(np.float32)


def frame_lines_vec(T, objs, rng, K=TUM3_K, w=640, h=480, n_clutter=12):
    """frame_lines' segment model, vectorised over objects and edges (its own draw
    order; used by the fr3 streams, whose maps hold ~100 objects)."""
    fx, fy, cx, cy = K
    if not objs:
        return np.zeros((0, 4), np.float32)
    ctr = np.stack([o["center"] for o in objs])
    ext = np.stack([np.asarray(o["ext"], np.float64) for o in objs])
    c = ctr[:, None, :] + (_CORNERS[None] - 0.5) * ext[:, None, :]  # (O, 8, 3)
    Pc = c @ T[:3, :3].T.astype(np.float64) + T[:3, 3]
    front = (Pc[..., 2] >= 0.1).all(1)
    with np.errstate(divide="ignore", invalid="ignore"):
        uv = np.stack([fx * Pc[..., 0] / Pc[..., 2] + cx, fy * Pc[..., 1] / Pc[..., 2] + cy], -1)
    ea, eb = np.array([e[0] for e in _EDGES]), np.array([e[1] for e in _EDGES])
    p, q = uv[:, ea].reshape(-1, 2), uv[:, eb].reshape(-1, 2)  # (O*12, 2)
    inside = lambda a: (a[:, 0] >= 0) & (a[:, 0] < w) & (a[:, 1] >= 0) & (a[:, 1] < h)
    ln = np.hypot(*(q - p).T)
    keep = np.repeat(front, len(_EDGES)) & inside(p) & inside(q) & (ln >= 15)
    p, q, ln = p[keep], q[keep], ln[keep]
    th = np.deg2rad(np.clip(rng.normal(0, 1.0, len(p)), -2, 2))
    m = (p + q) / 2
    cs, sn = np.cos(th)[:, None], np.sin(th)[:, None]
    rot = lambda a: m + np.concatenate([cs * (a - m)[:, :1] - sn * (a - m)[:, 1:], sn * (a - m)[:, :1] + cs * (a - m)[:, 1:]], 1)
    p, q = rot(p), rot(q)
    brk = (ln > 60) & (rng.random(len(p)) < 0.3)
    t0 = rng.uniform(0.3, 0.7, len(p))
    gap = 4.0 / np.maximum(ln, 1e-9)
    segs = [np.concatenate([p[~brk], q[~brk]], 1),
            np.concatenate([p[brk], p[brk] + (q[brk] - p[brk]) * (t0[brk] - gap[brk])[:, None]], 1),
            np.concatenate([p[brk] + (q[brk] - p[brk]) * (t0[brk] + gap[brk])[:, None], q[brk]], 1)]
    mc = rng.uniform([0, 0], [w, h], (n_clutter, 2))
    ang, cl = rng.uniform(0, np.pi, n_clutter), rng.uniform(10, 80, n_clutter)
    dd = 0.5 * cl[:, None] * np.stack([np.cos(ang), np.sin(ang)], 1)
    segs.append(np.concatenate([mc - dd, mc + dd], 1))
    L = np.concatenate(segs).astype(np.float64)
    flip = rng.random(len(L)) < 0.5
    L[flip] = L[flip][:, [2, 3, 0, 1]]
    return L[rng.permutation(len(L))].astype(np.float32)


def assoc_stream(n_frames=405, seed=0xEA1, K=TUM3_K, w=640, h=480, classes=None, obs_frac=0.7,
                 kf_every=5, pts_range=(150, 600), n_background=800, lines=False):
    """Per-frame replay inputs for the association path.
    lines=True adds each frame's line segments (frame_lines, own seeded stream
    0xEA2 so the rest of the stream is unchanged)."""
    fx, fy, cx, cy = K
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    lrng = np.random.Generator(np.random.PCG64(0xEA2 + seed))
    objs, P, owner = assoc_scene(seed, classes, pts_range, n_background)
    frames = []
    for t in range(n_frames):
        a = -0.6 + 1.6 * t / max(1, n_frames - 1)
        eye = np.array([2.3 * np.cos(a), 2.3 * np.sin(a), 1.3 + 0.1 * np.sin(3 * a)])
        T = _look_at(eye, np.array([0.0, 0.0, 0.3]))
        Pc = P @ T[:3, :3].T.astype(np.float64) + T[:3, 3]
        z = Pc[:, 2]
        u = fx * Pc[:, 0] / z + cx
        v = fy * Pc[:, 1] / z + cy
        vis = (z > 0.1) & (u >= 0) & (u < w) & (v >= 0) & (v < h)
        boxes = []
        for k, o in enumerate(objs):
            sel = np.arange(o["first"], o["first"] + o["n"])
            sv = sel[vis[sel]]
            if len(sv) < 0.6 * o["n"] or rng.random() > 0.9:
                continue
            core = sv[o["n"] // 20 <= sv - o["first"]]
            if len(core) < 3:
                continue
            x0, x1 = np.percentile(u[core], [1, 99])
            y0, y1 = np.percentile(v[core], [1, 99])
            j = rng.integers(-3, 4, 4)
            bx, by = int(max(0, x0 + j[0])), int(max(0, y0 + j[1]))
            bw, bh = int(min(w - 1, x1 + j[2]) - bx), int(min(h - 1, y1 + j[3]) - by)
            if bw > 4 and bh > 4:
                boxes.append([o["cls"], bx, by, bw, bh])
        order = rng.permutation(len(boxes))
        boxes = np.asarray([boxes[i] for i in order], np.int32).reshape(-1, 5)
        obs = np.nonzero(vis & (rng.random(len(P)) < obs_frac))[0]
        obs = obs[rng.permutation(len(obs))]
        uv = np.stack([u[obs], v[obs]], 1)
        uv = (np.round(uv * 10) / 10).astype(np.float32)
        frames.append(dict(T=T, boxes=boxes, ids=obs.astype(np.int32), pos=P[obs],
                           uv=uv, bad=np.zeros(len(obs), np.uint8), kf=(t % kf_every == kf_every - 1)))
        if lines:
            frames[-1]["lines"] = frame_lines(T, objs, lrng, K, w, h)
    return frames


def assoc_stream_fr3(n_frames=405, seed=0xEA1, lines=True):
    """The benchmark's association workload (BASELINE configs[1], SURVEY §8d input 2):
    EAO flag, so the frames carry line segments for the yaw sampling."""
    return assoc_stream(n_frames, seed=seed, classes=FR3_CLASSES, obs_frac=0.5, pts_range=(80, 400),
                        n_background=400, lines=lines)


# ----------------------------------------------------------------------------
# The reference's own fr3_long_office inputs (BASELINE configs[1] and [2], SURVEY §8d
# inputs 2-3): the real per-frame YOLO boxes of data/yolo_txts (scores parsed as 0, Q1)
# and the camera poses of data/groundtruth.txt, as committed in tests/golden/fr3_inputs.npz
# by tools/make_fr3_inputs.py.  The TUM images and the map the reference would build are
# not available, so the 3-D side is synthesised around the real detections: every box's
# centre ray is pushed to the depth its class size implies, same-class estimates are
# clustered into objects, and each object gets a seeded Gaussian point cloud (+5 %
# outliers, seed 0xEA1) of its class extent; background points fill the room.  The
# tracked map points of a frame are the visible points (GT pose), sub-sampled.
FR3_FIXTURE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                           "fr3_inputs.npz")
# COCO (darknet 0-based) class extents in metres (x, y, z = up) for the classes in yolo_txts
FR3_EXTENT = dict(CLASS_EXTENT)
FR3_EXTENT.update({15: (0.4, 0.2, 0.3), 44: (0.04, 0.15, 0.03), 45: (0.15, 0.15, 0.07), 60: (1.2, 0.8, 0.75),
                   63: (0.35, 0.25, 0.02), 65: (0.05, 0.18, 0.03), 67: (0.07, 0.02, 0.14), 69: (0.5, 0.5, 0.4),
                   75: (0.15, 0.15, 0.3), 76: (0.08, 0.18, 0.02)})


def fr3_inputs():
    d = np.load(FR3_FIXTURE)
    return {k: d[k] for k in d.files}


def tum_Tcw(p):
    """TUM pose row (tx ty tz qx qy qz qw, camera-to-world) -> Tcw (4x4 float32)."""
    x, y, z, w = p[3:7]
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                  [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                  [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    T = np.eye(4)
    T[:3, :3] = R.T
    T[:3, 3] = -R.T @ np.asarray(p[:3], np.float64)
    return T.astype(np.float32)


def fr3_world(start, n_frames, seed=0xEA1, K=TUM3_K, pts_range=(80, 400), n_background=1500, min_dets=10):
    """Objects (class, centre, extent, point cloud) clustered from the real boxes of frames
    [start, start + n_frames) and the background points; returns (objs, P, Tcw list)."""
    fx, fy, cx, cy = K
    d = fr3_inputs()
    boxes, off = d["boxes"].astype(np.float64), d["box_off"]
    Ts = [tum_Tcw(d["pose"][t]) for t in range(start, start + n_frames)]
    # per-detection 3-D centre estimates (vectorised), in frame order
    est, ecls = [], []
    for i, t in enumerate(range(start, start + n_frames)):
        b = boxes[off[t]:off[t + 1]]
        b = b[(b[:, 3] > 0) & (b[:, 4] > 0)]
        if not len(b):
            continue
        ext = np.asarray([FR3_EXTENT.get(int(c), (0.2, 0.2, 0.2)) for c in b[:, 0]])
        dep = np.clip(np.sqrt((fx * ext[:, :2].max(1) / b[:, 3]) * (fy * ext[:, 2] / b[:, 4])), 0.4, 5.0)
        ray = np.stack([(b[:, 1] + b[:, 3] / 2 - cx) / fx, (b[:, 2] + b[:, 4] / 2 - cy) / fy, np.ones(len(b))], 1)
        Rcw, tcw = Ts[i][:3, :3].astype(np.float64), Ts[i][:3, 3].astype(np.float64)
        est.append((ray * dep[:, None]) @ Rcw - (Rcw.T @ tcw)[None, :])
        ecls.append(b[:, 0].astype(np.int64))
    est, ecls = np.concatenate(est), np.concatenate(ecls)
    # greedy sequential clustering per class (running means), then merge close clusters
    centers = []
    for c in np.unique(ecls):
        X = est[ecls == c]
        r = max(0.4, float(max(FR3_EXTENT.get(int(c), (0.2, 0.2, 0.2)))))
        S = np.zeros((0, 3))
        N = np.zeros(0)
        for x in X:
            if len(N):
                dist = np.linalg.norm(S / N[:, None] - x, axis=1)
                j = int(np.argmin(dist))
                if dist[j] < r:
                    S[j] += x
                    N[j] += 1
                    continue
            S = np.vstack([S, x])
            N = np.append(N, 1.0)
        merged = True
        while merged and len(N) > 1:
            merged = False
            M = S / N[:, None]
            D = np.linalg.norm(M[:, None] - M[None], axis=2) + np.eye(len(N)) * 1e9
            a, b = np.unravel_index(int(np.argmin(D)), D.shape)
            if D[a, b] < r:
                S[a] += S[b]
                N[a] += N[b]
                S, N = np.delete(S, b, 0), np.delete(N, b)
                merged = True
        for s, k in zip(S, N):
            if k >= min_dets:
                centers.append((int(c), s / k))
    rng = np.random.Generator(np.random.PCG64(seed))
    objs, pos = [], []
    for c, center in centers:
        ext = np.asarray(FR3_EXTENT.get(c, (0.2, 0.2, 0.2)))
        n = int(rng.integers(*pts_range))
        p = np.clip(rng.normal(0, 1, (n, 3)) * (ext / 4), -ext / 2, ext / 2) + center
        n_out = max(1, n // 20)
        p[:n_out] = center + rng.uniform(-1, 1, (n_out, 3)) * (ext / 2 + 0.25)
        objs.append(dict(cls=c, center=center, ext=ext, first=len(pos), n=n))
        pos.extend(p.tolist())
    cs = np.asarray([o["center"] for o in objs])
    lo, hi = cs.min(0) - 1.0, cs.max(0) + 1.0
    pos.extend(rng.uniform(lo, hi, (n_background, 3)).tolist())
    return objs, np.asarray(pos, np.float32), Ts


def assoc_stream_fr3_real(start=None, n_frames=None, seed=0xEA1, K=TUM3_K, w=640, h=480, lines=True,
                          obs_frac=0.5, max_obs=1000, kf_every=5):
    """Replay inputs on the reference's fr3_long_office detections and GT poses.
    Defaults: the demo list (rgb_seq_pose.txt, 405 frames, BASELINE configs[1]);
    start=0, n_frames=2582 is the Full list (rgb_full_demo.txt, configs[2])."""
    fx, fy, cx, cy = K
    d = fr3_inputs()
    if start is None:
        start = int(d["demo_first"])
        n_frames = len(d["demo_timestamps"]) if n_frames is None else n_frames
    if n_frames is None:
        n_frames = len(d["timestamps"]) - start
    boxes, off = d["boxes"].astype(np.int32), d["box_off"]
    objs, P, Ts = fr3_world(start, n_frames, seed, K)
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    lrng = np.random.Generator(np.random.PCG64(0xEA2 + seed))
    frames = []
    for i, t in enumerate(range(start, start + n_frames)):
        T = Ts[i]
        Pc = P @ T[:3, :3].T.astype(np.float64) + T[:3, 3]
        z = Pc[:, 2]
        with np.errstate(divide="ignore", invalid="ignore"):
            u = fx * Pc[:, 0] / z + cx
            v = fy * Pc[:, 1] / z + cy
        vis = (z > 0.1) & (u >= 0) & (u < w) & (v >= 0) & (v < h)
        obs = np.nonzero(vis & (rng.random(len(P)) < obs_frac))[0]
        obs = obs[rng.permutation(len(obs))][:max_obs]
        uv = (np.round(np.stack([u[obs], v[obs]], 1) * 10) / 10).astype(np.float32)
        frames.append(dict(T=T, boxes=boxes[off[t]:off[t + 1]].reshape(-1, 5).copy(), ids=obs.astype(np.int32),
                           pos=P[obs], uv=uv, bad=np.zeros(len(obs), np.uint8), kf=(i % kf_every == kf_every - 1)))
        if lines:
            frames[-1]["lines"] = frame_lines_vec(T, objs, lrng, K, w, h)
    return frames


def with_point_updates(frames, seed=0xEA8, move_frac=0.3, sigma=0.004, cull_frac=0.01, replace_frac=0.01,
                       window=60):
    """LocalMapping's map-point changes on a replay stream (the trace of SURVEY appendix B plus a
    per-frame point record, eao_replay_update_points). At every keyframe, among the points seen
    in the last `window` frames (so most are held by objects but not observed by this frame):
      * LocalBundleAdjustment moves `move_frac` of them by N(0, sigma) m (SetWorldPos);
      * MapPointCulling / KeyFrameCulling retire `cull_frac` (SetBadFlag): never tracked again;
      * SearchInNeighbors replaces `replace_frac` (Replace: the old point turns bad, later
        observations of it report a fresh id at its position).
    Later frames observe the points' current state. Returns new frame dicts carrying
    upd_ids / upd_pos / upd_bad (empty on non-keyframes)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    cur, seen, repl, culled = {}, {}, {}, set()
    next_id = 1 + max(int(f["ids"].max()) for f in frames if len(f["ids"]))
    out = []
    for t, f in enumerate(frames):
        ids, pos, uv = [], [], []
        for k, i in enumerate(f["ids"].tolist()):
            while i in repl:
                i = repl[i]
            if i in culled:
                continue
            if i not in cur:
                cur[i] = np.asarray(f["pos"][k], np.float32)
            seen[i] = t
            ids.append(i)
            pos.append(cur[i])
            uv.append(f["uv"][k])
        g = dict(f, ids=np.asarray(ids, np.int32), pos=np.asarray(pos, np.float32).reshape(-1, 3),
                 uv=np.asarray(uv, np.float32).reshape(-1, 2), bad=np.zeros(len(ids), np.uint8))
        uid, upos, ubad = [], [], []
        if f["kf"]:
            cand = sorted(i for i, s in seen.items() if s >= t - window and i not in culled and i not in repl)
            r = rng.random((len(cand), 3))
            for i, (rm, rc, rr) in zip(cand, r):
                if rc < cull_frac:
                    culled.add(i)
                    uid.append(i), upos.append(cur[i]), ubad.append(1)
                elif rr < replace_frac:
                    repl[i] = next_id
                    cur[next_id] = cur[i] + rng.normal(0, sigma / 4, 3).astype(np.float32)
                    next_id += 1
                    uid.append(i), upos.append(cur[i]), ubad.append(1)
                elif rm < move_frac:
                    cur[i] = (cur[i] + rng.normal(0, sigma, 3)).astype(np.float32)
                    uid.append(i), upos.append(cur[i]), ubad.append(0)
        g["upd_ids"] = np.asarray(uid, np.int32)
        g["upd_pos"] = np.asarray(upos, np.float32).reshape(-1, 3)
        g["upd_bad"] = np.asarray(ubad, np.uint8)
        out.append(g)
    return out


# SURVEY.md §8d input 4 (Config C): 64 objects x 2000 map points, 16 classes,
# 8 detections per frame each observing m in [50, 300] points of one object
CONFIG_C_CLASSES = [39, 41, 62, 66, 73, 24, 26, 28, 45, 46, 47, 58, 59, 60, 61, 72]


def config_c_scene(seed=0xEA3, n_obj=64, n_pts=2000, spacing=1.5):
    rng = np.random.Generator(np.random.PCG64(seed))
    g = int(np.ceil(np.sqrt(n_obj)))
    objs, pos = [], []
    for k in range(n_obj):
        sd = rng.uniform(0.02, 0.2, 3)
        center = np.array([(k % g) * spacing, (k // g) * spacing, 2 * sd[2]])
        p = rng.normal(0, 1, (n_pts, 3)) * sd + center
        n_out = n_pts // 20
        p[:n_out] = center + rng.uniform(-1, 1, (n_out, 3)) * (2 * sd + 0.5)
        objs.append(dict(cls=CONFIG_C_CLASSES[k % len(CONFIG_C_CLASSES)], center=center, first=len(pos), n=n_pts))
        pos.extend(p.tolist())
    ext = (g - 1) * spacing
    bg = rng.uniform([-1.0, -1.0, 0.0], [ext + 1.0, ext + 1.0, 1.5], (800, 3))
    pos.extend(bg.tolist())
    return objs, np.asarray(pos, np.float32), ext


def assoc_stream_config_c(n_frames=1000, seed=0xEA3, K=TUM3_K, w=640, h=480, n_det=8, m_range=(50, 300),
                          kf_every=5):
    """Per-frame replay inputs of Config C: the camera sweeps the 8x8 object grid
    (serpentine), the n_det objects with the most visible points are detected,
    and each detection observes a random m in m_range of its visible points."""
    fx, fy, cx, cy = K
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    objs, P, ext = config_c_scene(seed)
    frames = []
    for t in range(n_frames):
        s = t / max(1, n_frames - 1)
        row = s * 3.0  # three serpentine passes over the grid
        y = (np.floor(row) + 0.5) * ext / 3.0
        x = (row % 1.0) if int(row) % 2 == 0 else 1.0 - (row % 1.0)
        target = np.array([x * ext, y, 0.0])
        eye = target + np.array([-0.3, -2.2, 3.0])
        T = _look_at(eye, target)
        Pc = P @ T[:3, :3].T.astype(np.float64) + T[:3, 3]
        z = Pc[:, 2]
        u = fx * Pc[:, 0] / z + cx
        v = fy * Pc[:, 1] / z + cy
        vis = (z > 0.1) & (u >= 0) & (u < w) & (v >= 0) & (v < h)
        cand = []
        for k, o in enumerate(objs):
            nv = int(vis[o["first"]:o["first"] + o["n"]].sum())
            if nv >= 0.6 * o["n"]:
                cand.append((-nv, k))
        chosen = [k for _, k in sorted(cand)[:n_det]]
        boxes, obs = [], []
        for k in chosen:
            o = objs[k]
            sel = np.arange(o["first"], o["first"] + o["n"])
            sv = sel[vis[sel]]
            core = sv[sv - o["first"] >= o["n"] // 20]
            x0, x1 = np.percentile(u[core], [1, 99])
            y0, y1 = np.percentile(v[core], [1, 99])
            j = rng.integers(-3, 4, 4)
            bx, by = int(max(0, x0 + j[0])), int(max(0, y0 + j[1]))
            bw, bh = int(min(w - 1, x1 + j[2]) - bx), int(min(h - 1, y1 + j[3]) - by)
            if bw > 4 and bh > 4:
                boxes.append([o["cls"], bx, by, bw, bh])
                m = int(rng.integers(m_range[0], m_range[1] + 1))
                obs.append(rng.choice(sv, size=min(m, len(sv)), replace=False))
        bg = np.arange(objs[-1]["first"] + objs[-1]["n"], len(P))
        bgv = bg[vis[bg] & (rng.random(len(bg)) < 0.5)]
        obs = np.concatenate(obs + [bgv]) if obs else bgv
        obs = obs[rng.permutation(len(obs))]
        order = rng.permutation(len(boxes))
        boxes = np.asarray([boxes[i] for i in order], np.int32).reshape(-1, 5)
        uv = (np.round(np.stack([u[obs], v[obs]], 1) * 10) / 10).astype(np.float32)
        frames.append(dict(T=T, boxes=boxes, ids=obs.astype(np.int32), pos=P[obs], uv=uv,
                           bad=np.zeros(len(obs), np.uint8), kf=(t % kf_every == kf_every - 1)))
    return frames


def line_frames(n, w=640, h=480, seed=0xEA7, n_quads=(6, 12)):
    """Line-rich gray frames for the line detector: a smooth shaded
    background with mild noise and several solid convex quadrilaterals / thin bars at random
    angles (the straight object and structure edges EDLine is built for). uint8 [n][h][w]."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    out = np.zeros((n, h, w), np.uint8)
    for f in range(n):
        img = 90 + 40 * np.sin(xx / 97.0 + f * 0.05) * np.cos(yy / 131.0) + rng.normal(0, 2.0, (h, w))
        for _ in range(int(rng.integers(*n_quads))):
            cx, cy = rng.uniform(40, w - 40), rng.uniform(40, h - 40)
            a = rng.uniform(0, np.pi)
            if rng.random() < 0.25:  # a thin bar
                hw, hh = rng.uniform(60, 220), rng.uniform(2, 5)
            else:
                hw, hh = rng.uniform(30, 160), rng.uniform(25, 120)
            c, s = np.cos(a), np.sin(a)
            u = (xx - cx) * c + (yy - cy) * s
            v = -(xx - cx) * s + (yy - cy) * c
            m = (np.abs(u) <= hw) & (np.abs(v) <= hh)
            img[m] = rng.uniform(20, 235) + rng.normal(0, 1.5, int(m.sum()))
        out[f] = np.clip(np.rint(img), 0, 255).astype(np.uint8)
    return out


def rodrigues(w):
    """rotation matrix of the axis-angle vector w (float64)."""
    th = float(np.linalg.norm(w))
    if th < 1e-12:
        return np.eye(3)
    k = np.asarray(w, np.float64) / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * (K @ K)


def pose_problem(seed, n=1000, frac_mp=0.7, frac_out=0.1, noise_px=1.0, rot_err=0.02, t_err=0.05,
                 K=TUM3_K, w=640, h=480, nlevels=8, scale=1.2):
    """A PoseOptimization input like TrackWithMotionModel's: n keypoints (mvKeysUn) of which
    frac_mp hold a map point seen at the true pose (level-scaled pixel noise, frac_out gross
    outliers), and the motion-model prior Tcw = true pose perturbed. Returns
    (Tcw_prior [4][4] f32, kps structured (x, y, size, angle, response, octave, class_id),
    has_mp u8[n], mp_pos f32[n][3], inv_level_sigma2 f32[nlevels], Tcw_true)."""
    fx, fy, cx, cy = K
    rng = np.random.default_rng(seed)
    Rt = rodrigues(rng.normal(0, 0.3, 3))
    tt = rng.normal(0, 0.5, 3)
    oct_ = rng.integers(0, nlevels, n).astype(np.int32)
    sc = scale ** oct_.astype(np.float64)
    u = rng.uniform(0, w, n)
    v = rng.uniform(0, h, n)
    z = rng.uniform(0.8, 6.0, n)
    Xc = np.stack([(u - cx) / fx * z, (v - cy) / fy * z, z], 1)
    Xw = (Xc - tt) @ Rt  # R^T (Xc - t)
    obs_u = u + rng.normal(0, noise_px, n) * sc
    obs_v = v + rng.normal(0, noise_px, n) * sc
    bad = rng.random(n) < frac_out
    obs_u[bad] = rng.uniform(0, w, bad.sum())
    obs_v[bad] = rng.uniform(0, h, bad.sum())
    kps = np.zeros(n, dtype=[("x", "f4"), ("y", "f4"), ("size", "f4"), ("angle", "f4"), ("response", "f4"),
                             ("octave", "i4"), ("class_id", "i4")])
    kps["x"], kps["y"], kps["size"] = obs_u, obs_v, 31 * sc
    kps["octave"], kps["class_id"] = oct_, -1
    has = (rng.random(n) < frac_mp).astype(np.uint8)
    Ttrue = np.eye(4)
    Ttrue[:3, :3], Ttrue[:3, 3] = Rt, tt
    Tp = np.eye(4)
    Tp[:3, :3] = rodrigues(rng.normal(0, rot_err, 3)) @ Rt
    Tp[:3, 3] = tt + rng.normal(0, t_err, 3)
    inv = (1.0 / (scale ** (2 * np.arange(nlevels)))).astype(np.float32)
    return Tp.astype(np.float32), kps, has, Xw.astype(np.float32), inv, Ttrue.astype(np.float32)


def _flip_bits(rows, nflip, rng):
    """flip nflip random bit positions (drawn with replacement) of each 32-byte row, in place."""
    m = len(rows)
    pos = rng.integers(0, 256, (m, nflip))
    r = np.repeat(np.arange(m), nflip)
    np.bitwise_xor.at(rows, (r, (pos >> 3).ravel()), (1 << (pos & 7)).astype(np.uint8).ravel())
    return rows


def vocabulary(K=10, L=4, seed=0xB0, stop_frac=0.02, flips=(48, 24, 12, 6, 4, 3)):
    """A synthetic DBoW2 ORB vocabulary (the reference's Vocabulary/ORBvoc.bin is a missing
    blob): a complete K-ary tree of depth L with node ids in breadth-first order (as
    loadFromTextFile numbers a saveToTextFile vocabulary), child descriptors = the parent's
    with flips[level] random bits flipped, leaves = words (ids in node order) with TF-IDF
    weights in (0.5, 5), stop_frac of them stopped (weight 0)."""
    rng = np.random.default_rng(seed)
    descs = [rng.integers(0, 256, (1, 32), dtype=np.uint8)]
    parents = [np.array([-1], np.int32)]
    levels = [np.zeros(1, np.int32)]
    first = 0
    for l in range(1, L + 1):
        prev = descs[-1]
        par = np.repeat(np.arange(first, first + len(prev), dtype=np.int32), K)
        d = np.repeat(prev, K, axis=0)
        _flip_bits(d, flips[min(l - 1, len(flips) - 1)], rng)
        first += len(prev)
        descs.append(d)
        parents.append(par)
        levels.append(np.full(len(d), l, np.int32))
    desc = np.concatenate(descs)
    parent = np.concatenate(parents)
    level = np.concatenate(levels)
    n = len(desc)
    word = np.full(n, -1, np.int32)
    leaves = np.nonzero(level == L)[0]
    word[leaves] = np.arange(len(leaves), dtype=np.int32)
    weight = np.zeros(n, np.float64)
    weight[leaves] = rng.uniform(0.5, 5.0, len(leaves))
    weight[leaves[rng.random(len(leaves)) < stop_frac]] = 0.0
    return {"desc": desc, "parent": parent, "word": word, "weight": weight, "L": L, "K": K, "leaves": leaves}


def bow_features(voc, n, seed=0, flips=6):
    """n ORB descriptors scattered around random vocabulary leaves (flips random bits each)."""
    rng = np.random.default_rng(seed)
    d = voc["desc"][rng.choice(voc["leaves"], n)].copy()
    return _flip_bits(d, flips, rng)


def bow_pair(voc, n_kf=1000, n_f=1000, seed=0, overlap=0.7, valid=0.8):
    """A keyframe and a frame observing partly the same features: -> (kf_kps, kf_desc, kf_valid,
    f_kps, f_desc); frame features are re-observations (a few extra bits flipped, the angle
    rotated by a common in-plane rotation plus noise) of `overlap` of the keyframe's."""
    rng = np.random.default_rng(seed)
    kd = bow_features(voc, n_kf, seed)
    dt = [("x", "f4"), ("y", "f4"), ("size", "f4"), ("angle", "f4"), ("response", "f4"), ("octave", "i4"),
          ("class_id", "i4")]
    kk = np.zeros(n_kf, dt)
    kk["x"], kk["y"] = rng.uniform(0, 640, n_kf), rng.uniform(0, 480, n_kf)
    kk["angle"] = rng.uniform(0, 360, n_kf)
    kk["octave"], kk["class_id"] = rng.integers(0, 8, n_kf), -1
    fd = bow_features(voc, n_f, seed + 7919)
    fk = np.zeros(n_f, dt)
    fk["x"], fk["y"] = rng.uniform(0, 640, n_f), rng.uniform(0, 480, n_f)
    fk["angle"] = rng.uniform(0, 360, n_f)
    fk["octave"], fk["class_id"] = rng.integers(0, 8, n_f), -1
    m = int(min(n_kf, n_f) * overlap)
    src = rng.permutation(n_kf)[:m]
    dst = rng.permutation(n_f)[:m]
    fd[dst] = _flip_bits(kd[src].copy(), 8, rng)
    rot = rng.uniform(0, 360)
    fk["angle"][dst] = np.mod(kk["angle"][src] - rot + rng.normal(0, 4, m), 360).astype(np.float32)
    kv = (rng.random(n_kf) < valid).astype(np.uint8)
    return kk, kd, kv, fk, fd
