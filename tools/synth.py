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
import numpy as np

TUM3_K = (535.4, 539.2, 320.1, 247.6)  # Examples/Monocular/TUM3.yaml:8-11


def _smooth(a, passes=1):
    for _ in range(passes):
        a = (a + np.roll(a, 1, 0) + np.roll(a, -1, 0) + np.roll(a, 1, 1) + np.roll(a, -1, 1)) / 5.0
    return a


def texture(seed=0xEA0, size=2048):
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


def frame_stream(n, w=640, h=480, seed=0xEA0, step=0.004):
    tex = texture(seed, 2048 if max(w, h) <= 640 else 4096)
    poses = camera_path(n, seed, step)
    frames = np.stack([render(tex, poses[i], w, h) for i in range(n)])
    return frames, poses
