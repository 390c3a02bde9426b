"""One frame stream chained through the hot path, as Tracking chains it (development and test
infrastructure): frame t's ORB extraction -> SearchByProjection(motion) against frame t-1's
tracked map points (src/Tracking.cc:1266-1281) -> the matched keypoints carry their map points
into the object association of frame t (AssociateObjAndPoints reads mvpMapPoints and the
keypoints, src/Tracking.cc:2434-2468) with YOLO-like boxes projected from object regions of the
scene.

The scene is synth's textured plane Z = 2 m seen along synth.camera_path; a map point is created
by back-projecting a keypoint onto the plane (with a small deterministic relief so object clouds
are 3-D), at frame 0 and at every keyframe for the keypoints the motion search left unmatched;
objects are rectangles of the plane (classes of the fr3 detections). `run(backend, n)` drives one
backend -- the engine or the oracle, the same calls -- and returns every stage's outputs."""
import numpy as np

from tools import synth

KF_EVERY = 5
CLASSES = [39, 56, 73, 62, 41, 66, 64, 39]


def relief(p):
    """Map point positions: the plane point plus a deterministic relief along Z."""
    q = p.astype(np.float64).copy()
    q[:, 2] += 0.03 * np.sin(17.0 * q[:, 0]) * np.cos(13.0 * q[:, 1])
    return q.astype(np.float32)


def regions(poses):
    """Object rectangles [x0, y0, x1, y1] of the plane around the camera path's mean view."""
    twc = np.array([-(P[:3, :3].T.astype(np.float64) @ P[:3, 3].astype(np.float64)) for P in poses])
    cx, cy = twc[:, 0].mean(), twc[:, 1].mean()
    out = []
    for k in range(8):
        gx, gy = (k % 4) - 1.5, (k // 4) - 0.5
        w, h = 0.16 + 0.04 * (k % 3), 0.14 + 0.05 * (k % 2)
        x0, y0 = cx + 0.42 * gx - w / 2, cy + 0.55 * gy - h / 2
        out.append([x0, y0, x0 + w, y0 + h])
    return np.array(out)


def boxes_for(T, regs, rng, K=synth.TUM3_K, w=640, h=480, depth=2.0):
    fx, fy, cx, cy = K
    out = []
    for k, (x0, y0, x1, y1) in enumerate(regs):
        P = np.array([[x0, y0, depth], [x1, y0, depth], [x0, y1, depth], [x1, y1, depth]])
        Pc = P @ T[:3, :3].T.astype(np.float64) + T[:3, 3].astype(np.float64)
        u = fx * Pc[:, 0] / Pc[:, 2] + cx
        v = fy * Pc[:, 1] / Pc[:, 2] + cy
        j = rng.integers(-2, 3, 4)
        bx, by = int(max(0, u.min() + j[0])), int(max(0, v.min() + j[1]))
        bw, bh = int(min(w - 1, u.max() + j[2]) - bx), int(min(h - 1, v.max() + j[3]) - by)
        if bw > 8 and bh > 8 and u.min() > -20 and v.min() > -20 and u.max() < w + 20 and v.max() < h + 20:
            out.append([CLASSES[k], bx, by, bw, bh])
    return np.array(out, np.int32).reshape(-1, 5)


def run(backend, n, seed=0xEA0, step=0.004):
    """backend: extract(gray) -> (kps, desc); match(T, last_kps, has_mp, mp_pos, mp_desc, cur_kps,
    cur_desc) -> (n, cur_match); replay_frame(t, T, boxes, ids, pos, uv, bad) -> det rows;
    local_mapping(). Returns per-frame dicts of every stage's outputs."""
    frames, poses = synth.frame_stream(n, seed=seed, step=step)
    regs = regions(poses)
    rng = np.random.Generator(np.random.PCG64(seed + 99))
    out = []
    last = None
    next_id = 0
    for t in range(n):
        T = poses[t]
        kps, desc = backend.extract(frames[t])
        nk = len(kps)
        mp_id = np.full(nk, -1, np.int64)
        mp_pos = np.zeros((nk, 3), np.float32)
        nmatch, cm = 0, np.full(nk, -1, np.int32)
        if last is not None:
            lk, ld, lid, lpos = last
            nmatch, cm = backend.match(T, lk, (lid >= 0).astype(np.uint8), lpos, ld, kps, desc)
            ok = cm >= 0
            mp_id[ok] = lid[cm[ok]]
            mp_pos[ok] = lpos[cm[ok]]
        kf = t % KF_EVERY == 0
        if kf:  # new map points for the keypoints left without one
            new = mp_id < 0
            mp_id[new] = next_id + np.arange(new.sum())
            next_id += int(new.sum())
            mp_pos[new] = relief(synth.backproject(T, kps["x"][new], kps["y"][new]))
        has = mp_id >= 0
        boxes = boxes_for(T, regs, rng)
        uv = np.stack([kps["x"][has], kps["y"][has]], 1).astype(np.float32)
        ids = mp_id[has].astype(np.int32)
        pos = mp_pos[has]
        det = backend.replay_frame(t + 1, T, boxes, ids, pos, uv, np.zeros(len(ids), np.uint8))
        if kf:
            backend.local_mapping()
        out.append(dict(kps=kps, desc=desc, nmatch=nmatch, match=cm, ids=ids, boxes=boxes, det=det))
        last = (kps, desc, mp_id, mp_pos)
    return out


class EngineBackend:
    def __init__(self, ea, flag="EAO"):
        self.ea = ea
        self.orb, self.mt = ea.Orb(), ea.Matcher()
        self.cam = ea.camera()
        self.rp = ea.Replay(ea.Assoc(), flag)
        self.scales = self.orb.scale_tables()[0]  # mvScaleFactors, the engine's own table

    def extract(self, g):
        return self.orb.extract(g)

    def match(self, T, lk, has, pos, ld, kps, desc):
        return self.mt.motion(self.cam, T, 15, 1, lk, has, pos, ld, kps, desc, self.scales)

    def replay_frame(self, t, T, boxes, ids, pos, uv, bad):
        return self.rp.frame(t, T, boxes, ids, pos, uv, bad)

    def local_mapping(self):
        self.rp.local_mapping()


class OracleBackend:
    def __init__(self, orc, flag="EAO"):
        self.orc = orc
        self.cam = orc.cam()
        self.scales = orc.orb_params()["scale"]
        self.rp = orc.Replay(flag)

    def extract(self, g):
        return self.orc.extract(g)

    def match(self, T, lk, has, pos, ld, kps, desc):
        return self.orc.match_motion(self.cam, T, 15, 1, lk, has, pos, ld, kps, desc, self.scales)

    def replay_frame(self, t, T, boxes, ids, pos, uv, bad):
        return self.rp.frame(t, T, boxes, ids, pos, uv, bad)

    def local_mapping(self):
        self.rp.local_mapping()
