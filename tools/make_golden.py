"""Regenerate the committed regression fixtures under tests/golden/.

These vectors come from the oracle (oracle/, the CPU restatement) on the
deterministic synthetic inputs of tools/synth.py.  They freeze the parity
target: tests/test_golden.py checks the oracle still reproduces them (CPU) and
tests/test_gpu_golden.py checks the engine against them (GPU).  The
reference's own data file in this directory is t_test.txt (data/t_test.txt).

usage: python tools/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import pyoracle as orc  # noqa: E402
from tools import synth  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def clouds():
    rng = np.random.default_rng(0x60D)
    out = []
    for n in (30, 257, 1200):
        c = rng.normal([0.2, -0.1, 2.0], [0.05, 0.12, 0.04], (n, 3)).astype(np.float32)
        c[: n // 15] += rng.uniform(-0.6, 0.6, (n // 15, 3)).astype(np.float32)
        out.append(c)
    return out


def np_pairs():
    rng = np.random.default_rng(0x60E)
    pairs = []
    for k in range(12):
        m, n = int(rng.integers(15, 200)), int(rng.integers(15, 1500))
        c = rng.normal(0, 0.2, 3)
        f = (rng.normal(0, 0.05, (m, 3)) + c).astype(np.float32)
        o = (rng.normal(0, 0.05, (n, 3)) + c + (k % 3) * rng.normal(0, 0.05, 3)).astype(np.float32)
        pairs.append((f, (rng.random(m) > 0.05).astype(np.uint8), o, (rng.random(n) > 0.05).astype(np.uint8)))
    return pairs


def main():
    os.makedirs(OUT, exist_ok=True)
    frames, poses = synth.frame_stream(2)
    k0, d0 = orc.extract(frames[0])
    k1, d1 = orc.extract(frames[1])
    pos = synth.backproject(poses[0], k0["x"], k0["y"])
    has = np.ones(len(k0), np.uint8)
    sc = orc.orb_params()["scale"]
    nm, m01 = orc.match_motion(orc.cam(), poses[1], 15, 1, k0, has, pos, d0, k1, d1, sc)
    np.savez_compressed(os.path.join(OUT, "orb_match.npz"), kps0=k0.view(np.uint8), desc0=d0,
                        kps1=k1.view(np.uint8), desc1=d1, match01=m01, nmatch01=np.int32(nm))
    cs = clouds()
    np.savez_compressed(os.path.join(OUT, "iforest.npz"),
                        **{"cloud%d" % i: c for i, c in enumerate(cs)},
                        **{"score%d" % i: orc.iforest(c) for i, c in enumerate(cs)})
    pr = np_pairs()
    stats = np.stack([orc.np_test(*p) for p in pr])
    np.savez_compressed(os.path.join(OUT, "np_pairs.npz"),
                        **{"f%d" % i: p[0] for i, p in enumerate(pr)}, **{"fv%d" % i: p[1] for i, p in enumerate(pr)},
                        **{"o%d" % i: p[2] for i, p in enumerate(pr)}, **{"ov%d" % i: p[3] for i, p in enumerate(pr)},
                        stats=stats.view(np.uint8))
    for name, lines in (("replay_eao60.npz", False), ("replay_eao_lines60.npz", True)):
        # EAO flag over 60 frames; the second fixture adds each frame's line
        # segments (object-line association + yaw sampling, Tracking.cc:2472-2871)
        fr = synth.assoc_stream(60, lines=lines)
        r = orc.Replay("EAO")
        outs = []
        for t, f in enumerate(fr):
            outs.append(r.frame(t + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"],
                                lines=f.get("lines")))
            if f["kf"]:
                r.local_mapping()
        ints, fl, pts = r.objects()
        np.savez_compressed(os.path.join(OUT, name), det_out=np.concatenate(outs),
                            det_count=np.array([len(o) for o in outs], np.int32), obj_ints=ints, obj_floats=fl,
                            obj_points=np.concatenate(pts), obj_npoints=np.array([len(p) for p in pts], np.int32))
    for n in sorted(os.listdir(OUT)):
        print(n, os.path.getsize(os.path.join(OUT, n)))


if __name__ == "__main__":
    main()
