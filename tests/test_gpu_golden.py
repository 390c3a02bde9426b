"""The engine against the committed regression fixtures (tests/golden/):
bit-exact keypoints / descriptors / match ids / NP verdicts and counts /
association outcomes, iForest scores and object statistics within 1e-5."""
import os

import numpy as np
import pytest

import eao_accel as ea
from tools import synth

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


def test_orb_and_motion_match_golden():
    g = load("orb_match.npz")
    frames, poses = synth.frame_stream(2)
    orb = ea.Orb()
    k0, d0 = orb.extract(frames[0])
    k1, d1 = orb.extract(frames[1])
    assert np.array_equal(k0.view(np.uint8), g["kps0"]) and np.array_equal(d0, g["desc0"])
    assert np.array_equal(k1.view(np.uint8), g["kps1"]) and np.array_equal(d1, g["desc1"])
    pos = synth.backproject(poses[0], k0["x"], k0["y"])
    n, m = ea.Matcher().motion(ea.camera(), poses[1], 15, 1, k0, np.ones(len(k0), np.uint8), pos, d0, k1, d1,
                               orb.scale_tables()[0])
    assert n == int(g["nmatch01"]) and np.array_equal(m, g["match01"])


def test_iforest_golden():
    g = load("iforest.npz")
    clouds = [g["cloud%d" % i] for i in range(3)]
    got = ea.Assoc().iforest(clouds)
    for i in range(3):
        assert np.allclose(got[i], g["score%d" % i], rtol=1e-5, atol=1e-5)


def test_np_golden():
    g = load("np_pairs.npz")
    stats = g["stats"].view(ea.NP_DTYPE)
    n = len(stats)
    got = ea.Assoc().np_batch([(g["f%d" % i], g["fv%d" % i]) for i in range(n)],
                              [(g["o%d" % i], g["ov%d" % i]) for i in range(n)])
    assert np.array_equal(got["verdict"], stats["verdict"])
    for f in ("cnt_gt", "cnt_lt", "cnt_eq"):
        assert np.array_equal(got[f], stats[f])
    assert np.allclose(got["w"], stats["w"], rtol=1e-5)


@pytest.mark.parametrize("name,lines", [("replay_eao60.npz", False), ("replay_eao_lines60.npz", True)])
def test_replay_golden(name, lines):
    g = load(name)
    fr = synth.assoc_stream(60, lines=lines)
    a = ea.Assoc()
    r = ea.Replay(a, "EAO")
    outs = []
    for t, f in enumerate(fr):
        outs.append(r.frame(t + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"], lines=f.get("lines")))
        if f["kf"]:
            r.local_mapping()
    assert np.array_equal(np.concatenate(outs), g["det_out"])
    ints, fl, pts = r.objects()
    assert np.array_equal(ints, g["obj_ints"])
    assert np.allclose(fl, g["obj_floats"], rtol=1e-5, atol=1e-5, equal_nan=True)
    assert np.array_equal(np.concatenate(pts), g["obj_points"])
