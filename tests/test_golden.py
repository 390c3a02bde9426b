"""The oracle reproduces the committed regression fixtures (tests/golden/,
made by tools/make_golden.py from the synthetic inputs of tools/synth.py).
CPU test: guards the parity target against drift of the restatement."""
import os

import numpy as np
import pytest

import pyoracle as orc
from tools import synth

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


def test_orb_and_motion_match_fixture():
    g = load("orb_match.npz")
    frames, poses = synth.frame_stream(2)
    k0, d0 = orc.extract(frames[0])
    assert np.array_equal(k0.view(np.uint8), g["kps0"]) and np.array_equal(d0, g["desc0"])
    k1, d1 = orc.extract(frames[1])
    assert np.array_equal(k1.view(np.uint8), g["kps1"]) and np.array_equal(d1, g["desc1"])
    pos = synth.backproject(poses[0], k0["x"], k0["y"])
    n, m = orc.match_motion(orc.cam(), poses[1], 15, 1, k0, np.ones(len(k0), np.uint8), pos, d0, k1, d1,
                            orc.orb_params()["scale"])
    assert n == int(g["nmatch01"]) and np.array_equal(m, g["match01"])


def test_iforest_fixture():
    g = load("iforest.npz")
    for i in range(3):
        assert np.array_equal(orc.iforest(g["cloud%d" % i]), g["score%d" % i])


def test_np_fixture():
    g = load("np_pairs.npz")
    stats = g["stats"].view(orc.NP_DTYPE)
    for i in range(len(stats)):
        r = orc.np_test(g["f%d" % i], g["fv%d" % i], g["o%d" % i], g["ov%d" % i])
        assert r.tobytes() == stats[i].tobytes()
    assert set(stats["verdict"].tolist()) >= {1, 2}


@pytest.mark.parametrize("name,lines", [("replay_eao60.npz", False), ("replay_eao_lines60.npz", True)])
def test_replay_fixture(name, lines):
    g = load(name)
    fr = synth.assoc_stream(60, lines=lines)
    r = orc.Replay("EAO")
    outs = []
    for t, f in enumerate(fr):
        outs.append(r.frame(t + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"], lines=f.get("lines")))
        if f["kf"]:
            r.local_mapping()
    assert np.array_equal(np.concatenate(outs), g["det_out"])
    ints, fl, pts = r.objects()
    assert np.array_equal(ints, g["obj_ints"]) and np.array_equal(fl, g["obj_floats"])
    assert np.array_equal(np.concatenate(pts), g["obj_points"])
    if lines:  # the yaw sampling ran and moved some objects off yaw 0
        alive = ints[:, 2] == 0
        assert (fl[:, 17] > 0).any() and (fl[alive, 16] != 0).any()
