"""CPU checks of the fr3_long_office fixtures (tools/make_fr3_inputs.py, make_fr3_golden.py).

* fr3_inputs.npz holds what the reference's readers produce from its data files: 2582 frames
  of the Full list (mono_tum.cc LoadImages skips 6 lines), the 405-frame demo list as a slice
  of it, the YOLO rows of every frame with the score parsed as the int 0 (Tracking.cc:435-466,
  SURVEY Q1), and the GT row the timestamp lookup of Tracking.cc:508-554 selects.
* The oracle reproduces the committed replay outputs on a prefix of the demo stream (the whole
  streams are replayed against the engine by tests/test_gpu_fr3.py)."""
import os

import numpy as np

import pyoracle as orc
from tools import synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_fr3_inputs_shape():
    d = synth.fr3_inputs()
    assert len(d["timestamps"]) == 2582 and len(d["demo_timestamps"]) == 405
    f = int(d["demo_first"])
    assert np.array_equal(d["timestamps"][f:f + 405], d["demo_timestamps"])
    off, boxes = d["box_off"], d["boxes"]
    assert off[0] == 0 and off[-1] == len(boxes) == 17204 and np.diff(off).max() <= 15
    # classes are COCO indices; boxes are integer pixel rectangles
    assert boxes[:, 0].min() >= 0 and boxes[:, 0].max() < 80 and (boxes[:, 3:] > 0).all()
    # every frame has a pose; rows found by the reference's lookup are GT rows verbatim
    ok = np.isfinite(d["gt"][:, 0])
    assert ok.sum() == 2171 and np.array_equal(d["pose"][ok], d["gt"][ok])
    assert np.allclose(np.linalg.norm(d["pose"][:, 3:], axis=1), 1.0, atol=1e-3)


def test_tum_pose_convention():
    # identity rotation: Tcw = [I | -t]
    T = synth.tum_Tcw(np.array([1.0, 2.0, 3.0, 0, 0, 0, 1.0]))
    assert np.allclose(T[:3, :3], np.eye(3)) and np.allclose(T[:3, 3], [-1, -2, -3])
    # 90 degrees about z (camera-to-world): a world point on +y is on the camera's +x... inverse
    s = np.sqrt(0.5)
    T = synth.tum_Tcw(np.array([0, 0, 0, 0, 0, s, s]))
    assert np.allclose(T[:3, :3] @ np.array([0, 1.0, 0]), [1, 0, 0], atol=1e-6)


def test_oracle_reproduces_demo_prefix():
    g = np.load(os.path.join(GOLDEN, "replay_fr3_demo_eao.npz"))
    frames = synth.assoc_stream_fr3_real()[:120]
    r = orc.Replay("EAO")
    outs = []
    for t, f in enumerate(frames):
        outs.append(r.frame(t + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"], lines=f.get("lines")))
        if f["kf"]:
            r.local_mapping()
    det = np.concatenate(outs)
    assert np.array_equal(det, g["det_out"][:len(det)])
