"""Association replay parity: engine (GPU NP / iForest / rects + host decisions)
vs the CPU restatement of Object.cc / Tracking.cc / LocalMapping.cc.

Outcomes and associated object ids per detection must be identical every
frame; final object point sets identical; object statistics within 1e-5."""
import numpy as np
import pytest

import eao_accel as ea
import pyoracle as orc
from tools import synth

pytestmark = pytest.mark.gpu


def _run(flag, frames, start=1):
    a = ea.Assoc()
    g = ea.Replay(a, flag)
    o = orc.Replay(flag)
    for i, f in enumerate(frames):
        og = g.frame(i + start, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"], lines=f.get("lines"))
        oo = o.frame(i + start, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"], lines=f.get("lines"))
        assert np.array_equal(og, oo), "frame %d: %s vs %s" % (i, og.tolist(), oo.tolist())
        if f["kf"]:
            g.local_mapping()
            o.local_mapping()
    gi, gf, gp = g.objects()
    oi, of, op = o.objects()
    assert np.array_equal(gi, oi)
    assert np.allclose(gf, of, rtol=1e-5, atol=1e-5, equal_nan=True)
    for a_, b_ in zip(gp, op):
        assert np.array_equal(a_, b_)
    return oi


@pytest.mark.parametrize("flag,lines", [("iForest", False), ("None", False), ("NP", False), ("IoU", False),
                                        ("NA", False), ("EAO", False), ("EAO", True), ("Full", True)])
def test_replay_flags(flag, lines):
    frames = synth.assoc_stream(80, lines=lines)
    ints = _run(flag, frames)
    assert len(ints) > 5


def test_replay_long_bad_points():
    frames = synth.assoc_stream(200, seed=0xEA2)
    rng = np.random.default_rng(3)
    for f in frames:
        f["bad"] = (rng.random(len(f["ids"])) < 0.01).astype(np.uint8)
    _run("iForest", frames, start=40)


def test_replay_bench_stream_full():
    """The benchmark's 405-frame fr3-shaped stream (with line segments), EAO flag, end to end."""
    _run("EAO", synth.assoc_stream_fr3(405))


def test_replay_run_stream_matches_per_frame_oracle():
    """eao_replay_run (packed stream, one call) == the oracle frame by frame."""
    frames = synth.assoc_stream_fr3(120, seed=0xEA5)
    a = ea.Assoc()
    g = ea.Replay(a, "EAO")
    det = g.run(ea.Replay.pack(frames))
    o = orc.Replay("EAO")
    ref = []
    for i, f in enumerate(frames):
        ref.append(o.frame(i + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"], lines=f.get("lines")))
        if f["kf"]:
            o.local_mapping()
    assert np.array_equal(det, np.concatenate(ref))
    gi, gf, gp = g.objects()
    oi, of, op = o.objects()
    assert np.array_equal(gi, oi)
    assert np.allclose(gf, of, rtol=1e-5, atol=1e-5, equal_nan=True)
