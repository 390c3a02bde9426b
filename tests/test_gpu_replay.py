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


def _run_steps(flag, frames, start=1):
    """frame + map-point record + local mapping per frame, engine vs oracle (step())."""
    g = ea.Replay(ea.Assoc(), flag)
    o = orc.Replay(flag)
    for i, f in enumerate(frames):
        og, oo = g.step(i + start, f), o.step(i + start, f)
        assert np.array_equal(og, oo), "frame %d: %s vs %s" % (i, og.tolist(), oo.tolist())
    gi, gf, gp = g.objects()
    oi, of, op = o.objects()
    assert np.array_equal(gi, oi)
    assert np.allclose(gf, of, rtol=1e-5, atol=1e-5, equal_nan=True)
    assert all(np.array_equal(a_, b_) for a_, b_ in zip(gp, op))
    return g, oi


def test_replay_point_updates_fr3_eao_405():
    """The drop-in boundary's LocalMapping channel: on the fr3 demo stream (real boxes, EAO),
    every keyframe moves (LocalBA), culls and replaces points the objects hold, most of them
    not observed by that frame (eao_replay_update_points); ids, statistics and point sets
    identical to the oracle."""
    frames = synth.with_point_updates(synth.assoc_stream_fr3_real())
    held_unobserved = 0
    g = ea.Replay(ea.Assoc(), "EAO")
    o = orc.Replay("EAO")
    for i, f in enumerate(frames):
        if len(f["upd_ids"]):
            held = set(g.held_points().tolist())
            held_unobserved += len((set(f["upd_ids"].tolist()) & held) - set(f["ids"].tolist()))
        og, oo = g.step(i + 1, f), o.step(i + 1, f)
        assert np.array_equal(og, oo), "frame %d: %s vs %s" % (i, og.tolist(), oo.tolist())
    assert held_unobserved > 1000
    gi, gf, gp = g.objects()
    oi, of, op = o.objects()
    assert np.array_equal(gi, oi)
    assert np.allclose(gf, of, rtol=1e-5, atol=1e-5, equal_nan=True)
    assert all(np.array_equal(a_, b_) for a_, b_ in zip(gp, op))


def test_replay_point_updates_fr3_full_slice():
    """Full flag (iForest + lines + yaw + LocalMapping merges) over the first 600 frames of the
    Full list with the per-keyframe point records."""
    _run_steps("Full", synth.with_point_updates(synth.assoc_stream_fr3_real(0, 600), seed=0xEA9))


def test_replay_run_updates_packed():
    """eao_replay_run_updates: the recorded stream with its point records in one call."""
    frames = synth.with_point_updates(synth.assoc_stream_fr3_real()[:200], seed=7)
    g = ea.Replay(ea.Assoc(), "EAO")
    det = g.run(ea.Replay.pack(frames))
    o = orc.Replay("EAO")
    ref = np.concatenate([o.step(i + 1, f) for i, f in enumerate(frames)])
    assert np.array_equal(det, ref)
    gi, gf, _ = g.objects()
    oi, of, _ = o.objects()
    assert np.array_equal(gi, oi) and np.allclose(gf, of, rtol=1e-5, atol=1e-5, equal_nan=True)


def test_replay_none_flag_fr3_405():
    """BASELINE configs[0]'s flag (None: no iForest, no yaw) on the fr3 demo stream."""
    _run_steps("None", synth.assoc_stream_fr3_real())


@pytest.mark.parametrize("flag", ["EAO", "Full"])
def test_replay_split_frames_fr3(flag):
    """eao_replay_frame_begin / _end on the engine (HSA lanes), the lines staged between the calls as
    the drop-in's overlapped pass does: every frame's rows and the objects equal the oracle's."""
    frames = synth.assoc_stream_fr3_real()[:200]
    a = ea.Assoc()
    rp = ea.Replay(a, flag)
    o = orc.Replay(flag)
    for i, f in enumerate(frames):
        rp.frame_begin(i + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"])
        det = rp.frame_end(lines=f.get("lines"))
        ref = o.frame(i + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"], lines=f.get("lines"))
        assert np.array_equal(det, ref), i
        if f["kf"]:
            rp.local_mapping()
            o.local_mapping()
    gi, gf, gp = rp.objects()
    oi, of, op = o.objects()
    assert np.array_equal(gi, oi) and np.allclose(gf, of, rtol=1e-5, atol=1e-5, equal_nan=True)
    assert all(np.array_equal(x, y) for x, y in zip(gp, op))
    rp.close()
