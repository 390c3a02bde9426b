"""CPU test of the engine's HOST association orchestration (replay.cpp).

tests/native/ compiles eao-slam_amd/csrc/replay.cpp with g++ against a
host-only HIP stand-in whose three GPU primitives (NP pair statistics,
isolation forest, projected rects) are served by the oracle. This checks the
sequential decision logic, deferred-forest bookkeeping and duplicate hashing
of the product without a device; the GPU kernels themselves are covered by the
-m gpu tests. Test infrastructure only."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

import eao_accel as ea
import pyoracle as orc
from tools import synth

NATIVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")


@pytest.fixture(scope="module")
def harness():
    orc.lib()
    subprocess.check_call(["make", "-s", "-C", NATIVE])
    # EAO_HARNESS_SO: a sanitizer build of the same harness (tests/test_replay_sanitizers.py)
    H = ctypes.CDLL(os.environ.get("EAO_HARNESS_SO") or os.path.join(NATIVE, "_build", "libreplay_host.so"))
    H.harness_assoc_create.restype = ctypes.c_void_p
    return H


class _HostReplay(ea.Replay):
    def __init__(self, H, flag):
        class A:
            pass
        a = A()
        a.h = ctypes.c_void_p(H.harness_assoc_create())
        saved = ea._lib
        ea._lib = H
        try:
            super().__init__(a, flag)
        finally:
            ea._lib = saved
        self.H = H

    def _with(self, fn, *args):
        saved = ea._lib
        ea._lib = self.H
        try:
            return fn(*args)
        finally:
            ea._lib = saved

    def frame(self, *a, **k):
        return self._with(lambda *x: super(_HostReplay, self).frame(*x, **k), *a)

    def local_mapping(self):
        return self._with(super().local_mapping)

    def objects(self):
        return self._with(super().objects)

    def step(self, *a):
        return self._with(super().step, *a)

    def update_points(self, *a):
        return self._with(super().update_points, *a)

    def held_points(self):
        return self._with(super().held_points)

    def close(self):
        if self.h:
            self.H.eao_replay_destroy(self.h)
            self.h = ctypes.c_void_p()

    __del__ = close


@pytest.mark.parametrize("flag,lines", [("iForest", False), ("None", False), ("NP", False), ("IoU", False),
                                        ("NA", False), ("EAO", True), ("Full", True), ("NP", True)])
def test_host_orchestration_matches_oracle(harness, flag, lines):
    frames = synth.assoc_stream(60, lines=lines)
    g = _HostReplay(harness, flag)
    o = orc.Replay(flag)
    for i, f in enumerate(frames):
        og = g.frame(i + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"], lines=f.get("lines"))
        oo = o.frame(i + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"], lines=f.get("lines"))
        assert np.array_equal(og, oo), (i, og.tolist(), oo.tolist())
        if f["kf"]:
            g.local_mapping()
            o.local_mapping()
    gi, gf, gp = g.objects()
    oi, of, op = o.objects()
    assert np.array_equal(gi, oi)
    assert np.allclose(gf, of, rtol=1e-5, atol=1e-5, equal_nan=True)
    assert all(np.array_equal(x, y) for x, y in zip(gp, op))


def test_host_run_stream_matches_oracle(harness):
    frames = synth.assoc_stream_fr3(50, seed=0xEA6)
    g = _HostReplay(harness, "EAO")
    det = g._with(ea.Replay.run, g, ea.Replay.pack(frames))
    o = orc.Replay("EAO")
    ref = []
    for i, f in enumerate(frames):
        ref.append(o.frame(i + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"], lines=f.get("lines")))
        if f["kf"]:
            o.local_mapping()
    assert np.array_equal(det, np.concatenate(ref))
    gi, gf, _ = g.objects()
    oi, of, _ = o.objects()
    assert np.array_equal(gi, oi) and np.allclose(gf, of, rtol=1e-5, atol=1e-5, equal_nan=True)


@pytest.mark.parametrize("flag", ["EAO", "Full"])
def test_host_fr3_real_stream_matches_oracle(harness, flag):
    """The reference's fr3 detections (tools/synth.assoc_stream_fr3_real): many same-class
    boxes per frame, so later detections meet objects whose forests are still pending
    (the held / deferred path of replay.cpp's associate) on every frame."""
    frames = synth.assoc_stream_fr3_real()[:150]
    g = _HostReplay(harness, flag)
    det = g._with(ea.Replay.run, g, ea.Replay.pack(frames))
    o = orc.Replay(flag)
    ref = []
    for i, f in enumerate(frames):
        ref.append(o.frame(i + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"], lines=f.get("lines")))
        if f["kf"]:
            o.local_mapping()
    assert np.array_equal(det, np.concatenate(ref))
    gi, gf, gp = g.objects()
    oi, of, op = o.objects()
    assert np.array_equal(gi, oi) and np.allclose(gf, of, rtol=1e-5, atol=1e-5, equal_nan=True)
    assert all(np.array_equal(x, y) for x, y in zip(gp, op))


def _compare(g, o):
    gi, gf, gp = g.objects()
    oi, of, op = o.objects()
    assert np.array_equal(gi, oi) and np.allclose(gf, of, rtol=1e-5, atol=1e-5, equal_nan=True)
    assert all(np.array_equal(x, y) for x, y in zip(gp, op))
    return oi, of


@pytest.mark.parametrize("flag", ["EAO", "Full"])
def test_host_point_updates_match_oracle(harness, flag):
    """LocalMapping's map-point record (eao_replay_update_points): at every keyframe points the
    objects hold -- most of them not observed by that frame -- move (LocalBA), are culled or
    replaced (bad); ids and statistics identical to the oracle, frame by frame."""
    frames = synth.with_point_updates(synth.assoc_stream_fr3_real()[:150])
    g = _HostReplay(harness, flag)
    o = orc.Replay(flag)
    held_unobserved = 0
    for i, f in enumerate(frames):
        if len(f["upd_ids"]):
            held = set(g.held_points().tolist())
            held_unobserved += len((set(f["upd_ids"].tolist()) & held) - set(f["ids"].tolist()))
        og, oo = g.step(i + 1, f), o.step(i + 1, f)
        assert np.array_equal(og, oo), (i, og.tolist(), oo.tolist())
    assert held_unobserved > 100  # the record reaches points no frame re-reported
    oi, of = _compare(g, o)
    # the record matters: without it the object statistics come out differently
    o2 = orc.Replay(flag)
    for i, f in enumerate(frames):
        o2.frame(i + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"], lines=f.get("lines"))
        if f["kf"]:
            o2.local_mapping()
    i2, f2, _ = o2.objects()
    assert not (np.array_equal(i2, oi) and np.allclose(f2, of, rtol=1e-6, atol=1e-7, equal_nan=True))


def test_host_run_updates_matches_oracle(harness):
    """eao_replay_run_updates (packed stream with the per-frame point records) == the oracle."""
    frames = synth.with_point_updates(synth.assoc_stream_fr3(60, seed=0xEA6), seed=5)
    g = _HostReplay(harness, "EAO")
    det = g._with(ea.Replay.run, g, ea.Replay.pack(frames))
    o = orc.Replay("EAO")
    ref = [o.step(i + 1, f) for i, f in enumerate(frames)]
    assert np.array_equal(det, np.concatenate(ref))
    _compare(g, o)


def test_host_two_threads_share_one_handle(harness):
    """The Tracking thread replays frames while a LocalMapping thread polls the handle
    (held_points, update_points with unchanged state, num_objects) with no ordering: the
    handle's lock keeps the containers whole and the outcome equals the serial oracle."""
    import threading
    frames = synth.assoc_stream_fr3_real()[:80]
    g = _HostReplay(harness, "EAO")
    stop = threading.Event()
    errors = []

    H = harness  # called directly: _HostReplay._with swaps a module global, not thread-safe

    def local_mapping_thread():
        try:
            buf = np.zeros(1 << 16, np.int32)
            while not stop.is_set():
                n = H.eao_replay_held_points(g.h, ea.P(buf), len(buf))
                assert n >= 0
                ids = buf[:min(n, 64)].copy()
                pos = np.zeros((len(ids), 3), np.float32)
                # an empty record, then a record of nothing the replay knows (ids < 0)
                assert H.eao_replay_update_points(g.h, 0, ea.P(ids), None, None) == 0
                neg = -1 - ids
                assert H.eao_replay_update_points(g.h, len(neg), ea.P(neg), ea.P(pos), None) == 0
                assert H.eao_replay_num_objects(g.h) >= 0
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = threading.Thread(target=local_mapping_thread)
    th.start()
    try:
        dets = [g.step(i + 1, f) for i, f in enumerate(frames)]
    finally:
        stop.set()
        th.join()
    assert not errors
    o = orc.Replay("EAO")
    ref = [o.step(i + 1, f) for i, f in enumerate(frames)]
    assert all(np.array_equal(a, b) for a, b in zip(dets, ref))
    _compare(g, o)


def test_host_outputs_complete_without_events(harness):
    """The unsharded waits end on the outputs themselves: with every event query reporting
    "not ready" (harness_set_events_never), the fr3 stream still completes -- each frame start
    and forest completion sees its sentinel-prefilled outputs overwritten (replay.cpp
    spin_ready) -- with the oracle's ids and statistics."""
    frames = synth.assoc_stream_fr3_real()[:120]
    harness.harness_set_events_never(1)
    try:
        g = _HostReplay(harness, "EAO")
        det = g._with(ea.Replay.run, g, ea.Replay.pack(frames))
        o = orc.Replay("EAO")
        ref = np.concatenate([o.step(i + 1, f) for i, f in enumerate(frames)])
        assert np.array_equal(det, ref)
        _compare(g, o)
    finally:
        harness.harness_set_events_never(0)


def _resume_after_failure(env):
    """Run the fr3 stream through eao_replay_run with the K-th forest launch failing (harness fault
    injection), then resume frame by frame with frames that do not continue the failed stream; in a
    fresh process (the switches are read at load). Returns the resumed frames' rows, the held map
    points and the object records."""
    import json
    import subprocess
    code = r'''
import ctypes, json, os, subprocess, sys
sys.path[:0] = sys.argv[1].split(os.pathsep)
import numpy as np
import eao_accel as ea
import test_replay_host as T
from tools import synth
subprocess.check_call(["make", "-s", "-C", T.NATIVE])
H = ctypes.CDLL(os.path.join(T.NATIVE, "_build", "libreplay_host.so"))
H.harness_assoc_create.restype = ctypes.c_void_p
frames = synth.assoc_stream_fr3_real()[:60]
g = T._HostReplay(H, "EAO")
try:
    g._with(ea.Replay.run, g, ea.Replay.pack(frames[:40]))
    failed = False
except Exception:
    failed = True
rows = [g.step(41 + i, f).tolist() for i, f in enumerate(frames[45:60])]  # not the stream's next frames
gi, gf, gp = g.objects()
print(json.dumps(dict(failed=failed, rows=rows, held=g._with(g.held_points).tolist(), ints=gi.tolist(),
                      floats=np.nan_to_num(gf).tolist(), pts=[p.tolist() for p in gp])))
'''
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    path = os.pathsep.join([here, root, os.path.join(root, "oracle"), os.path.join(root, "eao-slam_amd", "python")])
    out = subprocess.run([sys.executable, "-c", code, path], env=dict(os.environ, **env), capture_output=True,
                         text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_host_resume_after_failed_stream_with_other_frames(harness):
    """a stream call that fails after its wait ran the next frame's look-ahead discards
    that look-ahead -- the map points its step 1 created are erased and the staged line set its
    step 3 consumed is staged again -- so a caller resuming with other frames gets what a replay
    whose look-ahead never ran gets (EAO_LOOKAHEAD_EAGER=1 runs every wait's look-ahead to the end on
    the harness, whose kernels finish at launch; EAO_HARNESS_FAIL_IFOREST fails the 40th forest
    launch, inside the 40-frame stream)."""
    a = _resume_after_failure({"EAO_LOOKAHEAD_EAGER": "1", "EAO_HARNESS_FAIL_IFOREST": "40"})
    b = _resume_after_failure({"EAO_LOOKAHEAD_EAGER": "0", "EAO_HARNESS_FAIL_IFOREST": "40"})
    assert a["failed"] and b["failed"]
    assert a["rows"] == b["rows"]
    assert a["held"] == b["held"] and a["ints"] == b["ints"] and a["pts"] == b["pts"]
    assert np.allclose(a["floats"], b["floats"], rtol=1e-6, atol=1e-6)


def test_host_mean_std_skips_checked_point_by_point(harness):
    """The ComputeMeanAndStandard / BigToSmall skips (replay.cpp mean_std_same, big_to_small) trust
    each object's change mark, set through the votes of a point that moves or turns bad. With
    EAO_MS_VERIFY=1 every skip also compares each held point's own change epoch (abort on a miss);
    the point-record streams, where LocalMapping moves points no frame re-reports, run under it in a
    fresh process (the switch is read at load) and still equal the oracle."""
    here = os.path.dirname(os.path.abspath(__file__))
    out = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", os.path.join(here, "test_replay_host.py"),
                          "-k", "point_updates or run_updates or fr3_real_stream"],
                         env=dict(os.environ, EAO_MS_VERIFY="1"), capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, (out.stdout[-2000:], out.stderr[-2000:])
    assert "5 passed" in out.stdout, out.stdout[-500:]


@pytest.mark.parametrize("flag", ["EAO", "Full"])
def test_host_split_frame_matches_oracle(harness, flag):
    """eao_replay_frame_begin / _end with the frame's lines staged between them (the drop-in's line
    detection still running while the association starts): every frame's rows and the object state
    equal the oracle's one-call frames; a second begin, a local mapping or an end without an open
    frame are refused (EAO_E_STATE) and change nothing."""
    frames = synth.assoc_stream_fr3_real()[:150]
    g = _HostReplay(harness, flag)
    o = orc.Replay(flag)
    for i, f in enumerate(frames):
        g._with(ea.Replay.frame_begin, g, i + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"])
        if i == 3:
            H = harness
            assert H.eao_replay_local_mapping(g.h) == -5
            assert H.eao_replay_frame_begin(g.h, i + 1, ea.P(np.asarray(f["T"], np.float32)), 0, None, 0, None, None,
                                            None, None) == -5
        det = g._with(ea.Replay.frame_end, g, f.get("lines"))
        ref = o.frame(i + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"], lines=f.get("lines"))
        assert np.array_equal(det, ref), i
        if f["kf"]:
            g.local_mapping()
            o.local_mapping()
    assert harness.eao_replay_frame_end(g.h, None) == -5
    _compare(g, o)
