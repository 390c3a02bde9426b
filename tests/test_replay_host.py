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
    H = ctypes.CDLL(os.path.join(NATIVE, "_build", "libreplay_host.so"))
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
