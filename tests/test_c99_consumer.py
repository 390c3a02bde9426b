"""A plain C99 program over include/eao_accel.h (tests/native/c99_consumer.c, built by the engine's
Makefile with -std=c99 -pedantic -Wall -Wextra -Werror and linked against libeao_accel.so).

CPU: the header compiles as C99 and the library links and runs from C: without a gfx950 device
eao_orb_create / eao_assoc_create return EAO_E_NODEVICE.
GPU: one extraction of a synthetic 640x480 frame from C equals the oracle's keypoints and
descriptors; one association replay frame runs (ORBextractor::operator(), src/ORBextractor.cc:1043-1105;
the object section of TrackWithMotionModel, src/Tracking.cc:1241-1696)."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "eao-slam_amd", "lib")
EXE = os.path.join(LIB, "c99_consumer")
KP = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
               ("octave", "<i4"), ("class_id", "<i4")])


def _exe():
    if not os.path.exists(EXE):  # the CPU container builds it (build() does too); the GPU box ships it
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "eao-slam_amd"), "lib/c99_consumer"])
    return EXE


def synth_frame(W=640, H=480):
    y, x = np.mgrid[0:H, 0:W]
    v = np.where(((x // 24 + y // 24) & 1) == 1, 200, 40) + ((x * 7 + y * 13) & 15) - 8
    v = np.where((x - 320) ** 2 + (y - 240) ** 2 < 90 * 90, 255 - v, v)
    return np.clip(v, 0, 255).astype(np.uint8)


def test_c99_header_compiles_strict(tmp_path):
    # the header alone, as a C99 translation unit with every warning an error
    src = tmp_path / "h.c"
    src.write_text('#include "eao_accel.h"\nint main(void) { return eao_version() ? 0 : 1; }\n')
    subprocess.check_call(["cc", "-std=c99", "-pedantic", "-Wall", "-Wextra", "-Werror", "-c",
                           "-I" + os.path.join(ROOT, "include"), str(src), "-o", str(tmp_path / "h.o")])


def test_c99_consumer_without_device():
    import eao_accel as ea
    if ea.device_ok(0):
        pytest.skip("a gfx950 device is present (the GPU test covers it)")
    r = subprocess.run([_exe(), "cpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "EAO_E_NODEVICE" in r.stdout


@pytest.mark.gpu
def test_c99_consumer_extracts_and_associates(tmp_path):
    import pyoracle as orc
    out = tmp_path / "kps.bin"
    r = subprocess.run([_exe(), "gpu", str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "replay: frame 1 ->" in r.stdout
    b = out.read_bytes()
    n = int(np.frombuffer(b[:4], np.int32)[0])
    kps = np.frombuffer(b[4:4 + 28 * n], KP)
    desc = np.frombuffer(b[4 + 28 * n:4 + 60 * n], np.uint8).reshape(n, 32)
    ok, od = orc.extract(synth_frame())
    assert n == len(ok) and n > 100
    for f in KP.names:
        assert np.array_equal(kps[f], ok[f]), f
    assert np.array_equal(desc, od)
