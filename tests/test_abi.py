"""The drop-in boundary: the C-ABI library loads, exports every entry point
include/eao_accel.h declares, and without a gfx950 device refuses to compute
(EAO_E_NODEVICE) instead of falling back to a CPU path. CPU test."""
import ctypes
import os
import re

import pytest

import eao_accel as ea

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "eao_accel.h")


def declared():
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w[\w\s\*]*?\b(eao_\w+)\s*\(", txt, flags=re.M)))


def test_header_declares_the_boundary():
    names = declared()
    for must in ("eao_orb_create", "eao_orb_extract", "eao_orb_extract_batch_device", "eao_match_motion",
                 "eao_match_local", "eao_match_init", "eao_np_test_batch", "eao_iforest_scores_batch",
                 "eao_replay_frame", "eao_replay_local_mapping"):
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = ea.lib()
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_no_cpu_fallback_without_device():
    lib = ea.lib()
    assert b"gfx950" in lib.eao_version()
    if ea.device_ok(0):
        pytest.skip("a gfx950 device is present")
    h = ctypes.c_void_p()
    p = ea.OrbParams(1000, 1.2, 8, 20, 7, 640, 480, 1)
    assert lib.eao_orb_create(ctypes.byref(p), 0, ctypes.byref(h)) == ea.EAO_E_NODEVICE
    assert lib.eao_matcher_create(0, 4096, 2, ctypes.byref(h)) == ea.EAO_E_NODEVICE
    assert lib.eao_assoc_create(0, 65536, ctypes.byref(h)) == ea.EAO_E_NODEVICE
    assert b"no CPU fallback" in lib.eao_last_error()
    with pytest.raises(ea.EaoError):
        ea.Orb()
