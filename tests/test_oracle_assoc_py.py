"""Second, independent restatement of the association (oracle/assoc_py.py) against the C++
oracle (oracle/assoc_ref.cpp), CPU only.

assoc_py.py is pure Python written from the reference text (Object.cc, Tracking.cc's object
section, LocalMapping.cc's object maintenance, isolation_forest.h), not from assoc_ref.cpp;
the two share nothing but the replay model and the documented quirk
definitions. They must agree on every detection outcome, every object's point
set and integer state, and its statistics within the north-star tolerance (1e-5):
  * the first 60 frames of the fr3 demo stream, flag EAO (BASELINE configs[1]);
  * a slice of the Full list, flag Full, with LocalMapping's point records, long enough for
    MergePotentialAssObjs and WhetherOverlapObject to merge objects;
  * short synthetic streams under the other flags (None / NP / IoU / NA).
The random pieces of the Python forest are pinned to THIS toolchain's libstdc++ through
tests/native/std_rng_kat.cpp (the library isolation_forest.h draws from), and its std::sort
restatement to libstdc++'s introsort, which orders the yaw measurements (Tracking.cc:2849).
Divergences found while writing it: none -- both restatements agree frame by frame.
"""
import os
import subprocess

import numpy as np
import pytest

import assoc_py as ap
import pyoracle as orc
from tools import synth

HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE = os.path.join(HERE, "native")
KAT = os.path.join(NATIVE, "_build", "std_rng_kat")


@pytest.fixture(scope="module")
def kat():
    subprocess.check_call(["make", "-s", "-C", NATIVE, "_build/std_rng_kat"])
    return KAT


def run_kat(kat, *args, dtype=np.uint32, stdin=None):
    out = subprocess.run([kat] + [str(a) for a in args], input=stdin, stdout=subprocess.PIPE, check=True).stdout
    return np.frombuffer(out, dtype)


def test_mt19937_and_distributions_match_libstdcxx(kat):
    g = ap.MT19937(5489)
    assert np.array_equal(np.array([g() for _ in range(1300)], np.uint32), run_kat(kat, "mt", 5489, 1300))
    for rng in (2, 3, 7, 1000003):
        g = ap.MT19937(77)
        got = np.array([ap.uniform_u32(g, rng) for _ in range(700)], np.uint32)
        assert np.array_equal(got, run_kat(kat, "lemire", 77, 700, rng)), rng
    g = ap.MT19937(3)
    got = np.array([ap.uniform_float(g, -1.5, 2.25) for _ in range(700)], np.float32)
    assert np.array_equal(got, run_kat(kat, "real", 3, 700, -1.5, 2.25, dtype=np.float32))


@pytest.mark.parametrize("n", [1, 2, 3, 10, 101, 1500, 70000])
def test_shuffle_matches_libstdcxx(kat, n):
    # 70000 > 65535 takes std::shuffle's one-draw-per-position branch
    g = ap.MT19937(99)
    ids = list(range(n))
    ap.shuffle(ids, g)
    assert np.array_equal(np.array(ids, np.uint32), run_kat(kat, "shuffle", 99, n))


@pytest.mark.parametrize("n", [30, 31, 257, 1200])
def test_forest_matches_libstdcxx_and_oracle(kat, n):
    rng = np.random.default_rng(n)
    pts = rng.normal(size=(n, 3)).astype(np.float32)
    pts[: n // 20 + 1] *= 8
    pts[n // 2:n // 2 + 5] = pts[0]  # exact duplicates: equal split values go the same way
    pts[:, 2] = np.round(pts[:, 2], 1)  # many ties in one dimension
    got = ap.iforest_scores(pts, 50, 12345, n // 2)
    ref = run_kat(kat, "iforest", n, 50, 12345, n // 2, dtype=np.float64, stdin=pts.tobytes())
    assert np.array_equal(got, ref)
    assert np.array_equal(got, orc.iforest(pts))


@pytest.mark.parametrize("n", [5, 16, 17, 30, 60])
def test_std_sort_matches_libstdcxx(kat, n):
    rng = np.random.default_rng(n)
    rows = np.zeros((n, 5), np.float32)
    rows[:, 0] = np.arange(n)  # identifies the row
    rows[:, 1] = rng.integers(1, 4, n)  # few distinct keys: the order of ties is the point
    rows[:, 2:] = rng.random((n, 3))
    got = [list(r) for r in rows]
    ap.std_sort(got, lambda a, b: a[1] > b[1])
    ref = run_kat(kat, "sort5", n, dtype=np.float32, stdin=rows.tobytes()).reshape(n, 5)
    assert np.array_equal(np.array(got, np.float32), ref)


def test_merge_break_lines_small_case():
    # object_3d_util.cpp:349-434: collinear pieces 10 px apart merge, the short stub is dropped
    L = [[0.0, 0.0, 40.0, 0.0], [50.0, 0.5, 100.0, 0.5], [200.0, 200.0, 210.0, 200.0]]
    out = ap.merge_break_lines(L, 20.0, 5.0, 30.0)
    assert out == [[0.0, 0.0, 100.0, 0.5]]


def _run_both(flag, frames):
    o = orc.Replay(flag)
    p = ap.Replay(flag)
    for i, f in enumerate(frames):
        a = o.step(i + 1, f)
        b = p.step(i + 1, f)
        assert np.array_equal(a, b), (i + 1, a.tolist(), b.tolist())
        if (i + 1) % 20 == 0 or i + 1 == len(frames):
            _same_objects(o, p, i + 1)
    return p


def _same_objects(o, p, fid):
    oi, of, op = o.objects()
    pi, pf, pp = p.objects()
    assert np.array_equal(oi, pi), (fid, oi.tolist(), pi.tolist())
    assert np.allclose(of, pf, rtol=1e-5, atol=1e-5, equal_nan=True), fid
    assert all(np.array_equal(x, y) for x, y in zip(op, pp)), fid


def test_fr3_demo_first_60_frames_eao():
    """BASELINE configs[1] stream, flag EAO: IoU / NP / projected IoU / t-test / create,
    DataAssociateUpdate, ComputeMeanAndStandard, the iForest erase, yaw sampling."""
    p = _run_both("EAO", synth.assoc_stream_fr3_real()[:60])
    assert p.stats["forests"] > 200 and p.stats["yaw"] > 50


def test_full_slice_with_localmapping_merges():
    """Full list (BASELINE configs[2]) slice with LocalMapping's point records (BA moves,
    culled / replaced points): WhetherMergeTwoMapObjs and DealTwoOverlapObjs both merge."""
    frames = synth.with_point_updates(synth.assoc_stream_fr3_real(0, 300)[:110], seed=0xEA9)
    p = _run_both("Full", frames)
    assert p.stats["merges"] >= 2 and p.stats["overlap_merges"] >= 1


@pytest.mark.parametrize("flag", ["None", "NP", "IoU", "NA"])
def test_other_flags_short_stream(flag):
    _run_both(flag, synth.assoc_stream(16, lines=True))


GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("name", ["replay_fr3_demo_eao", "replay_fr3_full", "replay_config_c_200"])
def test_independent_restatement_over_whole_streams(name):
    """The pure-Python restatement's outputs over the WHOLE streams (all 405 EAO frames, all 2582
    Full frames, and the 200 Config C frames at the config's scale -- 64 objects x 2000 points, NP
    subsampling at n > 3m, forests over clouds of >= 1500 points; tools/make_assoc_py_golden.py,
    minutes of pure Python, hence fixtures) equal the C++ oracle's fixtures that the engine's GPU
    tests compare against (tests/test_gpu_fr3.py, tests/test_gpu_shard.py): every detection's
    outcome and object id, the object records (statistics within 1e-5) and their point sets."""
    c = np.load(os.path.join(GOLDEN, name + ".npz"))
    p = np.load(os.path.join(GOLDEN, name + "_py.npz"))
    assert int(c["digest"]) == int(p["digest"]) and c["flag"] == p["flag"]
    bad = np.nonzero((c["det_out"] != p["det_out"]).any(1))[0]
    assert not len(bad), "first differing detection %d" % (bad[0] if len(bad) else -1)
    assert np.array_equal(c["obj_ints"], p["obj_ints"])
    assert np.allclose(c["obj_floats"], p["obj_floats"], rtol=1e-5, atol=1e-5, equal_nan=True)
    assert np.array_equal(c["obj_pts_len"], p["obj_pts_len"]) and np.array_equal(c["obj_pts_crc"], p["obj_pts_crc"])
    if name == "replay_config_c_200":  # the config's scale is reached: clouds of >= 1500 points
        assert int(p["obj_pts_len"].max()) >= 1500


def test_cpp_oracle_reproduces_demo_fixture():
    """The C++ oracle as built now still writes the committed demo fixture (so the fixture the
    engine and the Python restatement are held to is the oracle's current output)."""
    import zlib
    g = np.load(os.path.join(GOLDEN, "replay_fr3_demo_eao.npz"))
    frames = synth.assoc_stream_fr3_real()
    o = orc.Replay("EAO")
    det = np.concatenate([o.step(i + 1, f) for i, f in enumerate(frames)])
    assert np.array_equal(det, g["det_out"])
    ints, fl, pts = o.objects()
    assert np.array_equal(ints, g["obj_ints"]) and np.allclose(fl, g["obj_floats"], rtol=1e-5, atol=1e-5, equal_nan=True)
    crc = np.array([zlib.crc32(np.sort(q).astype(np.int32).tobytes()) for q in pts], np.uint32)
    assert np.array_equal(crc, g["obj_pts_crc"])
