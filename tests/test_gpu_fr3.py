"""Association replay on the reference's own fr3_long_office inputs (real YOLO boxes of
data/yolo_txts with scores parsed as 0, GT poses of data/groundtruth.txt; 3-D clouds
synthesised around them, tools/synth.assoc_stream_fr3_real), engine vs oracle fixtures:

  * BASELINE configs[1]: the demo list (rgb_seq_pose.txt, 405 frames), flag EAO;
  * BASELINE configs[2]: the Full list (rgb_full_demo.txt, all 2582 frames), flag Full
    (iForest + object lines + yaw sampling + EAO association + LocalMapping merges).

The oracle outputs are committed (tools/make_fr3_golden.py; the Full stream is a minute
of oracle time) together with a digest of the generated inputs. Bars: association
outcome and object id of every detection identical, object records identical in their
integer fields and within 1e-5 in their statistics, object point sets identical (CRC of
the sorted map-point ids)."""
import os
import zlib

import numpy as np
import pytest

import eao_accel as ea
from tools import synth

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _digest(frames):
    h = 0
    for f in frames:
        for k in ("T", "boxes", "ids", "pos", "uv", "bad", "lines"):
            h = zlib.crc32(np.ascontiguousarray(f[k]).tobytes(), h)
        h = zlib.crc32(bytes([1 if f["kf"] else 0]), h)
    return h


def _check(name, start, n):
    g = np.load(os.path.join(GOLDEN, name))
    frames = synth.assoc_stream_fr3_real(start, n)
    assert _digest(frames) == int(g["digest"]), "generated inputs differ from the fixture's"
    rp = ea.Replay(ea.Assoc(), g["flag"].item().decode())
    det = rp.run(ea.Replay.pack(frames))
    bad = np.nonzero((det != g["det_out"]).any(1))[0]
    assert not len(bad), "first differing detection %d: %s vs %s" % (bad[0], det[bad[0]], g["det_out"][bad[0]])
    ints, fl, pts = rp.objects()
    assert np.array_equal(ints, g["obj_ints"])
    assert np.allclose(fl, g["obj_floats"], rtol=1e-5, atol=1e-5, equal_nan=True)
    crc = np.array([zlib.crc32(np.sort(p).astype(np.int32).tobytes()) for p in pts], np.uint32)
    assert np.array_equal(np.array([len(p) for p in pts]), g["obj_pts_len"])
    assert np.array_equal(crc, g["obj_pts_crc"])
    rp.close()
    return det


def test_fr3_demo_eao_405():
    det = _check("replay_fr3_demo_eao.npz", None, None)
    assert (det[:, 0] == 1).sum() > 100  # IoU associations happen on the real boxes


def test_fr3_full_2582():
    det = _check("replay_fr3_full.npz", 0, 2582)
    assert len(det) == 17204
    assert {1, 2, 3, 4, 5} <= set(det[:, 0].tolist())  # every association route is taken


def test_fr3_demo_eao_405_hip_streams():
    """The same replay with the association's launches on HIP streams (EAO_HSA_LANES=0) instead
    of the HSA lanes (AQL packets, BAR-written inputs): the lane kind is fixed per process, so
    the check runs in one child process."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path[:0] = [%r, %r, %r]; import test_gpu_fr3 as t; "
            "t._check('replay_fr3_demo_eao.npz', None, None); print('ok')"
            % (root, os.path.join(root, "tests"), os.path.join(root, "eao-slam_amd", "python")))
    env = dict(os.environ, EAO_HSA_LANES="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-2000:] + r.stderr[-2000:]
