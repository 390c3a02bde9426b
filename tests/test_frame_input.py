"""Frame input stage host functions (src/Tracking.cc:415-554) through
the C ABI, against the reference's own data files kept as fixtures (a few
data/yolo_txts files, the head of data/groundtruth.txt) and the values
tools/make_fr3_inputs.py derived from the full files (tests/golden/fr3_inputs.npz).
Host-only: no device needed."""
import glob
import os

import numpy as np
import pytest

import eao_accel as ea
from tools import synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_yolo_parse_reference_files():
    d = synth.fr3_inputs()
    ts = ["%f" % t for t in d["timestamps"]]
    files = sorted(glob.glob(os.path.join(GOLDEN, "yolo_sample", "*.txt")))
    assert len(files) >= 5
    for f in files:
        i = ts.index(os.path.basename(f)[:-4])
        got = ea.yolo_parse(open(f, "rb").read())
        want = d["boxes"][d["box_off"][i]:d["box_off"][i + 1]]
        assert got.shape == (len(want), 6)
        assert np.array_equal(got[:, :5], want) and (got[:, 5] == 0).all()  # scores "0.82" -> 0 (Q1)


def test_yolo_parse_int_semantics_and_order():
    # `istr >> int`: a fractional token yields its integer part and ends the row
    assert ea.yolo_parse("39 289 18 23 92 0.767674\n").tolist() == [[39, 289, 18, 23, 92, 0]]
    assert ea.yolo_parse("1 2 3 4 5 1.5 77\n").tolist() == [[1, 2, 3, 4, 5, 1]]
    # a short row's missing fields read as 0; a bad token ends the row; CRLF and no final newline
    assert ea.yolo_parse("7 8 9\r\n4 5 x 6\r\n3 1 1 1 1 2").tolist() == [[3, 1, 1, 1, 1, 2], [7, 8, 9, 0, 0, 0],
                                                                       [4, 5, 0, 0, 0, 0]]
    # a sign right after digits starts the next extraction ("2-3" reads 2, then -3); a lone sign
    # fails it and ends the row
    assert ea.yolo_parse("1 2-3 4 5 6\n").tolist() == [[1, 2, -3, 4, 5, 6]]
    assert ea.yolo_parse("5+3 1 1 1 1\n").tolist() == [[5, 3, 1, 1, 1, 1]]
    assert ea.yolo_parse("1 2+ 3 4 5 6\n").tolist() == [[1, 2, 0, 0, 0, 0]]
    # std::sort by score, descending; <= 16 equal scores keep the file order (insertion sort)
    rows = [[c, c, 0, 1, 1, 0] for c in range(15)]
    txt = "".join("%d %d %d %d %d 0.5\n" % tuple(r[:5]) for r in rows)
    assert ea.yolo_parse(txt).tolist() == rows
    rnd = np.random.default_rng(1).permutation(40)
    txt = "".join("%d 0 0 1 1 %d\n" % (c, s) for c, s in zip(range(40), rnd))
    got = ea.yolo_parse(txt)
    assert got[:, 5].tolist() == sorted(rnd.tolist(), reverse=True)
    assert all(got[k, 0] == int(np.nonzero(rnd == got[k, 5])[0][0]) for k in range(40))


def _gt_head():
    rows = [l.split() for l in open(os.path.join(GOLDEN, "groundtruth_head.txt")).read().split("\n")[3:] if l.strip()]
    return np.array(rows, np.float64)


def test_gt_lookup_matches_reference_selection():
    d = synth.fr3_inputs()
    gt = _gt_head()
    ts = d["timestamps"][:300]
    idx, T = ea.gt_lookup(gt, ts)
    # Tracking.cc:508-519: first row whose to_string(t)[:-4] equals the frame's
    keys = ["%f" % t for t in gt[:, 0]]
    for i, t in enumerate(ts):
        k = ("%f" % t)[:-4]
        want = next((r for r, s in enumerate(keys) if s[:-4] == k), -1)
        assert idx[i] == want
        if want < 0:
            assert not np.isfinite(d["gt"][i, 0]) and (T[i] == 0).all()
        else:
            assert np.array_equal(gt[want, 1:], d["gt"][i])
            # Twc of g2o::SE3Quat(t, q) with the quaternion normalised (normalizeRotation)
            row = gt[want, 1:].copy()
            row[3:] /= np.linalg.norm(row[3:])
            assert np.allclose(T[i], np.linalg.inv(synth.tum_Tcw(row).astype(np.float64)), atol=2e-6)
    assert (idx >= 0).sum() > 200 and (idx < 0).sum() > 0  # gaps in the 100 Hz GT exist


def test_undistort_zero_is_a_copy_and_rejects_distortion():
    import ctypes
    img = np.random.default_rng(2).integers(0, 256, (48, 64), np.uint8)
    out = np.zeros_like(img)
    zero = np.zeros(5, np.float32)
    L = ea.lib()
    bad = np.array([0.1, 0, 0, 0, 0], np.float32)
    assert L.eao_undistort_zero(ea.P(bad), 5, ea.P(img), 64, 48, 64, ea.P(out), 64, None) == -1
    rc = L.eao_undistort_zero(ea.P(zero), 5, ea.P(img), 64, 48, 64, ea.P(out), 64, None)
    if rc == -3:
        pytest.skip("no HIP runtime device for the copy in this container")
    assert rc == 0 and np.array_equal(out, img)
