"""Pinning of the line-detector restatement (oracle/lines_ref.cpp, the EDLineDetector of
src/line_detect/libs/binary_descriptor.cpp) against the only outputs the reference holds for this
algorithm family: the Edge Drawing library's edge map of lena (Thirdparty/EDTest/ED-EdgeMap.pgm,
DetectEdgesByED(SOBEL, 36, 8, 1.0), EDTest/main.cpp:57-74) and EDLines' 168 segments of house
(EDLinesTest/LineSegments.txt, EDLines/main.cpp:46-75). Fixtures: tests/golden/ed_pin.npz, made
by tools/make_ed_fixtures.py from those data files.

The library is a different implementation of the same algorithms (binary only, never run here),
so agreement is measured, not bit-exact: pixel agreement of the edge maps and line-support
agreement of the segments, with the divergences attributed in DESIGN.md §6. The floors below are
the measured values (deterministic) rounded down."""
import os

import numpy as np
import pytest

import pyoracle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

G = np.load(os.path.join(ROOT, "tests", "golden", "ed_pin.npz"))


def dilate1(m):
    p = np.pad(m, 1)
    out = np.zeros_like(m)
    h, w = m.shape
    for dy in range(3):
        for dx in range(3):
            out |= p[dy:dy + h, dx:dx + w]
    return out


def edge_agreement(ours, ref):
    exact = (ours & ref).sum()
    return dict(n_ours=int(ours.sum()), n_ref=int(ref.sum()), exact_recall=exact / ref.sum(),
                exact_precision=exact / ours.sum(), recall_1px=(ref & dilate1(ours)).sum() / ref.sum(),
                precision_1px=(ours & dilate1(ref)).sum() / ours.sum())


def coverage(A, B, tol, step=0.5, max_deg=10.0):
    """Fraction of A's total segment length whose points lie within tol px of a segment of B of
    about the same orientation (within max_deg)."""
    bx0, by0, bx1, by1 = B.T
    bdx, bdy = bx1 - bx0, by1 - by0
    bl2 = np.maximum(bdx * bdx + bdy * bdy, 1e-12)
    bang = np.arctan2(bdy, bdx)
    cov = tot = 0.0
    for a in A:
        L = float(np.hypot(a[2] - a[0], a[3] - a[1]))
        t = np.linspace(0, 1, max(2, int(L / step) + 1))
        px, py = a[0] + t * (a[2] - a[0]), a[1] + t * (a[3] - a[1])
        ang = np.arctan2(a[3] - a[1], a[2] - a[0])
        ok = np.abs((bang - ang + np.pi / 2) % np.pi - np.pi / 2) < np.radians(max_deg)
        u = np.clip(((px[:, None] - bx0) * bdx + (py[:, None] - by0) * bdy) / bl2, 0, 1)
        d = np.hypot(px[:, None] - (bx0 + u * bdx), py[:, None] - (by0 + u * bdy))
        d[:, ~ok] = np.inf
        cov += (d.min(1) <= tol).mean() * L
        tot += L
    return cov / tot


ED_MAP = np.unpackbits(G["ed_edge_map"])[:G["lena"].size].reshape(G["lena"].shape).astype(bool)


def test_fixture_shapes():
    assert G["lena"].shape == (512, 512) and G["house"].shape == (400, 400)
    assert ED_MAP.sum() == 17302 and G["ed_segments"].shape == (168, 4)


def test_edge_map_with_ed_knobs_matches_ed_edgemap():
    # ED's knobs on the restatement: Sobel |dx|+|dy| unscaled (gdiv 1), gradient threshold 36,
    # anchor threshold 8, scan interval 1, sigma 1 (the 5x5 blur), chains shorter than ED's
    # minimum path length 10 dropped
    m, n = orc.ed_edge_map(G["lena"], 36, 8, 1, 10, 1)
    a = edge_agreement(m > 0, ED_MAP)
    print("ED knobs on lena:", n, "chains", a)
    assert abs(a["n_ours"] - a["n_ref"]) / a["n_ref"] < 0.03
    assert a["exact_recall"] >= 0.82 and a["exact_precision"] >= 0.81
    assert a["recall_1px"] >= 0.94 and a["precision_1px"] >= 0.94


def test_edge_map_with_descriptor_scaling():
    # the same knobs through EDLineDetector's own scaling (gImg_ = thresholded sum / 4 with the
    # anchor test on the quarter values, binary_descriptor.cpp:1630-1660) and its chain minimum 15
    m, n = orc.ed_edge_map(G["lena"], 36, 8, 1, 15, 4)
    a = edge_agreement(m > 0, ED_MAP)
    print("descriptor scaling on lena:", n, "chains", a)
    assert a["precision_1px"] >= 0.95 and a["recall_1px"] >= 0.82


def test_segments_match_edlines_house():
    ref = G["ed_segments"]
    S = orc.ed_segments(G["house"], 36, 8, 1, 12, 1, 1.6).astype(np.float64)
    ours_on_ref = coverage(S, ref, 1.0)
    ref_on_ours = coverage(ref, S, 1.0)
    print("house: %d segments (EDLines %d); our length on EDLines' lines %.3f, EDLines' on ours %.3f"
          % (len(S), len(ref), ours_on_ref, ref_on_ours))
    assert ours_on_ref >= 0.78  # what the restatement keeps is on EDLines' lines
    assert ref_on_ours >= 0.55  # EDLines keeps more (validation)
    assert coverage(S, ref, 2.0) >= 0.88


def test_segment_divergence_is_the_validation():
    # with LineValidation_ off (bValidate_ = false), the restatement's fitted segments cover most
    # of EDLines' line length: the divergence is the validation test, not the chains or the fits
    ref = G["ed_segments"]
    S = orc.ed_segments(G["house"], 36, 8, 1, 12, 1, 1.6, validate=0).astype(np.float64)
    S = S[np.isfinite(S).all(1)]
    r = coverage(ref, S, 1.0)
    print("house, validation off: %d segments, EDLines' length on ours %.3f" % (len(S), r))
    assert r >= 0.70
