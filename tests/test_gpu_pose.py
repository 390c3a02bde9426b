"""GPU pose-only optimisation (k_pose_opt) vs the CPU restatement oracle/pose_ref.cpp.

Reference: src/Optimizer.cc:243-457 (PoseOptimization; called at src/Tracking.cc:1106,1699,1741)
on g2o's Levenberg-Marquardt. Bars (BASELINE north_star: 1e-5 on floating-point statistics):
inlier count and every outlier flag identical, pose entries within 1e-5. The GPU sums the
normal equations in a fixed wave-tree order, the oracle in edge order (g2o's), so the two
differ only in rounding.
"""
import numpy as np
import pytest

import eao_accel as ea
import pyoracle as orc
from tools import synth

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _check(g, o):
    ni_g, T_g, out_g = g
    ni_o, T_o, out_o = o
    assert ni_g == ni_o
    assert np.array_equal(out_g, out_o), int((out_g != out_o).sum())
    assert np.abs(T_g - T_o).max() < TOL, float(np.abs(T_g - T_o).max())


# sizes: both register layouts of the 256-thread kernel (<= 1024, <= 2048 edges) and the
# 1024-thread one (> 2048); < 10 edges (one round, Optimizer.cc:446); < 3 (early return)
@pytest.mark.parametrize("seed,n", [(0, 1000), (1, 300), (2, 8), (3, 2000), (4, 60), (5, 1576), (6, 4000),
                                    (7, 3), (9, 2)])
def test_pose_single(seed, n):
    Tp, kps, has, pos, inv, Tt = synth.pose_problem(seed, n)
    if n <= 3:
        has[:] = 1
    p = ea.Pose(max_kps=8192)
    g = p.optimize(ea.camera(), Tp, kps, has, pos, inv)
    o = orc.pose_optimization(orc.cam(), Tp, kps, has, pos, inv)
    _check((g[0], g[1], g[2] * has), (o[0], o[1], o[2] * has))
    if n > 3:
        assert np.abs(g[1] - Tt).max() < 0.02


def test_pose_variants():
    """all edges inliers (exact observations); heavy outlier share; large prior error;
    no map points at all; outlier flags of points without a map point left untouched."""
    p = ea.Pose(max_kps=4096)
    cases = [dict(noise_px=0.0, frac_out=0.0), dict(frac_out=0.4), dict(rot_err=0.08, t_err=0.2),
             dict(frac_mp=0.0), dict(frac_mp=0.05, n=100)]
    for i, kw in enumerate(cases):
        n = kw.pop("n", 800)
        Tp, kps, has, pos, inv, Tt = synth.pose_problem(100 + i, n, **kw)
        pre = np.full(n, 7, np.uint8)
        g = p.optimize(ea.camera(), Tp, kps, has, pos, inv, outlier=pre)
        o = orc.pose_optimization(orc.cam(), Tp, kps, has, pos, inv)
        assert np.all(g[2][has == 0] == 7)  # only has_mp entries are written
        _check((g[0], g[1], g[2] * has), (o[0], o[1], o[2] * has))


def test_pose_batch_device():
    """HBM-resident batch of frames with mixed sizes against the oracle frame by frame."""
    import torch
    dev = torch.device("cuda", 0)
    sizes = [1000, 0, 2, 9, 500, 1576, 1200, 64, 1576, 777] * 4
    F, cap = len(sizes), 1576
    T = np.zeros((F, 16), np.float32)
    kp = np.zeros((F, cap), dtype=[("x", "f4"), ("y", "f4"), ("size", "f4"), ("angle", "f4"), ("response", "f4"),
                                   ("octave", "i4"), ("class_id", "i4")])
    has = np.zeros((F, cap), np.uint8)
    pos = np.zeros((F, cap, 3), np.float32)
    probs = []
    for f, n in enumerate(sizes):
        Tp, k, h, X, inv, _ = synth.pose_problem(1000 + f, max(n, 1))
        k, h, X = k[:n], h[:n], X[:n]
        T[f] = Tp.reshape(16)
        kp[f, :n], has[f, :n], pos[f, :n] = k, h, X
        probs.append((Tp, k, h, X))
    d_T = torch.from_numpy(T).to(dev)
    d_cnt = torch.tensor(sizes, dtype=torch.int32, device=dev)
    d_kp = torch.from_numpy(kp.view(np.uint8).reshape(F, cap, 28)).to(dev)
    d_has = torch.from_numpy(has).to(dev)
    d_pos = torch.from_numpy(pos).to(dev)
    d_To = torch.zeros((F, 16), dtype=torch.float32, device=dev)
    d_out = torch.full((F, cap), 9, dtype=torch.uint8, device=dev)
    d_ni = torch.full((F,), -1, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream())
    ea.Pose(max_kps=cap, max_batch=F).optimize_batch_device(
        ea.camera(), F, cap, d_T.data_ptr(), d_cnt.data_ptr(), d_kp.data_ptr(), d_has.data_ptr(), d_pos.data_ptr(),
        inv, d_To.data_ptr(), d_out.data_ptr(), d_ni.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    To, out, ni = d_To.cpu().numpy(), d_out.cpu().numpy(), d_ni.cpu().numpy()
    for f, (Tp, k, h, X) in enumerate(probs):
        n = sizes[f]
        o = orc.pose_optimization(orc.cam(), Tp, k, h, X, inv)
        g_out = out[f, :n].copy()
        assert np.all(g_out[h == 0] == 9)
        assert np.all(out[f, n:] == 9)
        _check((int(ni[f]), To[f].reshape(4, 4), g_out * h), (o[0], o[1], o[2] * h))


def test_pose_args():
    p = ea.Pose(max_kps=64)
    Tp, kps, has, pos, inv, _ = synth.pose_problem(0, 100)
    with pytest.raises(ea.EaoError):
        p.optimize(ea.camera(), Tp, kps, has, pos, inv)  # n > max_kps
