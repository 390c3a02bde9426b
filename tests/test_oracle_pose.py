"""Pose-only optimisation oracle (oracle/pose_ref.cpp) against an independent numpy restatement.

Reference: src/Optimizer.cc:243-457 (PoseOptimization) on g2o's Levenberg-Marquardt
(Thirdparty/g2o/g2o/core/optimization_algorithm_levenberg.cpp:61-189), the
EdgeSE3ProjectXYZOnlyPose Jacobian (types/types_six_dof_expmap.cpp:266-296) and
SE3Quat::exp (types/se3quat.h:223-257).

The numpy restatement below shares no code with the oracle: it keeps the pose as a rotation
matrix (not a quaternion), sums the normal equations with vectorised einsum and solves them
with numpy's LU; only rounding separates the two, so the comparison is to 1e-5 on the pose
(BASELINE's tolerance for floating-point statistics) and exact on the outlier flags.
g2o itself cannot be built here (Eigen absent): parity against the original is unpinned.
"""
import numpy as np
import pytest

import pyoracle as orc
from tools import synth

DELTA = float(np.float32(np.sqrt(5.991)))


def _exp(u):
    w, v = u[:3], u[3:]
    th = np.sqrt(w @ w)
    O = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
    if th < 1e-5:
        R = np.eye(3) + O + O @ O
        V = R
    else:
        R = np.eye(3) + np.sin(th) / th * O + (1 - np.cos(th)) / th ** 2 * (O @ O)
        V = np.eye(3) + (1 - np.cos(th)) / th ** 2 * O + (th - np.sin(th)) / th ** 3 * (O @ O)
    return R, V @ v


def _errors(R, t, X, obs, K):
    fx, fy, cx, cy = K
    Xc = X @ R.T + t
    proj = np.stack([Xc[:, 0] / Xc[:, 2] * fx + cx, Xc[:, 1] / Xc[:, 2] * fy + cy], 1)
    return obs - proj, Xc


def _robust(chi, robust):
    if not robust:
        return chi, np.ones_like(chi)
    d2 = DELTA * DELTA
    s = np.sqrt(chi)
    return np.where(chi <= d2, chi, 2 * s * DELTA - d2), np.where(chi <= d2, 1.0, DELTA / s)


def _lm(R, t, X, obs, inv, K, robust, iters=10):
    """g2o SparseOptimizer::optimize(iters) with Levenberg; returns the final (R, t) and the
    errors of the last computeActiveErrors (which the outlier test reads)."""
    fx, fy = K[0], K[1]
    lam, ni, nbad = 0.0, 2.0, 0
    last = None
    for it in range(iters):
        e, Xc = _errors(R, t, X, obs, K)
        last = e
        chi = (e * e).sum(1) * inv
        rho0, rho1 = _robust(chi, robust)
        cur = rho0.sum()
        ini = cur
        x, y, iz = Xc[:, 0], Xc[:, 1], 1.0 / Xc[:, 2]
        J = np.zeros((len(X), 2, 6))
        J[:, 0] = np.stack([x * y * iz ** 2 * fx, -(1 + x * x * iz ** 2) * fx, y * iz * fx, -iz * fx, 0 * x,
                            x * iz ** 2 * fx], 1)
        J[:, 1] = np.stack([(1 + y * y * iz ** 2) * fy, -x * y * iz ** 2 * fy, -x * iz * fy, 0 * x, -iz * fy,
                            y * iz ** 2 * fy], 1)
        W = rho1 * inv
        H = np.einsum("nki,n,nkj->ij", J, W, J)
        b = -np.einsum("nki,n,nk->i", J, W, e)
        if it == 0:
            lam, ni, nbad = 1e-5 * np.abs(np.diag(H)).max(), 2.0, 0
        q = 0
        while True:
            dx = np.linalg.solve(H + lam * np.eye(6), b)
            dR, dt = _exp(dx)
            R2, t2 = dR @ R, dR @ t + dt
            e2, _ = _errors(R2, t2, X, obs, K)
            last = e2
            tmp = _robust((e2 * e2).sum(1) * inv, robust)[0].sum()
            rho = (cur - tmp) / (dx @ (lam * dx + b) + 1e-3)
            if rho > 0 and np.isfinite(tmp):
                lam *= max(1 / 3, min(1 - (2 * rho - 1) ** 3, 2 / 3))
                ni = 2.0
                cur = tmp
                R, t = R2, t2
            else:
                lam *= ni
                ni *= 2
            q += 1
            if not (rho < 0 and q < 10):
                break
        if q == 10 or rho == 0:
            break
        nbad = nbad + 1 if (ini - cur) * 1e3 < ini else 0
        if nbad >= 3:
            break
    return R, t, last


def pose_numpy(K, Tcw, kps, has, pos, inv_lvl):
    idx = np.nonzero(has)[0]
    n0 = len(idx)
    if n0 < 3:
        return 0, Tcw.copy(), np.zeros(len(kps), np.uint8)
    obs = np.stack([kps["x"][idx], kps["y"][idx]], 1).astype(np.float64)
    X = pos[idx].astype(np.float64)
    inv = inv_lvl[kps["octave"][idx]].astype(np.float64)
    R0, t0 = Tcw[:3, :3].astype(np.float64), Tcw[:3, 3].astype(np.float64)
    out = np.zeros(n0, bool)
    robust = True
    nbad = 0
    R, t = R0, t0
    for it in range(4):
        act = ~out
        if act.any():
            R, t, last = _lm(R0, t0, X[act], obs[act], inv[act], K, robust)
            e = np.zeros((n0, 2))
            e[act] = last
        else:
            R, t = R0, t0
            e = np.zeros((n0, 2))
        e_out, _ = _errors(R, t, X[out], obs[out], K)
        e[out] = e_out
        chi = ((e * e).sum(1) * inv).astype(np.float32)
        out = chi > np.float32(5.991)
        nbad = int(out.sum())
        if it == 2:
            robust = False
        if n0 < 10:
            break
    To = np.eye(4, dtype=np.float32)
    To[:3, :3], To[:3, 3] = R, t
    flags = np.zeros(len(kps), np.uint8)
    flags[idx] = out
    return n0 - nbad, To, flags


@pytest.mark.parametrize("seed,n", [(0, 1000), (1, 300), (2, 8), (3, 2000), (4, 60)])
def test_oracle_vs_numpy(seed, n):
    Tp, kps, has, pos, inv, Tt = synth.pose_problem(seed, n)
    K = synth.TUM3_K
    ni_o, To_o, out_o = orc.pose_optimization(orc.cam(), Tp, kps, has, pos, inv)
    ni_n, To_n, out_n = pose_numpy(K, Tp, kps, has, pos, inv)
    assert ni_o == ni_n
    assert np.array_equal(out_o[has == 1], out_n[has == 1])
    assert np.abs(To_o - To_n).max() < 1e-5
    assert np.abs(To_o - Tt).max() < 0.02  # recovers the true pose from the perturbed prior


def test_oracle_edge_cases():
    Tp, kps, has, pos, inv, Tt = synth.pose_problem(7, 50)
    none = np.zeros_like(has)
    ni, To, out = orc.pose_optimization(orc.cam(), Tp, kps, none, pos, inv)
    assert ni == 0 and np.array_equal(To, Tp)  # < 3 correspondences: pose untouched
    two = none.copy()
    two[:2] = 1
    ni, To, out = orc.pose_optimization(orc.cam(), Tp, kps, two, pos, inv)
    assert ni == 0 and np.array_equal(To, Tp)
    # exact observations: every edge an inlier, the true pose recovered
    Tp, kps, has, pos, inv, Tt = synth.pose_problem(8, 400, noise_px=0.0, frac_out=0.0)
    ni, To, out = orc.pose_optimization(orc.cam(), Tp, kps, has, pos, inv)
    assert ni == int(has.sum()) and not out.any()
    assert np.abs(To - Tt).max() < 1e-4
