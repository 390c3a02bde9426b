/*
 * pose_ref.cpp -- CPU restatement of Optimizer::PoseOptimization (monocular edges)
 * TEST INFRASTRUCTURE ONLY: the checker of tests/ and the CPU leg of bench.py.
 *
 * Reference: src/Optimizer.cc:243-457 on g2o (Thirdparty/g2o):
 *   OptimizationAlgorithmLevenberg::solve     core/optimization_algorithm_levenberg.cpp:61-189
 *   SparseOptimizer::optimize / active errors core/sparse_optimizer.cpp:61-114,354-420
 *   BlockSolver::buildSystem / setLambda      core/block_solver.hpp:502-570,573-600
 *   BaseUnaryEdge::constructQuadraticForm     core/base_unary_edge.hpp:43-72
 *   LinearSolverDense (Eigen LDLT)            solvers/linear_solver_dense.h:65-113
 *   EdgeSE3ProjectXYZOnlyPose                 types/types_six_dof_expmap.h:143-171, .cpp:266-296
 *   VertexSE3Expmap::oplusImpl, SE3Quat::exp  types/types_six_dof_expmap.h:73-76, types/se3quat.h:223-257
 *   RobustKernelHuber::robustify              core/robust_kernel_impl.cpp:65-91
 *   Converter::toSE3Quat / toCvMat            src/Converter.cc:28-62
 *
 * Eigen (absent from the image) is restated by its published scalar semantics: the
 * Quaternion(Matrix3) branch rule, q*v = v + w uv + vec x uv with uv = 2 vec x v,
 * toRotationMatrix, the scalar Hamilton product, squaredNorm of a 4-vector as two
 * 2-wide packets, and LDLT with diagonal pivoting (Eigen 3.3 ldlt_inplace<Lower>). Where
 * the SSE-dispatched binary rounds differently the result is "parity unpinned"; sums over
 * edges run in edge insertion order (EdgeIDCompare), one accumulator per entry.
 */
#include <algorithm>
#include <cmath>
#include <limits>
#include <cstdint>
#include <cstring>
#include <vector>
#include "oracle.h"

namespace {

struct Se3 {
  double w, x, y, z;  // Quaterniond
  double t[3];
};

void normalize_rot(Se3& s) {  // SE3Quat::normalizeRotation (se3quat.h:280-285)
  if (s.w < 0) {
    s.w = -s.w;
    s.x = -s.x;
    s.y = -s.y;
    s.z = -s.z;
  }
  const double n = std::sqrt((s.x * s.x + s.z * s.z) + (s.y * s.y + s.w * s.w));
  s.x /= n;
  s.y /= n;
  s.z /= n;
  s.w /= n;
}

Se3 from_matrix(const double R[3][3], const double t[3]) {  // SE3Quat(R, t)
  Se3 s;
  double tr = (R[0][0] + R[1][1]) + R[2][2];
  if (tr > 0) {
    tr = std::sqrt(tr + 1.0);
    s.w = 0.5 * tr;
    tr = 0.5 / tr;
    s.x = (R[2][1] - R[1][2]) * tr;
    s.y = (R[0][2] - R[2][0]) * tr;
    s.z = (R[1][0] - R[0][1]) * tr;
  } else {
    int i = 0;
    if (R[1][1] > R[0][0]) i = 1;
    if (R[2][2] > R[i][i]) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    double c[3];
    tr = std::sqrt(R[i][i] - R[j][j] - R[k][k] + 1.0);
    c[i] = 0.5 * tr;
    tr = 0.5 / tr;
    s.w = (R[k][j] - R[j][k]) * tr;
    c[j] = (R[j][i] + R[i][j]) * tr;
    c[k] = (R[k][i] + R[i][k]) * tr;
    s.x = c[0];
    s.y = c[1];
    s.z = c[2];
  }
  for (int a = 0; a < 3; a++) s.t[a] = t[a];
  normalize_rot(s);
  return s;
}

void rotate(const Se3& s, const double v[3], double o[3]) {
  double u0 = s.y * v[2] - s.z * v[1];
  double u1 = s.z * v[0] - s.x * v[2];
  double u2 = s.x * v[1] - s.y * v[0];
  u0 += u0;
  u1 += u1;
  u2 += u2;
  o[0] = v[0] + s.w * u0 + (s.y * u2 - s.z * u1);
  o[1] = v[1] + s.w * u1 + (s.z * u0 - s.x * u2);
  o[2] = v[2] + s.w * u2 + (s.x * u1 - s.y * u0);
}

void map_point(const Se3& s, const double X[3], double o[3]) {  // SE3Quat::map
  double r[3];
  rotate(s, X, r);
  for (int a = 0; a < 3; a++) o[a] = r[a] + s.t[a];
}

void to_matrix(const Se3& s, double R[3][3]) {  // Quaternion::toRotationMatrix
  const double tx = 2 * s.x, ty = 2 * s.y, tz = 2 * s.z;
  const double twx = tx * s.w, twy = ty * s.w, twz = tz * s.w;
  const double txx = tx * s.x, txy = ty * s.x, txz = tz * s.x;
  const double tyy = ty * s.y, tyz = tz * s.y, tzz = tz * s.z;
  R[0][0] = 1 - (tyy + tzz);
  R[0][1] = txy - twz;
  R[0][2] = txz + twy;
  R[1][0] = txy + twz;
  R[1][1] = 1 - (txx + tzz);
  R[1][2] = tyz - twx;
  R[2][0] = txz - twy;
  R[2][1] = tyz + twx;
  R[2][2] = 1 - (txx + tyy);
}

// SE3Quat::exp(update) * estimate (VertexSE3Expmap::oplusImpl)
Se3 oplus(const Se3& est, const double u[6]) {
  const double om[3] = {u[0], u[1], u[2]};
  const double theta = std::sqrt((om[0] * om[0] + om[1] * om[1]) + om[2] * om[2]);
  const double O[3][3] = {{0, -om[2], om[1]}, {om[2], 0, -om[0]}, {-om[1], om[0], 0}};
  double O2[3][3];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) O2[i][j] = (O[i][0] * O[0][j] + O[i][1] * O[1][j]) + O[i][2] * O[2][j];
  double R[3][3], V[3][3];
  if (theta < 0.00001) {
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) R[i][j] = ((i == j ? 1.0 : 0.0) + O[i][j]) + O2[i][j];
    std::memcpy(V, R, sizeof(R));
  } else {
    const double s = std::sin(theta), c = std::cos(theta);
    const double a = s / theta, b = (1 - c) / (theta * theta), g = (theta - s) / std::pow(theta, 3);
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        const double I = i == j ? 1.0 : 0.0;
        R[i][j] = (I + a * O[i][j]) + b * O2[i][j];
        V[i][j] = (I + b * O[i][j]) + g * O2[i][j];
      }
  }
  double vt[3];
  for (int i = 0; i < 3; i++) vt[i] = (V[i][0] * u[3] + V[i][1] * u[4]) + V[i][2] * u[5];
  const Se3 e = from_matrix(R, vt);
  // operator*: t = e.t + e.r * est.t; r = e.r * est.r; normalizeRotation
  Se3 r;
  double rt[3];
  rotate(e, est.t, rt);
  for (int a = 0; a < 3; a++) r.t[a] = e.t[a] + rt[a];
  r.w = e.w * est.w - e.x * est.x - e.y * est.y - e.z * est.z;
  r.x = e.w * est.x + e.x * est.w + e.y * est.z - e.z * est.y;
  r.y = e.w * est.y + e.y * est.w + e.z * est.x - e.x * est.z;
  r.z = e.w * est.z + e.z * est.w + e.x * est.y - e.y * est.x;
  normalize_rot(r);
  return r;
}

// Eigen 3.3 LDLT<MatrixXd> (Lower, diagonal pivoting) + solve; isPositive()
bool ldlt_solve(const double Hin[6][6], const double b[6], double x[6]) {
  double m[6][6];
  std::memcpy(m, Hin, sizeof(m));
  int tr[6];
  enum { Zero, PosSemi, NegSemi, Indef } sign = Zero;
  bool all_zero = false;
  for (int k = 0; k < 6; k++) {
    int big = k;
    double bv = std::fabs(m[k][k]);
    for (int i = k + 1; i < 6; i++)
      if (std::fabs(m[i][i]) > bv) {
        bv = std::fabs(m[i][i]);
        big = i;
      }
    tr[k] = big;
    if (k != big) {
      for (int j = 0; j < k; j++) std::swap(m[k][j], m[big][j]);
      for (int i = big + 1; i < 6; i++) std::swap(m[i][k], m[i][big]);
      std::swap(m[k][k], m[big][big]);
      for (int i = k + 1; i < big; i++) {
        const double tmp = m[i][k];
        m[i][k] = m[big][i];
        m[big][i] = tmp;
      }
    }
    double tmp[6];
    if (k > 0) {
      for (int j = 0; j < k; j++) tmp[j] = m[j][j] * m[k][j];
      double s = 0;
      for (int j = 0; j < k; j++) s = j ? s + m[k][j] * tmp[j] : m[k][j] * tmp[j];
      m[k][k] -= s;
      for (int i = k + 1; i < 6; i++) {
        double a = 0;
        for (int j = 0; j < k; j++) a = j ? a + m[i][j] * tmp[j] : m[i][j] * tmp[j];
        m[i][k] -= a;
      }
    }
    const double akk = m[k][k];
    const bool valid = std::fabs(akk) > 0;
    if (k == 0 && !valid) {
      all_zero = true;
      for (int j = 0; j < 6; j++) tr[j] = j;
      break;
    }
    if (valid)
      for (int i = k + 1; i < 6; i++) m[i][k] /= akk;
    if (sign == PosSemi) {
      if (akk < 0) sign = Indef;
    } else if (sign == NegSemi) {
      if (akk > 0) sign = Indef;
    } else if (sign == Zero) {
      if (akk > 0) sign = PosSemi;
      else if (akk < 0) sign = NegSemi;
    }
  }
  if (!(sign == PosSemi || sign == Zero)) return false;
  double y[6];
  for (int i = 0; i < 6; i++) y[i] = b[i];
  for (int k = 0; k < 6; k++) std::swap(y[k], y[tr[k]]);  // P b
  if (!all_zero)
    for (int i = 0; i < 6; i++)  // L y = Pb (unit lower)
      for (int j = 0; j < i; j++) y[i] -= m[i][j] * y[j];
  for (int i = 0; i < 6; i++) {  // D^+ (Eigen: |d| > DBL_MIN else 0)
    const double d = all_zero ? 0.0 : m[i][i];
    y[i] = std::fabs(d) > 2.2250738585072014e-308 ? y[i] / d : 0.0;
  }
  if (!all_zero)
    for (int i = 5; i >= 0; i--)  // L^T x = y
      for (int j = i + 1; j < 6; j++) y[i] -= m[j][i] * y[j];
  for (int k = 5; k >= 0; k--) std::swap(y[k], y[tr[k]]);  // P^T
  for (int i = 0; i < 6; i++) x[i] = y[i];
  return true;
}

struct Edge {
  double obs[2], X[3], inv;
  int idx;
  int level;     // 0 active, 1 outlier
  bool robust;
  double err[2];  // _error as last computed
};

struct Problem {
  double fx, fy, cx, cy, delta, dsqr;
  std::vector<Edge> edges;
  void compute_error(Edge& e, const Se3& s) const {  // EdgeSE3ProjectXYZOnlyPose::computeError
    double Xc[3];
    map_point(s, e.X, Xc);
    const double px = Xc[0] / Xc[2], py = Xc[1] / Xc[2];
    e.err[0] = e.obs[0] - (px * fx + cx);
    e.err[1] = e.obs[1] - (py * fy + cy);
  }
  static double chi2(const Edge& e) { return e.err[0] * (e.inv * e.err[0]) + e.err[1] * (e.inv * e.err[1]); }
  void robustify(double chi, double rho[2]) const {
    if (chi <= dsqr) {
      rho[0] = chi;
      rho[1] = 1.;
    } else {
      const double sq = std::sqrt(chi);
      rho[0] = 2 * sq * delta - dsqr;
      rho[1] = delta / sq;
    }
  }
  double active_chi(const Se3& s, bool recompute) {  // computeActiveErrors + activeRobustChi2
    double chi = 0;
    for (Edge& e : edges) {
      if (e.level != 0) continue;
      if (recompute) compute_error(e, s);
      const double c = chi2(e);
      if (e.robust) {
        double rho[2];
        robustify(c, rho);
        chi += rho[0];
      } else {
        chi += c;
      }
    }
    return chi;
  }
  // BlockSolver::buildSystem: H (lower triangle used by LDLT) and b
  void build(const Se3& s, double H[6][6], double b[6]) const {
    std::memset(H, 0, sizeof(double) * 36);
    std::memset(b, 0, sizeof(double) * 6);
    for (const Edge& e : edges) {
      if (e.level != 0) continue;
      double Xc[3];
      map_point(s, e.X, Xc);
      const double x = Xc[0], y = Xc[1], invz = 1.0 / Xc[2], invz2 = invz * invz;
      double J[2][6];
      J[0][0] = x * y * invz2 * fx;
      J[0][1] = -(1 + (x * x * invz2)) * fx;
      J[0][2] = y * invz * fx;
      J[0][3] = -invz * fx;
      J[0][4] = 0;
      J[0][5] = x * invz2 * fx;
      J[1][0] = (1 + y * y * invz2) * fy;
      J[1][1] = -x * y * invz2 * fy;
      J[1][2] = -x * invz * fy;
      J[1][3] = 0;
      J[1][4] = -invz * fy;
      J[1][5] = y * invz2 * fy;
      double r1 = 1.0;
      if (e.robust) {
        double rho[2];
        robustify(chi2(e), rho);
        r1 = rho[1];
      }
      const double w = r1 * e.inv;  // robustInformation = rho'(e) * Omega
      for (int i = 0; i < 6; i++) {
        const double a0 = J[0][i] * w, a1 = J[1][i] * w;
        for (int j = 0; j <= i; j++) H[i][j] += a0 * J[0][j] + a1 * J[1][j];
        b[i] -= ((r1 * J[0][i]) * e.inv) * e.err[0] + ((r1 * J[1][i]) * e.inv) * e.err[1];
      }
    }
    for (int i = 0; i < 6; i++)
      for (int j = i + 1; j < 6; j++) H[i][j] = H[j][i];
  }
};

// SparseOptimizer::optimize(iterations) with OptimizationAlgorithmLevenberg
void optimize(Problem& P, Se3& est, int iterations) {
  int nact = 0;
  for (const Edge& e : P.edges) nact += e.level == 0;
  if (nact == 0) return;  // no active vertex: optimize() returns -1 untouched
  double lambda = 0, ni = 2;
  int nbad = 0;
  double x[6] = {0, 0, 0, 0, 0, 0};  // the solver's _x: left as is when LDLT is not positive
  for (int it = 0; it < iterations; it++) {
    double cur = P.active_chi(est, true);
    const double ini = cur;
    double H[6][6], b[6];
    P.build(est, H, b);
    if (it == 0) {
      double md = 0;
      for (int j = 0; j < 6; j++) md = std::max(std::fabs(H[j][j]), md);
      lambda = 1e-5 * md;
      ni = 2;
      nbad = 0;
    }
    double rho = 0;
    int q = 0;
    do {
      const Se3 saved = est;
      double Hl[6][6];
      std::memcpy(Hl, H, sizeof(H));
      for (int j = 0; j < 6; j++) Hl[j][j] += lambda;
      const bool ok = ldlt_solve(Hl, b, x);
      est = oplus(est, x);
      double tmp = P.active_chi(est, true);
      if (!ok) tmp = std::numeric_limits<double>::max();
      rho = cur - tmp;
      double scale = 0;
      for (int j = 0; j < 6; j++) scale += x[j] * (lambda * x[j] + b[j]);
      scale += 1e-3;
      rho /= scale;
      if (rho > 0 && std::isfinite(tmp)) {
        double alpha = 1. - std::pow((2 * rho - 1), 3);
        alpha = std::min(alpha, 2. / 3.);
        lambda *= std::max(1. / 3., alpha);
        ni = 2;
        cur = tmp;
      } else {
        lambda *= ni;
        ni *= 2;
        est = saved;
      }
      q++;
    } while (rho < 0 && q < 10);
    if (q == 10 || rho == 0) return;
    if ((ini - cur) * 1e3 < ini) nbad++;
    else nbad = 0;
    if (nbad >= 3) return;
  }
}

}  // namespace

extern "C" int orc_pose_optimization(const orc_camera* cam, const float* Tcw_in, int n,
                                     const orc_keypoint* kps, const uint8_t* has_mp,
                                     const float* mp_pos, const float* inv_level_sigma2,
                                     float* Tcw_out, uint8_t* outlier, int* n_inliers) {
  Problem P;
  P.fx = cam->fx;
  P.fy = cam->fy;
  P.cx = cam->cx;
  P.cy = cam->cy;
  const float delta_mono = std::sqrt(5.991);  // Optimizer.cc:279
  P.delta = delta_mono;
  P.dsqr = P.delta * P.delta;
  for (int i = 0; i < n; i++) {
    if (!has_mp[i]) continue;
    outlier[i] = 0;
    Edge e;
    e.obs[0] = kps[i].x;
    e.obs[1] = kps[i].y;
    e.inv = inv_level_sigma2[kps[i].octave];
    for (int a = 0; a < 3; a++) e.X[a] = mp_pos[3 * i + a];
    e.idx = i;
    e.level = 0;
    e.robust = true;
    e.err[0] = e.err[1] = 0;
    P.edges.push_back(e);
  }
  std::memcpy(Tcw_out, Tcw_in, 16 * sizeof(float));
  const int n0 = (int)P.edges.size();
  if (n0 < 3) {
    *n_inliers = 0;
    return 0;
  }
  double R[3][3], t[3];
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) R[i][j] = Tcw_in[4 * i + j];
    t[i] = Tcw_in[4 * i + 3];
  }
  const Se3 init = from_matrix(R, t);
  Se3 est = init;
  const float chi2_mono = 5.991f;
  int nbad = 0;
  for (int it = 0; it < 4; it++) {
    est = init;  // vSE3->setEstimate(toSE3Quat(pFrame->mTcw)): the input pose every round
    optimize(P, est, 10);
    nbad = 0;
    for (Edge& e : P.edges) {
      if (outlier[e.idx]) P.compute_error(e, est);
      const float c2 = (float)Problem::chi2(e);
      if (c2 > chi2_mono) {
        outlier[e.idx] = 1;
        e.level = 1;
        nbad++;
      } else {
        outlier[e.idx] = 0;
        e.level = 0;
      }
      if (it == 2) e.robust = false;
    }
    if (n0 < 10) break;  // optimizer.edges().size() < 10
  }
  double Rf[3][3];
  to_matrix(est, Rf);
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) Tcw_out[4 * i + j] = (float)Rf[i][j];
    Tcw_out[4 * i + 3] = (float)est.t[i];
  }
  Tcw_out[12] = Tcw_out[13] = Tcw_out[14] = 0.f;
  Tcw_out[15] = 1.f;
  *n_inliers = n0 - nbad;
  return 0;
}
