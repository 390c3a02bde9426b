// pose.hip -- Optimizer::PoseOptimization (src/Optimizer.cc:243-457), monocular edges, on gfx950.
//
// One workgroup per frame. The frame's edges (keypoints holding a map point, in keypoint
// order = g2o's EdgeIDCompare order) are compacted once through LDS and then live in the
// registers of the thread that owns them (edge e -> thread e % T, slot e / T): observation,
// world point, information, level (inlier / outlier) and the last computed error. Every pass
// over the edges is one register sweep plus one block reduction:
//   * build pass: computeActiveErrors + activeRobustChi2 + BlockSolver::buildSystem fused
//     (error, Huber rho, analytic Jacobian, 21 lower-triangle H entries + 6 b entries + chi),
//   * trial pass: computeActiveErrors + activeRobustChi2 of a Levenberg trial,
//   * classification pass: the chi2 > 5.991 outlier test between the four rounds.
// The 6x6 LDLT solve, the SE3 exponential update and the Levenberg lambda schedule are
// uniform scalar work done redundantly by every thread (same inputs, same results), so the
// workgroup never leaves lockstep and needs no broadcast. Reductions: wave butterfly
// (__shfl_xor) then the waves' partials summed in wave order from LDS -- a fixed order, so
// the result is deterministic; it differs from g2o's sequential edge sum only in rounding
// (parity: pose within 1e-5, outlier flags and inlier count identical, tests/test_gpu_pose.py).
//
// g2o / Eigen semantics restated (see oracle/pose_ref.cpp for the citations):
//   EdgeSE3ProjectXYZOnlyPose computeError / linearizeOplus (types_six_dof_expmap.cpp:266-296),
//   OptimizationAlgorithmLevenberg::solve (optimization_algorithm_levenberg.cpp:61-189),
//   RobustKernelHuber (robust_kernel_impl.cpp:78-91), SE3Quat::exp and operator*
//   (se3quat.h:104-110,223-257), Eigen LDLT with diagonal pivoting (linear_solver_dense.h:104-111).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cfloat>
#include <cstring>
#include <vector>

#include "../../include/eao_accel.h"
#include "common.h"
#include "orb.h"

namespace eao {
namespace {

constexpr int kRed = 28;  // 21 lower-triangle H entries, 6 b entries, chi
constexpr int kMaxLevels = 32;

struct PoseArgs {
  double fx, fy, cx, cy;
  double delta, dsqr;  // Huber delta = (float)sqrt(5.991) (Optimizer.cc:279)
  float inv_sigma2[kMaxLevels];
  int nlevels;
};

struct Se3 {
  double w, x, y, z, t0, t1, t2;
};

__device__ __forceinline__ void normalize_rot(Se3& s) {
  if (s.w < 0) {
    s.w = -s.w;
    s.x = -s.x;
    s.y = -s.y;
    s.z = -s.z;
  }
  const double n = sqrt((s.x * s.x + s.z * s.z) + (s.y * s.y + s.w * s.w));
  s.x = s.x / n;
  s.y = s.y / n;
  s.z = s.z / n;
  s.w = s.w / n;
}

// SE3Quat(Matrix3d R, t): Eigen's Quaternion(Matrix3) branches, then normalizeRotation
__device__ Se3 se3_from(const double R[9], double t0, double t1, double t2) {
  Se3 s;
  double tr = (R[0] + R[4]) + R[8];
  if (tr > 0) {
    tr = sqrt(tr + 1.0);
    s.w = 0.5 * tr;
    tr = 0.5 / tr;
    s.x = (R[7] - R[5]) * tr;
    s.y = (R[2] - R[6]) * tr;
    s.z = (R[3] - R[1]) * tr;
  } else {
    int i = 0;
    if (R[4] > R[0]) i = 1;
    if (R[8] > R[4 * i]) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    double c[3];
    tr = sqrt(R[4 * i] - R[4 * j] - R[4 * k] + 1.0);
    c[i] = 0.5 * tr;
    tr = 0.5 / tr;
    s.w = (R[3 * k + j] - R[3 * j + k]) * tr;
    c[j] = (R[3 * j + i] + R[3 * i + j]) * tr;
    c[k] = (R[3 * k + i] + R[3 * i + k]) * tr;
    s.x = c[0];
    s.y = c[1];
    s.z = c[2];
  }
  s.t0 = t0;
  s.t1 = t1;
  s.t2 = t2;
  normalize_rot(s);
  return s;
}

// q * v (Eigen: uv = 2 vec x v; v + w uv + vec x uv)
__device__ __forceinline__ void qrot(const Se3& s, double v0, double v1, double v2, double& o0, double& o1,
                                     double& o2) {
  double u0 = s.y * v2 - s.z * v1, u1 = s.z * v0 - s.x * v2, u2 = s.x * v1 - s.y * v0;
  u0 += u0;
  u1 += u1;
  u2 += u2;
  o0 = v0 + s.w * u0 + (s.y * u2 - s.z * u1);
  o1 = v1 + s.w * u1 + (s.z * u0 - s.x * u2);
  o2 = v2 + s.w * u2 + (s.x * u1 - s.y * u0);
}

// VertexSE3Expmap::oplusImpl: SE3Quat::exp(u) * est
__device__ Se3 se3_oplus(const Se3& est, const double u[6]) {
  const double o0 = u[0], o1 = u[1], o2 = u[2];
  const double theta = sqrt((o0 * o0 + o1 * o1) + o2 * o2);
  const double O[9] = {0, -o2, o1, o2, 0, -o0, -o1, o0, 0};
  double O2[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++)
      O2[3 * i + j] = (O[3 * i] * O[j] + O[3 * i + 1] * O[3 + j]) + O[3 * i + 2] * O[6 + j];
  double R[9], V[9];
  if (theta < 0.00001) {
    for (int i = 0; i < 9; i++) R[i] = ((i % 4 == 0 ? 1.0 : 0.0) + O[i]) + O2[i];
    for (int i = 0; i < 9; i++) V[i] = R[i];
  } else {
    const double sn = sin(theta), cs = cos(theta);
    const double a = sn / theta, b = (1 - cs) / (theta * theta), g = (theta - sn) / pow(theta, 3.0);
    for (int i = 0; i < 9; i++) {
      const double I = i % 4 == 0 ? 1.0 : 0.0;
      R[i] = (I + a * O[i]) + b * O2[i];
      V[i] = (I + b * O[i]) + g * O2[i];
    }
  }
  const Se3 e = se3_from(R, (V[0] * u[3] + V[1] * u[4]) + V[2] * u[5], (V[3] * u[3] + V[4] * u[4]) + V[5] * u[5],
                         (V[6] * u[3] + V[7] * u[4]) + V[8] * u[5]);
  Se3 r;
  double a0, a1, a2;
  qrot(e, est.t0, est.t1, est.t2, a0, a1, a2);
  r.t0 = e.t0 + a0;
  r.t1 = e.t1 + a1;
  r.t2 = e.t2 + a2;
  r.w = e.w * est.w - e.x * est.x - e.y * est.y - e.z * est.z;
  r.x = e.w * est.x + e.x * est.w + e.y * est.z - e.z * est.y;
  r.y = e.w * est.y + e.y * est.w + e.z * est.x - e.x * est.z;
  r.z = e.w * est.z + e.z * est.w + e.x * est.y - e.y * est.x;
  normalize_rot(r);
  return r;
}

// Eigen 3.3 LDLT (Lower, diagonal pivoting) of (H + lambda I) x = b, H read from the LDS copy
// of the reduced system (lower triangle, packed), + solve. Every index is a compile-time
// constant after unrolling (pivot swaps as predicated moves), so the 6x6 stays in registers.
// Returns false when not isPositive(); x is then left as it was (the solver's _x buffer).
__device__ __forceinline__ void cswap(bool p, double& a, double& b) {
  const double t = a;
  a = p ? b : a;
  b = p ? t : b;
}

__device__ __forceinline__ bool ldlt_solve(const double* sys, double lambda, double* x) {
  double m[36], y[6];
#pragma unroll
  for (int i = 0, q = 0; i < 6; i++)
#pragma unroll
    for (int j = 0; j <= i; j++, q++) {
      m[6 * i + j] = sys[q];
      m[6 * j + i] = sys[q];
    }
#pragma unroll
  for (int i = 0; i < 6; i++) {
    m[7 * i] += lambda;
    y[i] = sys[21 + i];
  }
  int tr[6];
  int sign = 0;  // 0 zero, 1 positive semi-definite, 2 negative semi-definite, 3 indefinite
  bool all_zero = false;
#pragma unroll
  for (int k = 0; k < 6; k++) {
    tr[k] = k;
    if (all_zero) continue;
    int big = k;
    double bv = fabs(m[7 * k]);
#pragma unroll
    for (int i = k + 1; i < 6; i++)
      if (fabs(m[7 * i]) > bv) {
        bv = fabs(m[7 * i]);
        big = i;
      }
    tr[k] = big;
#pragma unroll
    for (int c = k + 1; c < 6; c++) {
      const bool p = big == c;
#pragma unroll
      for (int j = 0; j < k; j++) cswap(p, m[6 * k + j], m[6 * c + j]);
#pragma unroll
      for (int i = c + 1; i < 6; i++) cswap(p, m[6 * i + k], m[6 * i + c]);
      cswap(p, m[7 * k], m[7 * c]);
#pragma unroll
      for (int i = k + 1; i < c; i++) {
        const double t = m[6 * i + k];
        m[6 * i + k] = p ? m[6 * c + i] : m[6 * i + k];
        m[6 * c + i] = p ? t : m[6 * c + i];
      }
    }
    if (k > 0) {
      double tmp[6];
#pragma unroll
      for (int j = 0; j < k; j++) tmp[j] = m[7 * j] * m[6 * k + j];
      double s = m[6 * k] * tmp[0];
#pragma unroll
      for (int j = 1; j < k; j++) s = s + m[6 * k + j] * tmp[j];
      m[7 * k] -= s;
#pragma unroll
      for (int i = k + 1; i < 6; i++) {
        double a = m[6 * i] * tmp[0];
#pragma unroll
        for (int j = 1; j < k; j++) a = a + m[6 * i + j] * tmp[j];
        m[6 * i + k] -= a;
      }
    }
    const double akk = m[7 * k];
    const bool valid = fabs(akk) > 0;
    if (k == 0 && !valid) {
      all_zero = true;
      tr[0] = 0;
      continue;
    }
    if (valid) {
#pragma unroll
      for (int i = k + 1; i < 6; i++) m[6 * i + k] = m[6 * i + k] / akk;
    }
    if (sign == 1) {
      if (akk < 0) sign = 3;
    } else if (sign == 2) {
      if (akk > 0) sign = 3;
    } else if (sign == 0) {
      if (akk > 0) sign = 1;
      else if (akk < 0) sign = 2;
    }
  }
  if (!(sign == 1 || sign == 0)) return false;
#pragma unroll
  for (int k = 0; k < 6; k++)
#pragma unroll
    for (int c = k + 1; c < 6; c++) cswap(tr[k] == c, y[k], y[c]);
  if (!all_zero) {
#pragma unroll
    for (int i = 0; i < 6; i++)
#pragma unroll
      for (int j = 0; j < i; j++) y[i] -= m[6 * i + j] * y[j];
  }
#pragma unroll
  for (int i = 0; i < 6; i++) {
    const double d = all_zero ? 0.0 : m[7 * i];
    y[i] = fabs(d) > DBL_MIN ? y[i] / d : 0.0;
  }
  if (!all_zero) {
#pragma unroll
    for (int i = 5; i >= 0; i--)
#pragma unroll
      for (int j = i + 1; j < 6; j++) y[i] -= m[6 * j + i] * y[j];
  }
#pragma unroll
  for (int k = 5; k >= 0; k--)
#pragma unroll
    for (int c = k + 1; c < 6; c++) cswap(tr[k] == c, y[k], y[c]);
#pragma unroll
  for (int i = 0; i < 6; i++) x[i] = y[i];
  return true;
}

// wave butterfly of NV doubles, the waves' partials to LDS (buffer `buf`, alternating so one
// barrier per reduction suffices)
template <int T, int NV>
__device__ __forceinline__ double* block_partials(double (&v)[NV], double* red, int& buf) {
  constexpr int NW = T / 64;
#pragma unroll
  for (int k = 0; k < NV; k++)
    for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o, 64);
  double* r = red + buf * (NW * kRed);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int k = 0; k < NV; k++) r[w * kRed + k] = v[k];
  }
  __syncthreads();
  buf ^= 1;
  return r;
}

// every thread: the block sum of one value (partials summed in wave order)
template <int T>
__device__ __forceinline__ double block_sum1(double v, double* red, int& buf) {
  constexpr int NW = T / 64;
  double a[1] = {v};
  const double* r = block_partials<T, 1>(a, red, buf);
  double s = r[0];
  for (int q = 1; q < NW; q++) s = s + r[q * kRed];
  return s;
}

// DPP row_shr:n of a double (both dwords); lanes shifted in from outside the 16-lane row read 0
template <int N>
__device__ __forceinline__ double row_shr(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffff), 0x110 + N, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x110 + N, 0xF, 0xF, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// the block sum of NV doubles into out[0..NV) (LDS): per 16-lane row a Hillis-Steele scan by
// DPP (row sum in the row's last lane), the rows' sums to LDS, then thread k < NV adds the
// block's 4 * NW row sums of value k in row order -- a fixed order, so deterministic. Ends with
// a barrier: out is then visible to the whole block.
template <int T, int NV>
__device__ __forceinline__ void block_sum_rows(double (&v)[NV], double* part, double* out) {
  constexpr int NR = T / 16;
#pragma unroll
  for (int k = 0; k < NV; k++) {
    v[k] += row_shr<1>(v[k]);
    v[k] += row_shr<2>(v[k]);
    v[k] += row_shr<4>(v[k]);
    v[k] += row_shr<8>(v[k]);
  }
  const int r = threadIdx.x >> 4;
  if ((threadIdx.x & 15) == 15) {
#pragma unroll
    for (int k = 0; k < NV; k++) part[k * NR + r] = v[k];
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    const double* p = part + threadIdx.x * NR;
    double s = p[0];
    for (int q = 1; q < NR; q++) s = s + p[q];
    out[threadIdx.x] = s;
  }
  __syncthreads();
}

template <int EPT>
struct Edges {
  float ox[EPT], oy[EPT], X[EPT], Y[EPT], Z[EPT], inv[EPT];
  int idx[EPT];
  uint32_t outl;  // bit k: edge slot k is level 1 (outlier)
};


// EdgeSE3ProjectXYZOnlyPose::computeError at s; the camera-frame point is returned too
template <int EPT>
__device__ __forceinline__ void edge_error(const Edges<EPT>& E, int k, const Se3& s, const PoseArgs& a,
                                           double& e0, double& e1, double& xc, double& yc, double& zc) {
  qrot(s, (double)E.X[k], (double)E.Y[k], (double)E.Z[k], xc, yc, zc);
  xc = xc + s.t0;
  yc = yc + s.t1;
  zc = zc + s.t2;
  const double px = xc / zc, py = yc / zc;
  e0 = (double)E.ox[k] - (px * a.fx + a.cx);
  e1 = (double)E.oy[k] - (py * a.fy + a.cy);
}

__device__ __forceinline__ double chi2_of(double e0, double e1, double inv) {
  return e0 * (inv * e0) + e1 * (inv * e1);
}

template <int T, int EPT>
__global__ void __launch_bounds__(T) k_pose_opt(PoseArgs a, int cap, const float* __restrict__ Tin,
                                                const int* __restrict__ counts, const eao_keypoint_dev* __restrict__ kps,
                                                const uint8_t* __restrict__ has_mp, const float* __restrict__ mp_pos,
                                                float* __restrict__ Tout, uint8_t* __restrict__ outlier,
                                                int* __restrict__ n_inliers) {
  constexpr int NW = T / 64;
  __shared__ int s_list[T * EPT];
  __shared__ int s_wcnt[NW];
  __shared__ double s_red[2 * NW * kRed];
  __shared__ double s_part[kRed * (T / 16)];
  // two reduced systems (21 H lower packed | 6 b | chi): the current one and a trial's
  __shared__ double s_sysbuf[2][kRed];
  const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n = min(counts[f], cap);
  const float* T0 = Tin + 16 * f;
  float* T1 = Tout + 16 * f;
  const eao_keypoint_dev* K = kps + (size_t)f * cap;
  const uint8_t* H = has_mp + (size_t)f * cap;
  const float* MP = mp_pos + (size_t)f * cap * 3;
  uint8_t* OUT = outlier + (size_t)f * cap;

  // --- compaction of the edges (keypoints with a map point) in keypoint order
  int n0 = 0;
  for (int base = 0; base < n; base += T) {
    const int i = base + tid;
    const bool p = i < n && H[i];
    const uint64_t m = ballot(p);
    if (lane == 0) s_wcnt[w] = popc64(m);
    __syncthreads();
    int off = n0;
    for (int q = 0; q < w; q++) off += s_wcnt[q];
    int tot = n0;
    for (int q = 0; q < NW; q++) tot += s_wcnt[q];
    if (p) {
      const int pos = off + popc64(m & lanes_below());
      if (pos < T * EPT) s_list[pos] = i;
      OUT[i] = 0;  // pFrame->mvbOutlier[i] = false (Optimizer.cc:295)
    }
    n0 = tot;
    __syncthreads();
  }
  if (n0 > T * EPT) n0 = T * EPT;  // the host picks T * EPT >= cap
  if (n0 < 3) {  // Optimizer.cc:370-371: pose left as it is
    if (tid < 16) T1[tid] = T0[tid];
    if (tid == 0) n_inliers[f] = 0;
    return;
  }
  Edges<EPT> E;
  E.outl = 0;
#pragma unroll
  for (int k = 0; k < EPT; k++) {
    const int e = tid + k * T;
    E.idx[k] = -1;
    E.ox[k] = E.oy[k] = E.X[k] = E.Y[k] = E.Z[k] = E.inv[k] = 0.f;
    if (e < n0) {
      const int i = s_list[e];
      E.idx[k] = i;
      E.ox[k] = K[i].x;
      E.oy[k] = K[i].y;
      const int oct = K[i].octave;
      E.inv[k] = a.inv_sigma2[oct < 0 ? 0 : (oct >= a.nlevels ? a.nlevels - 1 : oct)];
      E.X[k] = MP[3 * i];
      E.Y[k] = MP[3 * i + 1];
      E.Z[k] = MP[3 * i + 2];
    }
  }
  double R0[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) R0[3 * i + j] = (double)T0[4 * i + j];
  const Se3 init = se3_from(R0, (double)T0[3], (double)T0[7], (double)T0[11]);
  Se3 est = init;
  // the estimate of the last computeActiveErrors: the errors g2o keeps in its edges (and the
  // outlier test reads for level-0 edges) are recomputed from it instead of being stored
  Se3 elast = init;
  bool robust = true;
  int buf = 0;
  int nbad_total = 0;

  for (int round = 0; round < 4; round++) {
    est = init;  // every round restarts from pFrame->mTcw (Optimizer.cc:383)
    double cnt = 0;
#pragma unroll
    for (int k = 0; k < EPT; k++)
      if (E.idx[k] >= 0 && !((E.outl >> k) & 1)) cnt += 1;
    cnt = block_sum1<T>(cnt, s_red, buf);
    if (cnt > 0) {
      // ---- SparseOptimizer::optimize(10) with OptimizationAlgorithmLevenberg. A pass at an
      // estimate gives computeActiveErrors + activeRobustChi2 + buildSystem at once; a trial's
      // pass is therefore also the next iteration's build when the trial is accepted (solve()
      // would recompute exactly those errors at exactly that estimate), so each Levenberg
      // trial costs one pass and only the first iteration has a pass of its own.
      int cur_buf = 0;
      auto build_pass = [&](const Se3& at, double* out) {
        double acc[kRed];
#pragma unroll
        for (int q = 0; q < kRed; q++) acc[q] = 0;
#pragma unroll
        for (int k = 0; k < EPT; k++) {
          if (E.idx[k] < 0 || ((E.outl >> k) & 1)) continue;
          double e0, e1, xc, yc, zc;
          edge_error(E, k, at, a, e0, e1, xc, yc, zc);
          const double inv = (double)E.inv[k];
          const double c = chi2_of(e0, e1, inv);
          double r1 = 1.0;
          if (robust) {
            if (c <= a.dsqr) {
              acc[27] += c;
            } else {
              const double sq = sqrt(c);
              acc[27] += 2 * sq * a.delta - a.dsqr;
              r1 = a.delta / sq;
            }
          } else {
            acc[27] += c;
          }
          const double invz = 1.0 / zc, invz2 = invz * invz;
          double J0[6], J1[6];
          J0[0] = xc * yc * invz2 * a.fx;
          J0[1] = -(1 + (xc * xc * invz2)) * a.fx;
          J0[2] = yc * invz * a.fx;
          J0[3] = -invz * a.fx;
          J0[4] = 0;
          J0[5] = xc * invz2 * a.fx;
          J1[0] = (1 + yc * yc * invz2) * a.fy;
          J1[1] = -xc * yc * invz2 * a.fy;
          J1[2] = -xc * invz * a.fy;
          J1[3] = 0;
          J1[4] = -invz * a.fy;
          J1[5] = yc * invz2 * a.fy;
          const double wgt = r1 * inv;
          int q = 0;
#pragma unroll
          for (int i = 0; i < 6; i++) {
            const double a0 = J0[i] * wgt, a1 = J1[i] * wgt;
#pragma unroll
            for (int j = 0; j <= i; j++) acc[q++] += a0 * J0[j] + a1 * J1[j];
            acc[21 + i] -= ((r1 * J0[i]) * inv) * e0 + ((r1 * J1[i]) * inv) * e1;
          }
        }
        block_sum_rows<T, kRed>(acc, s_part, out);
      };
      // one call site for the pass, the solve and the update (register pressure): a flat loop
      // whose first trip is the first iteration's own pass
      double x[6] = {0, 0, 0, 0, 0, 0};
      double lambda = 0, ni = 2, cur = 0, ini = 0;
      int nbad = 0, it = 0, qn = 0;
      bool first = true, ok = true;
      Se3 saved = est;
      for (;;) {
        double* target = s_sysbuf[first ? cur_buf : (cur_buf ^ 1)];
        if (!first) {
          saved = est;
          ok = ldlt_solve(s_sysbuf[cur_buf], lambda, x);
          est = se3_oplus(est, x);
        }
        build_pass(est, target);
        elast = est;
        if (first) {  // iteration 0: computeLambdaInit from the diagonal of H
          first = false;
          cur = target[27];
          ini = cur;
          double md = 0;
#pragma unroll
          for (int j = 0; j < 6; j++) md = fmax(fabs(target[j * (j + 3) / 2]), md);
          lambda = 1e-5 * md;
          ni = 2;
          nbad = 0;
          qn = 0;
          continue;
        }
        const double* sys = s_sysbuf[cur_buf];
        const double tmp = ok ? target[27] : DBL_MAX;
        double rho = cur - tmp;
        double scale = 0;
#pragma unroll
        for (int j = 0; j < 6; j++) scale += x[j] * (lambda * x[j] + sys[21 + j]);
        scale += 1e-3;
        rho /= scale;
        if (rho > 0 && isfinite(tmp)) {
          double alpha = 1. - pow((2 * rho - 1), 3.0);
          alpha = fmin(alpha, 2. / 3.);
          lambda *= fmax(1. / 3., alpha);
          ni = 2;
          cur = tmp;
          cur_buf ^= 1;  // the trial's system is the next iteration's
        } else {
          lambda *= ni;
          ni *= 2;
          est = saved;
        }
        qn++;
        if (rho < 0 && qn < 10) continue;  // another trial of the same iteration
        if (qn == 10 || rho == 0) break;
        if ((ini - cur) * 1e3 < ini) nbad++;
        else nbad = 0;
        if (nbad >= 3) break;
        if (++it >= 10) break;
        ini = cur;  // the next iteration's computeActiveErrors at est: the current system
        qn = 0;
      }
    }
    // ---- classification (Optimizer.cc:387-415): level-0 edges test the error of the last
    // computeActiveErrors, level-1 edges computeError() at the final estimate
    double nb = 0;
#pragma unroll
    for (int k = 0; k < EPT; k++) {
      if (E.idx[k] < 0) continue;
      const bool was_out = (E.outl >> k) & 1;
      double e0, e1, xc, yc, zc;
      edge_error(E, k, was_out ? est : elast, a, e0, e1, xc, yc, zc);
      const float c2 = (float)chi2_of(e0, e1, (double)E.inv[k]);
      if (c2 > 5.991f) {
        E.outl |= 1u << k;
        nb += 1;
      } else {
        E.outl &= ~(1u << k);
      }
    }
    if (round == 2) robust = false;
    nbad_total = (int)block_sum1<T>(nb, s_red, buf);
    if (n0 < 10) break;  // optimizer.edges().size() < 10
  }
#pragma unroll
  for (int k = 0; k < EPT; k++)
    if (E.idx[k] >= 0) OUT[E.idx[k]] = (E.outl >> k) & 1;
  if (tid == 0) {
    // Converter::toCvMat(SE3Quat): toRotationMatrix + translation, cast to float
    const double tx = 2 * est.x, ty = 2 * est.y, tz = 2 * est.z;
    const double twx = tx * est.w, twy = ty * est.w, twz = tz * est.w;
    const double txx = tx * est.x, txy = ty * est.x, txz = tz * est.x;
    const double tyy = ty * est.y, tyz = tz * est.y, tzz = tz * est.z;
    T1[0] = (float)(1 - (tyy + tzz));
    T1[1] = (float)(txy - twz);
    T1[2] = (float)(txz + twy);
    T1[3] = (float)est.t0;
    T1[4] = (float)(txy + twz);
    T1[5] = (float)(1 - (txx + tzz));
    T1[6] = (float)(tyz - twx);
    T1[7] = (float)est.t1;
    T1[8] = (float)(txz - twy);
    T1[9] = (float)(tyz + twx);
    T1[10] = (float)(1 - (txx + tyy));
    T1[11] = (float)est.t2;
    T1[12] = T1[13] = T1[14] = 0.f;
    T1[15] = 1.f;
    n_inliers[f] = n0 - nbad_total;
  }
}

}  // namespace

struct PoseEngine {
  int dev = 0, max_kps = 0, max_batch = 0;
  hipStream_t stream = nullptr;
  float* d_T = nullptr;       // [2][16]
  eao_keypoint_dev* d_kps = nullptr;
  uint8_t* d_has = nullptr;
  float* d_pos = nullptr;
  uint8_t* d_out = nullptr;
  int* d_i = nullptr;         // [0] count, [1] inliers
  float* h_T = nullptr;       // pinned [16] + int
  ~PoseEngine() {
    if (d_T) (void)hipFree(d_T);
    if (d_kps) (void)hipFree(d_kps);
    if (d_has) (void)hipFree(d_has);
    if (d_pos) (void)hipFree(d_pos);
    if (d_out) (void)hipFree(d_out);
    if (d_i) (void)hipFree(d_i);
    if (h_T) (void)hipHostFree(h_T);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

static int pose_args(const eao_camera* cam, const float* inv_sigma2, int nlevels, PoseArgs& a) {
  if (!cam || !inv_sigma2 || nlevels < 1 || nlevels > kMaxLevels) {
    set_error("eao_pose: camera / inv_level_sigma2 / nlevels (1..32) invalid");
    return EAO_E_ARG;
  }
  a.fx = cam->fx;
  a.fy = cam->fy;
  a.cx = cam->cx;
  a.cy = cam->cy;
  const float delta = std::sqrt(5.991);  // const float deltaMono = sqrt(5.991)
  a.delta = delta;
  a.dsqr = a.delta * a.delta;
  for (int l = 0; l < kMaxLevels; l++) a.inv_sigma2[l] = l < nlevels ? inv_sigma2[l] : 0.f;
  a.nlevels = nlevels;
  return EAO_OK;
}

static int pose_launch(const PoseArgs& a, int nframes, int cap, const float* dT, const int* dn,
                       const eao_keypoint_dev* dk, const uint8_t* dh, const float* dp, float* dTo, uint8_t* dout,
                       int* dni, hipStream_t s) {
  if (cap <= 256 * 4)
    hipLaunchKernelGGL((k_pose_opt<256, 4>), dim3(nframes), dim3(256), 0, s, a, cap, dT, dn, dk, dh, dp, dTo, dout,
                       dni);
  else if (cap <= 256 * 8)
    hipLaunchKernelGGL((k_pose_opt<256, 8>), dim3(nframes), dim3(256), 0, s, a, cap, dT, dn, dk, dh, dp, dTo,
                       dout, dni);
  else if (cap <= 1024 * 8)
    hipLaunchKernelGGL((k_pose_opt<1024, 8>), dim3(nframes), dim3(1024), 0, s, a, cap, dT, dn, dk, dh, dp, dTo,
                       dout, dni);
  else {
    set_error("eao_pose: more than 8192 keypoints per frame");
    return EAO_E_CAPACITY;
  }
  EAO_HIP_CHECK(hipGetLastError());
  return EAO_OK;
}

}  // namespace eao

using namespace eao;

struct eao_pose {
  PoseEngine e;
};

extern "C" {

int eao_pose_create(int device, int max_kps, int max_batch, eao_pose** out) {
  if (!out) return EAO_E_ARG;
  *out = nullptr;
  if (!eao_device_ok(device)) {
    set_error("no usable gfx950 device (the engine has no CPU fallback)");
    return EAO_E_NODEVICE;
  }
  if (max_kps < 1 || max_kps > 8192 || max_batch < 1) {
    set_error("eao_pose_create: max_kps outside [1, 8192] or max_batch < 1");
    return EAO_E_ARG;
  }
  eao_pose* p = new eao_pose();
  PoseEngine& e = p->e;
  e.dev = device;
  e.max_kps = max_kps;
  e.max_batch = max_batch;
  auto fail = [&](hipError_t r, const char* what) {
    set_error(std::string("eao_pose_create: ") + what + ": " + hipGetErrorString(r));
    delete p;
    return EAO_E_HIP;
  };
  hipError_t r;
  if ((r = hipSetDevice(device)) != hipSuccess) return fail(r, "hipSetDevice");
  if ((r = hipStreamCreateWithFlags(&e.stream, hipStreamNonBlocking)) != hipSuccess) return fail(r, "stream");
  if ((r = hipMalloc(&e.d_T, sizeof(float) * 32)) != hipSuccess) return fail(r, "hipMalloc");
  if ((r = hipMalloc(&e.d_kps, sizeof(eao_keypoint_dev) * max_kps)) != hipSuccess) return fail(r, "hipMalloc");
  if ((r = hipMalloc(&e.d_has, max_kps)) != hipSuccess) return fail(r, "hipMalloc");
  if ((r = hipMalloc(&e.d_pos, sizeof(float) * 3 * max_kps)) != hipSuccess) return fail(r, "hipMalloc");
  if ((r = hipMalloc(&e.d_out, max_kps)) != hipSuccess) return fail(r, "hipMalloc");
  if ((r = hipMalloc(&e.d_i, sizeof(int) * 2)) != hipSuccess) return fail(r, "hipMalloc");
  if ((r = hipHostMalloc(&e.h_T, sizeof(float) * 20)) != hipSuccess) return fail(r, "hipHostMalloc");
  *out = p;
  return EAO_OK;
}

int eao_pose_destroy(eao_pose* p) {
  delete p;
  return EAO_OK;
}

int eao_pose_optimization(eao_pose* p, const eao_camera* cam, const float* Tcw_in, int n,
                          const eao_keypoint* kps_un, const uint8_t* has_mp, const float* mp_pos,
                          const float* inv_level_sigma2, int nlevels, float* Tcw_out, uint8_t* outlier,
                          int32_t* n_inliers) {
  if (!p || !Tcw_in || !Tcw_out || !n_inliers || n < 0 || n > p->e.max_kps ||
      (n > 0 && (!kps_un || !has_mp || !mp_pos || !outlier))) {
    set_error("eao_pose_optimization: bad arguments (n outside [0, max_kps] or null buffer)");
    return EAO_E_ARG;
  }
  PoseArgs a;
  int rc = pose_args(cam, inv_level_sigma2, nlevels, a);
  if (rc) return rc;
  PoseEngine& e = p->e;
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  hipStream_t s = e.stream;
  std::memcpy(e.h_T, Tcw_in, sizeof(float) * 16);
  reinterpret_cast<int*>(e.h_T)[16] = n;
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_T, e.h_T, sizeof(float) * 16, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_i, e.h_T + 16, sizeof(int), hipMemcpyHostToDevice, s));
  if (n > 0) {
    EAO_HIP_CHECK(hipMemcpyAsync(e.d_kps, kps_un, sizeof(eao_keypoint) * n, hipMemcpyHostToDevice, s));
    EAO_HIP_CHECK(hipMemcpyAsync(e.d_has, has_mp, n, hipMemcpyHostToDevice, s));
    EAO_HIP_CHECK(hipMemcpyAsync(e.d_pos, mp_pos, sizeof(float) * 3 * n, hipMemcpyHostToDevice, s));
    EAO_HIP_CHECK(hipMemcpyAsync(e.d_out, outlier, n, hipMemcpyHostToDevice, s));
  }
  rc = pose_launch(a, 1, n > 0 ? n : 1, e.d_T, e.d_i, e.d_kps, e.d_has, e.d_pos, e.d_T + 16, e.d_out, e.d_i + 1, s);
  if (rc) return rc;
  EAO_HIP_CHECK(hipMemcpyAsync(e.h_T, e.d_T + 16, sizeof(float) * 16, hipMemcpyDeviceToHost, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.h_T + 17, e.d_i + 1, sizeof(int), hipMemcpyDeviceToHost, s));
  if (n > 0) EAO_HIP_CHECK(hipMemcpyAsync(outlier, e.d_out, n, hipMemcpyDeviceToHost, s));
  EAO_HIP_CHECK(hipStreamSynchronize(s));
  std::memcpy(Tcw_out, e.h_T, sizeof(float) * 16);
  *n_inliers = reinterpret_cast<int*>(e.h_T)[17];
  return EAO_OK;
}

int eao_pose_optimization_batch_device(eao_pose* p, const eao_camera* cam, int nframes, int cap,
                                       const float* d_Tcw_in, const int32_t* d_counts,
                                       const eao_keypoint* d_kps_un, const uint8_t* d_has_mp,
                                       const float* d_mp_pos, const float* inv_level_sigma2, int nlevels,
                                       float* d_Tcw_out, uint8_t* d_outlier, int32_t* d_n_inliers,
                                       void* stream) {
  if (!p || nframes < 0 || cap < 1 || cap > 8192 || (nframes > 0 && (!d_Tcw_in || !d_counts || !d_kps_un ||
                                                                      !d_has_mp || !d_mp_pos || !d_Tcw_out ||
                                                                      !d_outlier || !d_n_inliers))) {
    set_error("eao_pose_optimization_batch_device: bad arguments (cap outside [1, 8192] or null buffer)");
    return EAO_E_ARG;
  }
  if (nframes == 0) return EAO_OK;
  PoseArgs a;
  int rc = pose_args(cam, inv_level_sigma2, nlevels, a);
  if (rc) return rc;
  EAO_HIP_CHECK(hipSetDevice(p->e.dev));
  hipStream_t s = stream ? (hipStream_t)stream : p->e.stream;
  return pose_launch(a, nframes, cap, d_Tcw_in, d_counts, (const eao_keypoint_dev*)d_kps_un, d_has_mp, d_mp_pos,
                     d_Tcw_out, d_outlier, d_n_inliers, s);
}

}  // extern "C"
