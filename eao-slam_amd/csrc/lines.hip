// lines.hip -- per-frame line detection of the EAO Frame on gfx950: the MI355X replacement
// of line_lbd_detect::detect_raw_lines + filter_lines (reference src/Frame.cc:324-328,
// src/line_detect/line_lbd_allclass.cpp:137-214) with the tracker's single octave
// (Tracking.cc:161-163): GaussianBlur(5x5, sigma 1), then EDLineDetector::EDline
// (src/line_detect/libs/binary_descriptor.cpp:1583-2906) and OctaveKeyLines' endpoint
// ordering (:866-887, 1073-1141); lines longer than min_length are kept.
//
// Pipeline per batch of HBM-resident gray frames:
//   k_line_blur     64x16 output tiles: the 8U fixed-point separable 5-tap Gaussian
//                   (taps cvRound(k * 256), REFLECT_101, columns (s + 2^15) >> 16)
//   k_line_grad     one thread per pixel: Sobel 3x3 (REFLECT_101) dx, dy; code =
//                   thresholded |dx| + |dy| over 4 (cvRound) | Horizontal bit
//   k_line_anchors  one workgroup per frame, a thread per candidate column: the anchors in the
//                   reference's column-major scan order (w outer, h inner, step 2) from a
//                   block scan of the per-column counts, rows walked with coalesced reads
//   k_edge_draw     one wave per frame: the anchor walks (edge map as an LDS bitmap), the
//                   kept chains assembled by the whole wave
//   k_edlines       8 waves per frame, a wave per chain (chains are independent): least-
//                   squares fits and normal-equation sums as wave reductions (integer data,
//                   exact in double), the extension walk in wave-uniform control flow,
//                   LineValidation_'s per-pixel directions in parallel, nfa, endpoints,
//                   ordering and the length filter; the chains' lines then placed in chain
//                   order by a block scan of the per-chain counts
// The walks are sequential per frame by the reference's definition (each anchor's chain
// depends on the edge map left by all earlier ones); frames run concurrently.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <vector>

#include "../../include/eao_accel.h"
#include "common.h"

namespace eao {

constexpr int LN_HORIZ = 0x8000;  // code bit: dirImg_ == Horizontal (|dx| < |dy|)
constexpr int LN_UP = 1, LN_RIGHT = 2, LN_DOWN = 3, LN_LEFT = 4;
constexpr int LN_GRAD_TH = 80, LN_ANCHOR_TH = 8, LN_MIN_LEN = 15, LN_TRY = 6, LN_SKIP = 2;
constexpr int LN_WAVES = 8;  // k_edlines: waves per frame (chains are independent)
constexpr double LN_FIT_ERR = 1.6;

__device__ __forceinline__ int refl101(int p, int len) {
  if (len == 1) return 0;
  while (p < 0 || p >= len) p = p < 0 ? -p : 2 * len - 2 - p;
  return p;
}

// ---------------------------------------------------------------- blur
// CN = 1: gray input. CN = 3 / 4: the colour frame BinaryDescriptor::detectImpl receives
// (rawImage, Frame.cc:324), converted with COLOR_BGR2GRAY (binary_descriptor.cpp:490-493;
// OpenCV 3.2 RGB2Gray<uchar> with the BGR coefficient order: (B*1868 + G*9617 + R*4899 +
// 2^13) >> 14) as the tile is staged -- no gray plane is written or read.
constexpr int LB_TW = 64, LB_TH = 16;
template <int CN>
__global__ __launch_bounds__(256) void k_line_blur(const uint8_t* __restrict__ img, int pitch, long long fstride,
                                                   int w, int h, int k0, int k1, int k2,
                                                   uint8_t* __restrict__ blur) {
  __shared__ uint8_t in[LB_TH + 4][LB_TW + 4];
  __shared__ int hs[LB_TH + 4][LB_TW];
  const int f = blockIdx.z, x0 = blockIdx.x * LB_TW, y0 = blockIdx.y * LB_TH, t = threadIdx.x;
  const uint8_t* G = img + f * fstride;
  for (int i = t; i < (LB_TH + 4) * (LB_TW + 4); i += 256) {
    const int r = i / (LB_TW + 4), c = i - r * (LB_TW + 4);
    const uint8_t* q = G + (long long)refl101(y0 - 2 + r, h) * pitch + (long long)refl101(x0 - 2 + c, w) * CN;
    if (CN == 1)
      in[r][c] = q[0];
    else
      in[r][c] = (uint8_t)((q[0] * 1868 + q[1] * 9617 + q[2] * 4899 + (1 << 13)) >> 14);
  }
  __syncthreads();
  for (int i = t; i < (LB_TH + 4) * LB_TW; i += 256) {
    const int r = i / LB_TW, c = i - r * LB_TW;
    hs[r][c] = k0 * ((int)in[r][c] + in[r][c + 4]) + k1 * ((int)in[r][c + 1] + in[r][c + 3]) + k2 * in[r][c + 2];
  }
  __syncthreads();
  for (int i = t; i < LB_TH * LB_TW; i += 256) {
    const int r = i / LB_TW, c = i - r * LB_TW;
    const int x = x0 + c, y = y0 + r;
    if (x >= w || y >= h) continue;
    const int s = k0 * (hs[r][c] + hs[r + 4][c]) + k1 * (hs[r + 1][c] + hs[r + 3][c]) + k2 * hs[r + 2][c];
    blur[(long long)f * w * h + (long long)y * w + x] = (uint8_t)min((s + (1 << 15)) >> 16, 255);
  }
}

// ---------------------------------------------------------------- gradient
__global__ __launch_bounds__(256) void k_line_grad(const uint8_t* __restrict__ blur, int w, int h,
                                                   int16_t* __restrict__ dxo, int16_t* __restrict__ dyo,
                                                   uint16_t* __restrict__ code) {
  const int f = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= w * h) return;
  const int y = i / w, x = i - y * w;
  const uint8_t* B = blur + (long long)f * w * h;
  const int xm = refl101(x - 1, w), xp = refl101(x + 1, w), ym = refl101(y - 1, h), yp = refl101(y + 1, h);
  const int a = B[ym * w + xm], b = B[ym * w + x], c = B[ym * w + xp];
  const int d = B[y * w + xm], e = B[y * w + xp];
  const int g = B[yp * w + xm], hh = B[yp * w + x], k = B[yp * w + xp];
  const int gx = (c - a) + 2 * (e - d) + (k - g);
  const int gy = (g - a) + 2 * (hh - b) + (k - c);
  const long long o = (long long)f * w * h + i;
  dxo[o] = (int16_t)gx;
  dyo[o] = (int16_t)gy;
  const int ax = abs(gx), ay = abs(gy), s = ax + ay;
  const int tz = s > LN_GRAD_TH + 1 ? s : 0;                // threshold(TOZERO, 81)
  const int q = __float2int_rn(fmul((float)tz, 0.25f));     // saturate_cast<short>(v * 0.25f)
  code[o] = (uint16_t)(q | (ax < ay ? LN_HORIZ : 0));
}

// ---------------------------------------------------------------- anchors
// anchor id k <-> (w = 1 + 2 * (k / nh), h = 1 + 2 * (k % nh)): the reference's scan order
__device__ __forceinline__ bool is_anchor(const uint16_t* C, int W, int x, int y) {
  const int i = y * W + x;
  const int c = C[i], g = c & 0x7fff;
  if (c & LN_HORIZ) return g >= (C[i - W] & 0x7fff) + LN_ANCHOR_TH && g >= (C[i + W] & 0x7fff) + LN_ANCHOR_TH;
  return g >= (C[i - 1] & 0x7fff) + LN_ANCHOR_TH && g >= (C[i + 1] & 0x7fff) + LN_ANCHOR_TH;
}
// A thread per candidate column (x = 1 + 2 t, up to blockDim.x columns per pass): the anchors
// of one column are consecutive in the reference's column-major order, so a block scan of
// the per-column counts in thread order places every column; the column's rows are walked in
// order, adjacent threads reading adjacent pixels (coalesced).
__global__ __launch_bounds__(512) void k_line_anchors(const uint16_t* __restrict__ code, int W, int H,
                                                      uint32_t* __restrict__ anchors, int acap,
                                                      int* __restrict__ nanchor) {
  __shared__ int wsum[8], base;
  const int f = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const uint16_t* C = code + (long long)f * W * H;
  uint32_t* A = anchors + (long long)f * acap;
  const int nw = (W - 2 + 1) / 2, nh = (H - 2 + 1) / 2;
  if (t == 0) base = 0;
  __syncthreads();
  for (int x0 = 0; x0 < nw; x0 += blockDim.x) {
    const int col = x0 + t, x = 1 + 2 * col;
    int c = 0;
    if (col < nw)
      for (int j = 0; j < nh; j++) c += is_anchor(C, W, x, 1 + 2 * j) ? 1 : 0;
    int v = c;  // inclusive scan over the block's columns
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(v, o, 64);
      if (lane >= o) v += u;
    }
    if (lane == 63) wsum[wave] = v;
    __syncthreads();
    int o = base + v - c;
    for (int w = 0; w < wave; w++) o += wsum[w];
    if (col < nw)
      for (int j = 0; j < nh; j++) {
        const int y = 1 + 2 * j;
        if (is_anchor(C, W, x, y)) {
          if (o < acap) A[o] = (uint32_t)x | ((uint32_t)y << 16);
          o++;
        }
      }
    __syncthreads();
    if (t == blockDim.x - 1) {
      int tot = 0;
      for (int w = 0; w < (int)(blockDim.x >> 6); w++) tot += wsum[w];
      base += tot;
    }
    __syncthreads();
  }
  if (t == 0) nanchor[f] = base;
}

// ---------------------------------------------------------------- edge drawing
// EdgeDrawing's anchor loop (:1695-2327): the whole wave executes the walk with uniform
// values (lane 0 writes), the edge map is a per-frame LDS bitmap
struct WalkState {
  uint32_t lastX, lastY;
};
// one walk from (x, y); appends packed (y << 16 | x) to P[off..]; false on overflow
// The walk reads the gradient code through a 64 x 64 tile of it cached in LDS, reloaded
// (centred on the step's pixel, rows clamped to the plane) when the pixel's 3 x 3
// neighbourhood leaves it: one round of coalesced loads per ~30 steps instead of one
// global round trip per step.
constexpr int LN_TS = 64;
struct CodeTile {
  uint16_t* t;  // LDS [LN_TS][LN_TS]
  int x0, y0;   // origin in the plane (x0 = -LN_TS: empty)
};
__device__ __forceinline__ void tile_cover(const uint16_t* __restrict__ C, int W, int H, CodeTile& T, int x, int y) {
  const int ax = max(x - 1, 0), bx = min(x + 1, W - 1), ay = max(y - 1, 0), by = min(y + 1, H - 1);
  if (ax >= T.x0 && bx < T.x0 + LN_TS && ay >= T.y0 && by < T.y0 + LN_TS) return;  // uniform
  T.x0 = min(max(x - LN_TS / 2, 0), max(W - LN_TS, 0));
  T.y0 = min(max(y - LN_TS / 2, 0), max(H - LN_TS, 0));
  const int lane = lane_id(), cx = min(T.x0 + lane, W - 1);
  for (int r0 = 0; r0 < LN_TS; r0 += 16) {  // 16 row loads in flight per lane
    uint16_t v[16];
#pragma unroll
    for (int r = 0; r < 16; r++) v[r] = C[min(T.y0 + r0 + r, H - 1) * W + cx];
#pragma unroll
    for (int r = 0; r < 16; r++) T.t[(r0 + r) * LN_TS + lane] = v[r];
  }
}
__device__ __forceinline__ int tile_at(const CodeTile& T, int x, int y) {  // inside the plane
  return T.t[(y - T.y0) * LN_TS + (x - T.x0)];
}
__device__ bool walk(const uint16_t* __restrict__ C, int W, int H, uint32_t* bits, uint32_t x, uint32_t y, int lastDir,
                     WalkState& st, uint32_t* __restrict__ P, uint32_t& off, uint32_t cap, CodeTile& T) {
  const int lane = threadIdx.x;
  int idx = (int)(y * W + x);
  // the pixel and its 8 neighbours from the tile (neighbour coordinates clamped to the plane:
  // at a border the walk stops before using a neighbour)
  int c;
  uint8_t nUL, nU, nUR, nL, nR, nDL, nD, nDR;
  auto load9 = [&](int, int xx, int yy) {
    tile_cover(C, W, H, T, xx, yy);
    const int xl = max(xx - 1, 0), xr = min(xx + 1, W - 1), yu = max(yy - 1, 0), yd = min(yy + 1, H - 1);
    c = tile_at(T, xx, yy);
    nUL = (uint8_t)tile_at(T, xl, yu);
    nU = (uint8_t)tile_at(T, xx, yu);
    nUR = (uint8_t)tile_at(T, xr, yu);
    nL = (uint8_t)tile_at(T, xl, yy);
    nR = (uint8_t)tile_at(T, xr, yy);
    nDL = (uint8_t)tile_at(T, xl, yd);
    nD = (uint8_t)tile_at(T, xx, yd);
    nDR = (uint8_t)tile_at(T, xr, yd);
  };
  load9(idx, (int)x, (int)y);
  while (true) {
    if ((c & 0x7fff) == 0 || ((bits[idx >> 5] >> (idx & 31)) & 1u)) break;
    if (off >= cap) return false;
    if (lane == 0) {
      atomicOr(&bits[idx >> 5], 1u << (idx & 31));
      P[off] = x | (y << 16);
    }
    off++;
    int should = 0;
    if (c & LN_HORIZ) {
      if (lastDir == LN_UP || lastDir == LN_DOWN) should = x > st.lastX ? LN_RIGHT : LN_LEFT;
      st.lastX = x;
      st.lastY = y;
      if (lastDir == LN_RIGHT || should == LN_RIGHT) {
        if (x == (uint32_t)W - 1 || y == 0 || y == (uint32_t)H - 1) break;
        const uint8_t g1 = nUR, g2 = nR, g3 = nDR;
        if (g1 >= g2 && g1 >= g3) {
          x++;
          y--;
        } else if (g3 >= g2 && g3 >= g1) {
          x++;
          y++;
        } else {
          x++;
        }
        lastDir = LN_RIGHT;
      } else if (lastDir == LN_LEFT || should == LN_LEFT) {
        if (x == 0 || y == 0 || y == (uint32_t)H - 1) break;
        const uint8_t g1 = nUL, g2 = nL, g3 = nDL;
        if (g1 >= g2 && g1 >= g3) {
          x--;
          y--;
        } else if (g3 >= g2 && g3 >= g1) {
          x--;
          y++;
        } else {
          x--;
        }
        lastDir = LN_LEFT;
      }
    } else {
      if (lastDir == LN_RIGHT || lastDir == LN_LEFT) should = y > st.lastY ? LN_DOWN : LN_UP;
      st.lastX = x;
      st.lastY = y;
      if (lastDir == LN_DOWN || should == LN_DOWN) {
        if (x == 0 || x == (uint32_t)W - 1 || y == (uint32_t)H - 1) break;
        const uint8_t g1 = nDR, g2 = nD, g3 = nDL;
        if (g1 >= g2 && g1 >= g3) {
          x++;
          y++;
        } else if (g3 >= g2 && g3 >= g1) {
          x--;
          y++;
        } else {
          y++;
        }
        lastDir = LN_DOWN;
      } else if (lastDir == LN_UP || should == LN_UP) {
        if (x == 0 || x == (uint32_t)W - 1 || y == 0) break;
        const uint8_t g1 = nUR, g2 = nU, g3 = nUL;
        if (g1 >= g2 && g1 >= g3) {
          x++;
          y--;
        } else if (g3 >= g2 && g3 >= g1) {
          x--;
          y--;
        } else {
          y--;
        }
        lastDir = LN_UP;
      }
    }
    idx = (int)(y * W + x);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    load9(idx, (int)x, (int)y);
  }
  return true;
}

// per frame: anchors A[nanchor], parts scratch P1 / P2 [pcap], chains out Q[2 pcap] with
// sid S[ecap + 1]; nedge[f] = kept chains, or -1 on overflow (the reference's -1 paths)
__global__ __launch_bounds__(64) void k_edge_draw(const uint16_t* __restrict__ code, int W, int H,
                                                  const uint32_t* __restrict__ anchors, const int* __restrict__ nanchor,
                                                  int acap, uint32_t* __restrict__ p1, uint32_t* __restrict__ p2,
                                                  int pcap, uint32_t* __restrict__ chains, uint32_t* __restrict__ sid,
                                                  int ecap, int* __restrict__ nedge) {
  extern __shared__ uint32_t bits[];
  const int f = blockIdx.x, lane = threadIdx.x;
  const uint16_t* C = code + (long long)f * W * H;
  const int nb = (W * H + 31) / 32;
  CodeTile T{(uint16_t*)(bits + ((nb + 3) & ~3)), -LN_TS, -LN_TS};
  for (int i = lane; i < nb; i += 64) bits[i] = 0;
  __syncthreads();
  const uint32_t* A = anchors + (long long)f * acap;
  uint32_t* P1 = p1 + (long long)f * pcap;
  uint32_t* P2 = p2 + (long long)f * pcap;
  uint32_t* Q = chains + (long long)f * 2 * pcap;
  uint32_t* S = sid + (long long)f * (ecap + 1);
  const int na = nanchor[f];
  WalkState st{0u, 0u};
  uint32_t nq = 0;
  int ne = 0;
  bool fail = na > acap || na > pcap;  // anchorsSize > edgePixelArraySize
  for (int a = 0; a < na && !fail; a++) {
    const uint32_t ap = A[a], x = ap & 0xffffu, y = ap >> 16;
    const int idx = (int)(y * W + x);
    if ((bits[idx >> 5] >> (idx & 31)) & 1u) continue;
    if (ne > ecap) {
      fail = true;
      break;
    }
    const bool horiz = (C[idx] & LN_HORIZ) != 0;
    uint32_t o1 = 0, o2 = 0;
    if (!walk(C, W, H, bits, x, y, horiz ? LN_RIGHT : LN_DOWN, st, P1, o1, (uint32_t)pcap, T)) {
      fail = true;
      break;
    }
    if (lane == 0) atomicAnd(&bits[idx >> 5], ~(1u << (idx & 31)));  // the second part walks the anchor again
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (!walk(C, W, H, bits, x, y, horiz ? LN_LEFT : LN_UP, st, P2, o2, (uint32_t)pcap, T)) {
      fail = true;
      break;
    }
    if ((int)(o1 + o2) < LN_MIN_LEN + 1) continue;  // short edge: dropped, its pixels stay marked
    // chain: the first part reversed, then the second part without its copy of the anchor
    __syncthreads();
    if (nq + o1 + o2 > 2u * (uint32_t)pcap) {
      fail = true;
      break;
    }
    if (lane == 0) S[ne] = nq;
    for (uint32_t i = lane; i < o1; i += 64) Q[nq + i] = P1[o1 - 1 - i];
    for (uint32_t i = 1 + lane; i < o2; i += 64) Q[nq + o1 + i - 1] = P2[i];
    nq += o1 + (o2 > 0 ? o2 - 1 : 0);
    ne++;
    __syncthreads();
  }
  if (lane == 0) {
    if (!fail) S[ne] = nq;
    nedge[f] = fail ? -1 : ne;
  }
}

// ---------------------------------------------------------------- EDline
__device__ double ln_log_gamma(double x) {  // descriptor.hpp:694-727
  if (x > 15.0)
    return 0.918938533204673 + (x - 0.5) * log(x) - x + 0.5 * x * log(x * sinh(1 / x) + 1 / (810.0 * pow(x, 6.0)));
  const double q[7] = {75122.6331530, 80916.6278952, 36308.2951477, 8687.24529705,
                       1168.92649479, 83.8676043424, 2.50662827511};
  double a = (x + 0.5) * log(x + 5.5) - (x + 5.5);
  double b = 0.0;
  for (int n = 0; n < 7; n++) {
    a -= log(x + (double)n);
    b += q[n] * pow(x, (double)n);
  }
  return a + log(b);
}
__device__ double ln_nfa(int n, int k, double p, double logNT) {  // descriptor.hpp:763-844
  const double tolerance = 0.1;
  if (n == 0 || k == 0) return -logNT;
  if (n == k) return -logNT - (double)n * log10(p);
  const double p_term = p / (1.0 - p);
  const double log1term = ln_log_gamma((double)n + 1.0) - ln_log_gamma((double)k + 1.0) -
                          ln_log_gamma((double)(n - k) + 1.0) + (double)k * log(p) + (double)(n - k) * log(1.0 - p);
  double term = exp(log1term);
  {
    const double aa = fabs(term);
    double abs_max = aa > 0.0 ? aa : 0.0;
    if (abs_max < DBL_MIN) abs_max = DBL_MIN;
    if (term == 0.0 || aa / abs_max <= 100.0 * DBL_EPSILON) {  // double_equal(term, 0)
      if ((double)k > (double)n * p) return -log1term / 2.30258509299404568402 - logNT;
      return -logNT;
    }
  }
  double bin_tail = term;
  for (int i = k + 1; i <= n; i++) {
    const double bin_term = (double)(n - i + 1) / (double)i;
    const double mult_term = bin_term * p_term;
    term *= mult_term;
    bin_tail += term;
    if (bin_term < 1.0) {
      const double err = term * ((1.0 - pow(mult_term, (double)(n - i + 1))) / (1.0 - mult_term) - 1.0);
      if (err < tolerance * fabs(-log10(bin_tail) - logNT) * bin_tail) break;
    }
  }
  return -log10(bin_tail) - logNT;
}

__device__ __forceinline__ uint32_t px_x(uint32_t p) { return p & 0xffffu; }
__device__ __forceinline__ uint32_t px_y(uint32_t p) { return p >> 16; }

// sums over pixels [s, e) of u = x (horiz) or y, v = the other: sum u^2, sum u, count,
// sum u v, sum v -- integers, exact in double whatever the order; rounded to float once
// (cv::gemm's double accumulation), as LeastSquaresLineFit_'s ATA / ATV
__device__ void fit_block(const uint32_t* P, uint32_t s, uint32_t e, bool horiz, float* ata, float* atv) {
  double s00 = 0, s01 = 0, t0 = 0, t1 = 0;
  for (uint32_t i = s + lane_id(); i < e; i += 64) {
    const uint32_t p = P[i];
    const double u = (double)(horiz ? px_x(p) : px_y(p)), v = (double)(horiz ? px_y(p) : px_x(p));
    s00 += u * u;
    s01 += u;
    t0 += u * v;
    t1 += v;
  }
  s00 = wave_sum(s00);
  s01 = wave_sum(s01);
  t0 = wave_sum(t0);
  t1 = wave_sum(t1);
  ata[0] = (float)s00;
  ata[1] = ata[2] = (float)s01;
  ata[3] = (float)(double)(e - s);
  atv[0] = (float)t0;
  atv[1] = (float)t1;
}
__device__ __forceinline__ void solve2(const float* ata, const float* atv, double* le) {
  const double coef = 1.0 / __dsub_rn(__dmul_rn((double)ata[0], (double)ata[3]), __dmul_rn((double)ata[1], (double)ata[2]));
  le[0] = __dmul_rn(coef, __dsub_rn(__dmul_rn((double)ata[3], (double)atv[0]), __dmul_rn((double)ata[1], (double)atv[1])));
  le[1] = __dmul_rn(coef, __dsub_rn(__dmul_rn((double)ata[0], (double)atv[1]), __dmul_rn((double)ata[2], (double)atv[0])));
}

// one wave per frame: chains Q / S -> lines out [cap][6] (sx, sy, ex, ey, angle, length)
__global__ __launch_bounds__(64 * LN_WAVES) void k_edlines(const uint16_t* __restrict__ code,
                                                          const int16_t* __restrict__ dxi,
                                                          const int16_t* __restrict__ dyi, int W, int H,
                                                          const uint32_t* __restrict__ chains,
                                                          const uint32_t* __restrict__ sid,
                                                          const int* __restrict__ nedge, int pcap, int ecap,
                                                          uint32_t* __restrict__ lscratch,
                                                          uint32_t* __restrict__ ccount, float min_length,
                                                          float* __restrict__ out, int* __restrict__ nout, int cap) {
  const int f = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint16_t* C = code + (long long)f * W * H;
  const int16_t* DX = dxi + (long long)f * W * H;
  const int16_t* DY = dyi + (long long)f * W * H;
  const uint32_t* Q = chains + (long long)f * 2 * pcap;
  const uint32_t* S = sid + (long long)f * (ecap + 1);
  uint32_t* L = lscratch + (long long)f * 2 * pcap;
  float* O = out + (long long)f * cap * 6;
  int* CNT = (int*)(ccount + (long long)f * pcap);  // lines kept per chain
  const int ne = nedge[f];
  if (ne < 0) {  // the whole workgroup
    if (threadIdx.x == 0) nout[f] = -1;
    return;
  }
  const double logNT = 2.0 * (log10((double)W) + log10((double)H));
  auto horiz_at = [&](uint32_t p) { return (C[px_y(p) * W + px_x(p)] & LN_HORIZ) != 0; };
  // chains are independent: wave w takes chains w, w + nw, ...; a chain's line pixels use its
  // own stretch of the scratch [S[e], S[e + 1]), and its kept lines are parked at the start
  // of that stretch (record k at 6 k: below the next line's pixels, see the store) until the
  // block places every chain's lines in chain order
  for (int e = wave; e < ne; e += nw) {
    uint32_t s = S[e];
    const uint32_t end = S[e + 1];
    uint32_t offL = s;
    int nl = 0;
    double le2[2] = {0, 0};
    float ata[4], atv[2];
    while (end > s + LN_MIN_LEN) {
      double fitErr = 0;
      while (end > s + LN_MIN_LEN) {
        const bool h0 = horiz_at(Q[s]);
        fit_block(Q, s, s + LN_MIN_LEN, h0, ata, atv);
        solve2(ata, atv, le2);
        double c2 = 0;  // fit error in the reference's order: one lane, sequential
        for (uint32_t i = s; i < s + LN_MIN_LEN; i++) {
          const uint32_t p = Q[i];
          const double u = (double)(h0 ? px_x(p) : px_y(p)), v = (double)(h0 ? px_y(p) : px_x(p));
          const double c = __dsub_rn(__dsub_rn(v, __dmul_rn(u, le2[0])), le2[1]);
          c2 = __dadd_rn(c2, __dmul_rn(c, c));
        }
        fitErr = sqrt(c2);
        if (fitErr <= LN_FIT_ERR) break;
        s += LN_SKIP;
      }
      if (fitErr > LN_FIT_ERR) break;
      const uint32_t lineStart = offL;
      const bool horiz = horiz_at(Q[s]);
      double coef1 = 0;
      bool extended = true, first = true;
      int tryTimes = 0, outliers = 0;
      uint32_t newOffS = 0;
      while (extended) {
        tryTimes++;
        if (first) {
          first = false;
          for (int i = lane; i < LN_MIN_LEN; i += 64) L[offL + i] = Q[s + i];
          offL += LN_MIN_LEN;
          s += LN_MIN_LEN;
        } else {
          float ta[4], tv[2];
          fit_block(L, newOffS, offL, horiz, ta, tv);
          for (int q = 0; q < 4; q++) ata[q] = fadd(ata[q], ta[q]);
          for (int q = 0; q < 2; q++) atv[q] = fadd(atv[q], tv[q]);
          solve2(ata, atv, le2);
        }
        coef1 = 1 / sqrt(__dadd_rn(__dmul_rn(le2[0], le2[0]), 1.0));
        outliers = 0;
        newOffS = offL;
        // the extension walk: sequential in the reference (it stops after four outliers
        // in a row); evaluated 64 pixels at a time, the stop found by ballot
        while (end > s) {
          const uint32_t i = s + lane;
          bool out_ = false;
          if (i < end) {
            const uint32_t p = Q[i];
            const double xx = (double)px_x(p), yy = (double)px_y(p);
            const double d = horiz ? fabs(__dadd_rn(__dsub_rn(__dmul_rn(le2[0], xx), yy), le2[1]))
                                   : fabs(__dsub_rn(__dsub_rn(xx, __dmul_rn(le2[0], yy)), le2[1]));
            out_ = __dmul_rn(d, coef1) > LN_FIT_ERR;
            L[offL + lane] = p;
          }
          const uint64_t om = ballot(i < end && out_);
          const int nvalid = (int)min<uint32_t>(64u, end - s);
          // replay the sequential outlier counter over this block
          int stop = -1, run = outliers;
          for (int j = 0; j < nvalid; j++) {
            if ((om >> j) & 1ull) {
              if (++run > 3) {
                stop = j;
                break;
              }
            } else {
              run = 0;
            }
          }
          outliers = run;
          if (stop >= 0) {
            offL += (uint32_t)stop + 1;
            s += (uint32_t)stop + 1;
            break;
          }
          offL += (uint32_t)nvalid;
          s += (uint32_t)nvalid;
        }
        offL -= (uint32_t)outliers;
        s -= (uint32_t)outliers;
        extended = offL - newOffS > 0 && tryTimes < LN_TRY;
      }
      double le[3];
      if (horiz) {
        le[0] = __dmul_rn(le2[0], coef1);
        le[1] = -1 * coef1;
        le[2] = __dmul_rn(le2[1], coef1);
      } else {
        le[0] = 1 * coef1;
        le[1] = __dmul_rn(-le2[0], coef1);
        le[2] = __dmul_rn(-le2[1], coef1);
      }
      // LineValidation_ (:2793-2874)
      const int n = (int)(offL - lineStart);
      int mgx = 0, mgy = 0;
      for (int i = lane; i < n; i += 64) {
        const uint32_t p = L[lineStart + i];
        const int idx = px_y(p) * W + px_x(p);
        mgx += DX[idx];
        mgy += DY[idx];
      }
      mgx = wave_sum(mgx);
      mgy = wave_sum(mgy);
      const double dxl = fabs(le[1]), dyl = fabs(le[0]);
      bool ok = !(mgx == 0 && mgy == 0);
      float direction = 0.f;
      if (ok) {
        if (mgx > 0 && mgy >= 0) direction = (float)atan2(-dyl, dxl);
        if (mgx <= 0 && mgy > 0) direction = (float)atan2(dyl, dxl);
        if (mgx < 0 && mgy <= 0) direction = (float)atan2(dyl, -dxl);
        if (mgx >= 0 && mgy < 0) direction = (float)atan2(-dyl, -dxl);
        const double fd = (double)fabsf(direction);
        if (fd < 0.15 || M_PI - fd < 0.15)
          if (fabs(le[2]) < 10 || fabs(H - fabs(le[2])) < 10) ok = false;
        if (fabs(fd - M_PI * 0.5) < 0.15)
          if (fabs(le[2]) < 10 || fabs(W - fabs(le[2])) < 10) ok = false;
      }
      if (ok) {
        int k = 0;
        for (int i = lane; i < n; i += 64) {
          const uint32_t p = L[lineStart + i];
          const int idx = px_y(p) * W + px_x(p);
          const double pd = atan2(-(double)DX[idx], (double)DY[idx]);
          const double dd = fabs((double)direction - pd);
          if (fabs(2 * M_PI - dd) < 0.392699 || dd < 0.392699) k++;
        }
        k = wave_sum(k);
        ok = ln_nfa(n, k, 0.125, logNT) > 0;
      }
      if (ok) {
        const double a1 = __dmul_rn(le[1], le[1]), a2 = __dmul_rn(le[0], le[0]), a3 = __dmul_rn(le[0], le[1]),
                     a4 = __dmul_rn(le[2], le[0]), a5 = __dmul_rn(le[2], le[1]);
        const uint32_t p0 = L[lineStart], p1 = L[offL - 1];
        float ep[4];
        ep[0] = (float)__dsub_rn(__dsub_rn(__dmul_rn(a1, (double)px_x(p0)), __dmul_rn(a3, (double)px_y(p0))), a4);
        ep[1] = (float)__dsub_rn(__dsub_rn(__dmul_rn(a2, (double)px_y(p0)), __dmul_rn(a3, (double)px_x(p0))), a5);
        ep[2] = (float)__dsub_rn(__dsub_rn(__dmul_rn(a1, (double)px_x(p1)), __dmul_rn(a3, (double)px_y(p1))), a4);
        ep[3] = (float)__dsub_rn(__dsub_rn(__dmul_rn(a2, (double)px_y(p1)), __dmul_rn(a3, (double)px_x(p1))), a5);
        // OctaveKeyLines: length from the fitted endpoints, start / end by direction
        const float dxa = fabsf(fsub(ep[0], ep[2])), dya = fabsf(fsub(ep[1], ep[3]));
        // sqrt of the float sum, correctly rounded (through double: innocuous double rounding)
        const float length = (float)sqrt((double)fadd(fmul(dxa, dxa), fmul(dya, dya)));
        const float ddx = fsub(ep[2], ep[0]), ddy = fsub(ep[3], ep[1]);
        const double d = (double)direction;
        bool change = false;
        if (d >= -0.75 * M_PI && d < -0.25 * M_PI && ddy > 0) change = true;
        if (d >= -0.25 * M_PI && d < 0.25 * M_PI && ddx < 0) change = true;
        if (d >= 0.25 * M_PI && d < 0.75 * M_PI && ddy < 0) change = true;
        if (((d >= 0.75 * M_PI && d < M_PI) || (d >= -M_PI && d < -0.75 * M_PI)) && ddx > 0) change = true;
        if (length > min_length) {
          // record nl of this chain at L[S[e] + 6 nl]: every earlier kept line of the chain
          // spans >= LN_MIN_LEN - 3 > 6 pixels, so the record lies below this line's start
          // (or, for nl = 0, over this line's own pixels, read above)
          if (lane < 6) {
            const float v = lane == 0 ? (change ? ep[2] : ep[0])
                          : lane == 1 ? (change ? ep[3] : ep[1])
                          : lane == 2 ? (change ? ep[0] : ep[2])
                          : lane == 3 ? (change ? ep[1] : ep[3])
                          : lane == 4 ? direction : length;
            L[S[e] + 6 * nl + lane] = __float_as_uint(v);
          }
          nl++;
        }
      } else {
        offL = lineStart;
      }
    }
    if (lane == 0) CNT[e] = nl;
  }
  __syncthreads();
  // the chains' lines in chain order: a block scan of the per-chain counts; a chain's thread
  // copies its records (lines past cap are counted, not stored, as the reference's nl)
  __shared__ int wsum[16], carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int c0 = 0; c0 < ne; c0 += blockDim.x) {
    const int i = c0 + threadIdx.x;
    const int v = i < ne ? CNT[i] : 0;
    int x = v;
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(x, o, 64);
      if (lane >= o) x += u;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    int before = carry;
    for (int w = 0; w < wave; w++) before += wsum[w];
    const int base = before + x - v;
    if (i < ne) {
      const uint32_t* R = L + S[i];
      for (int j = 0; j < v; j++)
        if (base + j < cap)
          for (int q = 0; q < 6; q++) O[6 * (long long)(base + j) + q] = __uint_as_float(R[6 * j + q]);
    }
    __syncthreads();
    if (threadIdx.x == blockDim.x - 1) carry = base + v;
    __syncthreads();
  }
  if (threadIdx.x == 0) nout[f] = carry;
}

// ================================================================ host
struct LineEngine {
  int dev = 0, W = 0, H = 0, B = 0;
  int acap = 0, pcap = 0, ecap = 0;
  int k[3] = {0, 0, 0};
  hipStream_t stream = nullptr;
  uint8_t* d_blur = nullptr;
  int16_t *d_dx = nullptr, *d_dy = nullptr;
  uint16_t* d_code = nullptr;
  uint32_t *d_anch = nullptr, *d_p1 = nullptr, *d_p2 = nullptr, *d_chain = nullptr, *d_sid = nullptr,
           *d_lscr = nullptr;
  int *d_nanch = nullptr, *d_nedge = nullptr;
  uint8_t* d_img = nullptr;  // [H][W * 4]: one host frame of up to 4 channels
  float* d_lines = nullptr;
  int* d_nlines = nullptr;
  int* h_n = nullptr;  // pinned: the single-frame line count
  ~LineEngine() {
    void* p[] = {d_blur, d_dx, d_dy, d_code, d_anch, d_p1, d_p2, d_chain, d_sid, d_lscr, d_nanch, d_nedge, d_img,
                 d_lines, d_nlines};
    for (void* q : p)
      if (q) (void)hipFree(q);
    if (h_n) (void)hipHostFree(h_n);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

// getGaussianKernel(5, 1, CV_32F) -> the 8U fixed-point taps (cvRound(k * 256))
static void gauss5(int* k) {
  float cf[5];
  double sum = 0;
  for (int i = 0; i < 5; i++) {
    const double x = i - 2.0;
    cf[i] = (float)std::exp(-0.5 * x * x);
    sum += cf[i];
  }
  sum = 1. / sum;
  for (int i = 0; i < 5; i++) {
    cf[i] = (float)(cf[i] * sum);
    k[i] = (int)std::nearbyint((double)cf[i] * 256.0);
  }
}

}  // namespace eao

using namespace eao;
struct eao_lines {
  LineEngine e;
};

extern "C" {

int eao_lines_create(int device, int width, int height, int max_batch, eao_lines** out) {
  if (!out) return EAO_E_ARG;
  *out = nullptr;
  if (width < 8 || height < 8 || width > 8192 || height > 8192 || max_batch < 1) return EAO_E_ARG;
  if (!eao_device_ok(device)) {
    set_error("no usable gfx950 device (the engine has no CPU fallback)");
    return EAO_E_NODEVICE;
  }
  // the same dynamic LDS k_edge_draw is launched with: the edge bitmap (16-byte padded) +
  // the gradient-code tile
  if ((size_t)(((width * height + 31) / 32 + 3) & ~3) * 4 + sizeof(uint16_t) * LN_TS * LN_TS > 160 * 1024) {
    set_error("eao_lines_create: the per-frame edge bitmap and code tile exceed the LDS");
    return EAO_E_CAPACITY;
  }
  eao_lines* L = new eao_lines();
  LineEngine& e = L->e;
  e.dev = device;
  e.W = width;
  e.H = height;
  e.B = max_batch;
  // EdgeDrawing's arrays: edgePixelArraySize = pixels / 5, maxNumOfEdge = that / 20
  e.pcap = width * height / 5;
  e.acap = e.pcap;
  e.ecap = e.pcap / 20;
  int k5[5];
  gauss5(k5);
  e.k[0] = k5[0];
  e.k[1] = k5[1];
  e.k[2] = k5[2];
  const size_t px = (size_t)width * height * max_batch;
  auto fail = [&](int rc) {
    delete L;
    return rc;
  };
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&e.stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&e.d_blur, px) != hipSuccess || hipMalloc(&e.d_dx, px * 2) != hipSuccess ||
      hipMalloc(&e.d_dy, px * 2) != hipSuccess || hipMalloc(&e.d_code, px * 2) != hipSuccess ||
      hipMalloc(&e.d_anch, (size_t)e.acap * 4 * max_batch) != hipSuccess ||
      hipMalloc(&e.d_p1, (size_t)e.pcap * 4 * max_batch) != hipSuccess ||
      hipMalloc(&e.d_p2, (size_t)e.pcap * 4 * max_batch) != hipSuccess ||
      hipMalloc(&e.d_chain, (size_t)e.pcap * 8 * max_batch) != hipSuccess ||
      hipMalloc(&e.d_lscr, (size_t)e.pcap * 8 * max_batch) != hipSuccess ||
      hipMalloc(&e.d_sid, (size_t)(e.ecap + 1) * 4 * max_batch) != hipSuccess ||
      hipMalloc(&e.d_nanch, 4 * (size_t)max_batch) != hipSuccess ||
      hipMalloc(&e.d_nedge, 4 * (size_t)max_batch) != hipSuccess ||
      hipMalloc(&e.d_img, (size_t)width * height * 4) != hipSuccess ||
      hipMalloc(&e.d_lines, sizeof(float) * 6 * 4096) != hipSuccess || hipMalloc(&e.d_nlines, 4) != hipSuccess ||
      hipHostMalloc((void**)&e.h_n, sizeof(int), 0) != hipSuccess) {
    set_error("eao_lines_create: device allocation failed");
    return fail(EAO_E_HIP);
  }
  *out = L;
  return EAO_OK;
}

int eao_lines_destroy(eao_lines* L) {
  delete L;
  return EAO_OK;
}

int eao_lines_detect_color_batch_device(eao_lines* L, const uint8_t* d_img, int nframes, int pitch, int channels,
                                        float min_length, float* d_lines, int32_t* d_counts, int cap, void* stream) {
  if (!L || !d_img || !d_lines || !d_counts || nframes < 1 || cap < 1) return EAO_E_ARG;
  LineEngine& e = L->e;
  if (channels != 1 && channels != 3 && channels != 4) {
    set_error("eao_lines_detect: channels must be 1, 3 or 4");
    return EAO_E_ARG;
  }
  if (nframes > e.B || pitch < e.W * channels) {
    set_error("eao_lines_detect_batch_device: more frames than max_batch or pitch < width * channels");
    return EAO_E_ARG;
  }
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  hipStream_t s = stream ? (hipStream_t)stream : e.stream;
  const int W = e.W, H = e.H;
  const dim3 bg((W + LB_TW - 1) / LB_TW, (H + LB_TH - 1) / LB_TH, nframes);
  const long long fs = (long long)pitch * H;
  if (channels == 1)
    hipLaunchKernelGGL(k_line_blur<1>, bg, dim3(256), 0, s, d_img, pitch, fs, W, H, e.k[0], e.k[1], e.k[2], e.d_blur);
  else if (channels == 3)
    hipLaunchKernelGGL(k_line_blur<3>, bg, dim3(256), 0, s, d_img, pitch, fs, W, H, e.k[0], e.k[1], e.k[2], e.d_blur);
  else
    hipLaunchKernelGGL(k_line_blur<4>, bg, dim3(256), 0, s, d_img, pitch, fs, W, H, e.k[0], e.k[1], e.k[2], e.d_blur);
  hipLaunchKernelGGL(k_line_grad, dim3((W * H + 255) / 256, nframes), dim3(256), 0, s, e.d_blur, W, H, e.d_dx,
                     e.d_dy, e.d_code);
  hipLaunchKernelGGL(k_line_anchors, dim3(nframes), dim3(512), 0, s, e.d_code, W, H, e.d_anch, e.acap, e.d_nanch);
  const size_t lds = (size_t)(((W * H + 31) / 32 + 3) & ~3) * 4 + sizeof(uint16_t) * LN_TS * LN_TS;
  hipLaunchKernelGGL(k_edge_draw, dim3(nframes), dim3(64), lds, s, e.d_code, W, H, e.d_anch, e.d_nanch, e.acap,
                     e.d_p1, e.d_p2, e.pcap, e.d_chain, e.d_sid, e.ecap, e.d_nedge);
  // (the parts scratch P1 is dead after k_edge_draw: it holds the per-chain line counts)
  hipLaunchKernelGGL(k_edlines, dim3(nframes), dim3(64 * LN_WAVES), 0, s, e.d_code, e.d_dx, e.d_dy, W, H,
                     e.d_chain, e.d_sid, e.d_nedge, e.pcap, e.ecap, e.d_lscr, e.d_p1, min_length, d_lines, d_counts,
                     cap);
  EAO_HIP_CHECK(hipGetLastError());
  return EAO_OK;
}

int eao_lines_detect_batch_device(eao_lines* L, const uint8_t* d_gray, int nframes, int pitch, float min_length,
                                  float* d_lines, int32_t* d_counts, int cap, void* stream) {
  return eao_lines_detect_color_batch_device(L, d_gray, nframes, pitch, 1, min_length, d_lines, d_counts, cap, stream);
}

int eao_lines_detect_color(eao_lines* L, const uint8_t* img, int pitch, int channels, float min_length, float* lines,
                           int cap, int* n_out) {
  if (!L || !img || !n_out || cap < 0 || (cap && !lines)) return EAO_E_ARG;
  LineEngine& e = L->e;
  if ((channels != 1 && channels != 3 && channels != 4) || pitch < e.W * channels) return EAO_E_ARG;
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  hipStream_t s = e.stream;
  const int row = e.W * channels;
  EAO_HIP_CHECK(hipMemcpy2DAsync(e.d_img, row, img, pitch, row, e.H, hipMemcpyHostToDevice, s));
  int rc = eao_lines_detect_color_batch_device(L, e.d_img, 1, row, channels, min_length, e.d_lines, e.d_nlines, 4096, s);
  if (rc) return rc;
  EAO_HIP_CHECK(hipMemcpyAsync(e.h_n, e.d_nlines, 4, hipMemcpyDeviceToHost, s));
  EAO_HIP_CHECK(hipStreamSynchronize(s));
  const int n = *e.h_n;
  if (n < 0) {
    set_error("eao_lines_detect: edge arrays overflowed (the reference's EdgeDrawing -1)");
    return EAO_E_CAPACITY;
  }
  *n_out = n;
  const int k = n < cap ? n : cap;
  if (k > 0) EAO_HIP_CHECK(hipMemcpy(lines, e.d_lines, sizeof(float) * 6 * k, hipMemcpyDeviceToHost));
  return n > cap ? EAO_E_CAPACITY : EAO_OK;
}

int eao_lines_detect(eao_lines* L, const uint8_t* gray, int pitch, float min_length, float* lines, int cap,
                     int* n_out) {
  return eao_lines_detect_color(L, gray, pitch, 1, min_length, lines, cap, n_out);
}

// the intermediate maps of the last eao_lines_detect (frame slot 0): blur [h][w] u8,
// dx / dy [h][w] i16, code [h][w] u16 (thresholded |dx| + |dy| over 4 | 0x8000 if
// Horizontal), for parity tests
int eao_lines_debug_maps(eao_lines* L, uint8_t* blur, int16_t* dx, int16_t* dy, uint16_t* code) {
  if (!L) return EAO_E_ARG;
  LineEngine& e = L->e;
  const size_t n = (size_t)e.W * e.H;
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  EAO_HIP_CHECK(hipStreamSynchronize(e.stream));
  if (blur) EAO_HIP_CHECK(hipMemcpy(blur, e.d_blur, n, hipMemcpyDeviceToHost));
  if (dx) EAO_HIP_CHECK(hipMemcpy(dx, e.d_dx, n * 2, hipMemcpyDeviceToHost));
  if (dy) EAO_HIP_CHECK(hipMemcpy(dy, e.d_dy, n * 2, hipMemcpyDeviceToHost));
  if (code) EAO_HIP_CHECK(hipMemcpy(code, e.d_code, n * 2, hipMemcpyDeviceToHost));
  return EAO_OK;
}

}  // extern "C"
