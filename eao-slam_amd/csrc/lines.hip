// lines.hip -- per-frame line detection of the EAO Frame on gfx950: the MI355X replacement
// of line_lbd_detect::detect_raw_lines + filter_lines (reference src/Frame.cc:324-328,
// src/line_detect/line_lbd_allclass.cpp:137-214) with the tracker's single octave
// (Tracking.cc:161-163): GaussianBlur(5x5, sigma 1), then EDLineDetector::EDline
// (src/line_detect/libs/binary_descriptor.cpp:1583-2906) and OctaveKeyLines' endpoint
// ordering (:866-887, 1073-1141); lines longer than min_length are kept.
//
// Pipeline per batch of HBM-resident gray frames:
//   k_line_maps     64x32 output tiles through LDS: (COLOR_BGR2GRAY,) the 8U fixed-point
//                   separable 5-tap Gaussian, Sobel 3x3 dx, dy, code = thresholded |dx| + |dy|
//                   over 4 (cvRound) | Horizontal bit, and the walk's 16-bit move words
//   k_line_anchors  one workgroup per frame, a thread per candidate column (the candidates tested
//                   in k_line_maps, one row mask per column and band): the anchors in the
//                   reference's column-major scan order (w outer, h inner, step 2) from a
//                   block scan of the per-column counts
//   k_edge_draw     one wave per frame: the anchor walks over the move words (edge map as an
//                   LDS bitmap), the kept chains assembled by the whole wave
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
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/eao_accel.h"
#include "common.h"

namespace eao {

constexpr int LN_HORIZ = 0x8000;  // code bit: dirImg_ == Horizontal (|dx| < |dy|)
constexpr int LN_UP = 1, LN_RIGHT = 2, LN_DOWN = 3, LN_LEFT = 4;
constexpr int LN_GRAD_TH = 80, LN_ANCHOR_TH = 8, LN_MIN_LEN = 15, LN_TRY = 6, LN_SKIP = 2;
constexpr int LN_WAVES = 8;  // k_edlines: waves per frame (chains are independent)
constexpr double LN_FIT_ERR = 1.6;

// ---------------------------------------------------------------- move words
// A walk step (:1746-2000) depends on the pixel only: whether it is an edge pixel (gImg_ > 0),
// its direction (dirImg_), and, for each of the two directions a walk can take through it, which
// of the three forward neighbours has the largest gImg_ byte (the reference's if-chain, ties
// included) or that the image border ends the walk there. k_line_maps evaluates this once per
// pixel into a 16-bit move word, so a step of the sequential walk is two LDS reads (the
// word through a tile cache, the edge-map bit) and a few scalar operations. The walk's state is
// two bits st = (the last step increased x) << 1 | (it increased y) (ed_walk); nibble st of the
// word is the step the walk takes from the pixel in state st, as (dx + 1) | (dy + 1) << 2:
// a Horizontal pixel is left RIGHT when st's x bit is set, else LEFT; a Vertical one DOWN when
// st's y bit is set, else UP; of the three forward neighbours the one with the largest gImg_
// byte (the reference's if-chain, ties included). At the image border, and where the step would
// land on a non-edge pixel (gImg_ == 0, where the reference's walk ends without taking it), the
// step is (0, 0): stop after the pixel (the walk finds its own pixel marked next). So a walk,
// which starts at an anchor (an edge pixel), only ever reads edge pixels' words; a non-edge
// pixel's word is 0. Rows have the pitch MP (a multiple of 16) so the tile loads are aligned
// 16-byte loads.
constexpr int LM_STOP = 5;  // (0, 0)
// the nibble of a step: forward (fwd: RIGHT / DOWN) or back, ch the reference's choice
// (0 straight, 1 the g1 diagonal, 2 the g3 diagonal, 3 the border)
__device__ __forceinline__ int lm_nibble(bool hz, int fwd, int ch) {
  if (ch == 3) return LM_STOP;
  const int along = 2 * fwd - 1, side = (ch >> 1) - (ch & 1);  // ch 1: the g1 side (-1), 2: g3 (+1)
  const int dx = hz ? along : -side, dy = hz ? side : along;  // DOWN / UP: g1 is the x + 1 neighbour
  return (dx + 1) | (dy + 1) << 2;
}
__device__ __forceinline__ int ln_pick(int g1, int g2, int g3) {
  return (g1 >= g2 && g1 >= g3) ? 1 : ((g3 >= g2 && g3 >= g1) ? 2 : 0);
}

// ---------------------------------------------------------------- maps
// One kernel per 64x32 output tile: gray (CN = 3 / 4: the colour frame BinaryDescriptor::
// detectImpl receives, rawImage of Frame.cc:324, converted with COLOR_BGR2GRAY,
// binary_descriptor.cpp:490-493: OpenCV 3.2 RGB2Gray<uchar> with the BGR coefficient order
// (B*1868 + G*9617 + R*4899 + 2^13) >> 14), the 8U fixed-point separable 5-tap Gaussian (taps
// cvRound(k * 256), REFLECT_101, columns (s + 2^15) >> 16), Sobel 3x3 dx / dy (REFLECT_101), the
// gradient code (thresholded |dx| + |dy| over 4, cvRound | Horizontal bit) and the walk's move
// bytes (above), all staged in LDS with halos 4 / 2 / 1: the frame is read once and each map
// written once. The gray halo is read at reflected coordinates; because the Gaussian is
// symmetric, the blur evaluated 1-2 pixels outside the plane then equals the blur at the
// reflected pixel, which is what the Sobel's own REFLECT_101 reads.
constexpr int LF_TW = 64, LF_TH = 32;
// one reflection: exact for the positions in-plane outputs read (at most 4 outside, len >= 8);
// positions further out (a partial tile's unused tail) are only kept inside the plane
__device__ __forceinline__ int refl1(int p, int len) {
  return min(max(p < 0 ? -p : (p >= len ? 2 * len - 2 - p : p), 0), len - 1);
}
// the loops below walk a [rows][cols] region with a flat index t, t + 256, ...: (r, c) advanced
// incrementally (no division per element)
template <int COLS>
struct Walk2 {
  int r, c;
  __device__ __forceinline__ explicit Walk2(int t) : r(t / COLS), c(t - (t / COLS) * COLS) {}
  __device__ __forceinline__ void next() {
    r += 256 / COLS;
    c += 256 % COLS;
    if (c >= COLS) {
      c -= COLS;
      r++;
    }
  }
};
// RGB2Gray of one pixel: bg = b | g << 16
__device__ __forceinline__ uint32_t gray_bg(uint32_t bg, uint32_t r, uint32_t wbg) {
  typedef unsigned short us2 __attribute__((ext_vector_type(2)));
  return __builtin_amdgcn_udot2(__builtin_bit_cast(us2, bg), __builtin_bit_cast(us2, wbg), r * 4899u + (1u << 13), false) >> 14;
}
template <int CN>
__global__ __launch_bounds__(256) void k_line_maps(const uint8_t* __restrict__ img, int pitch, long long fstride,
                                                   int w, int h, int MP, int k0, int k1, int k2, int vec,
                                                   uint8_t* __restrict__ blur, int16_t* __restrict__ dxo,
                                                   int16_t* __restrict__ dyo, uint16_t* __restrict__ code,
                                                   uint16_t* __restrict__ moves, uint16_t* __restrict__ amask) {
  constexpr int GW = LF_TW + 8, GH = LF_TH + 8;  // gray: halo 4 (blur 2 + Sobel 1 + moves 1)
  constexpr int BW = LF_TW + 4, BH = LF_TH + 4;  // blur: halo 2
  constexpr int CW = LF_TW + 2, CH = LF_TH + 2;  // code: halo 1
  constexpr int RW = GW * CN, RD = RW / 4;       // a staged row: bytes, dwords
  constexpr int NL = (GH * RD + 255) / 256;      // dword loads per thread
  __shared__ __attribute__((aligned(16))) uint8_t raw[CN == 1 ? 16 : GH * RW];
  __shared__ __attribute__((aligned(16))) uint8_t g[GH][GW];
  __shared__ __attribute__((aligned(16))) uint16_t hs[GH][BW];
  __shared__ __attribute__((aligned(16))) uint8_t bl[BH][BW];
  __shared__ uint16_t cd[CH][CW];
  __shared__ uint32_t am[LF_TW / 2];
  const int f = blockIdx.z, x0 = blockIdx.x * LF_TW, y0 = blockIdx.y * LF_TH, t = threadIdx.x;
  const uint8_t* G = img + f * fstride;
  const long long fo = (long long)f * w * h;
  if (t < LF_TW / 2) am[t] = 0u;
  if (vec && x0 >= 4 && x0 + LF_TW + 4 <= w) {
    // an inner tile: its rows (reflected at the top / bottom) staged with aligned 4-byte
    // loads, all in flight before the first LDS store
    uint32_t v[NL];
    const uint8_t* base = G + (long long)(x0 - 4) * CN;
#pragma unroll
    for (int k = 0; k < NL; k++) {
      const int i = t + 256 * k, r = i / RD, c = i - r * RD;
      v[k] = 0u;
      if (i < GH * RD) v[k] = *(const uint32_t*)(base + (long long)refl1(y0 - 4 + r, h) * pitch + 4 * c);
    }
#pragma unroll
    for (int k = 0; k < NL; k++) {
      const int i = t + 256 * k, r = i / RD, c = i - r * RD;
      if (i < GH * RD) {
        if (CN == 1)
          *(uint32_t*)&g[r][4 * c] = v[k];
        else
          *(uint32_t*)&raw[r * RW + 4 * c] = v[k];
      }
    }
    if (CN == 3) {
      // 4 pixels (3 dwords: b0 g0 r0 b1 | g1 r1 b2 g2 | r2 b3 g3 r3) per item: each pixel's
      // (b, g) as a u16 pair through v_perm, one v_dot2 with (1868, 9617) on r * 4899 + 2^13
      __syncthreads();
      constexpr uint32_t WBG = 1868u | 9617u << 16;
      for (Walk2<GW / 4> q(t); q.r < GH; q.next()) {
        const uint32_t* p = (const uint32_t*)&raw[q.r * RW + 12 * q.c];
        const uint32_t d0 = p[0], d1 = p[1], d2 = p[2];
        const uint32_t g0 = gray_bg(__builtin_amdgcn_perm(d0, d0, 0x0c010c00u), (d0 >> 16) & 0xffu, WBG);
        const uint32_t g1 = gray_bg(__builtin_amdgcn_perm(d0, d1, 0x0c000c07u), (d1 >> 8) & 0xffu, WBG);
        const uint32_t g2 = gray_bg(__builtin_amdgcn_perm(d1, d1, 0x0c030c02u), d2 & 0xffu, WBG);
        const uint32_t g3 = gray_bg(__builtin_amdgcn_perm(d2, d2, 0x0c020c01u), d2 >> 24, WBG);
        *(uint32_t*)&g[q.r][4 * q.c] = g0 | g1 << 8 | g2 << 16 | g3 << 24;
      }
    } else if (CN == 4) {
      __syncthreads();
      Walk2<GW> q(t);
      for (; q.r < GH; q.next()) {
        const uint8_t* p = &raw[q.r * RW + q.c * CN];
        g[q.r][q.c] = (uint8_t)((p[0] * 1868 + p[1] * 9617 + p[2] * 4899 + (1 << 13)) >> 14);
      }
    }
  } else {
    // a border tile: gray at reflected coordinates (BORDER_REFLECT_101 of the blur's input)
    constexpr int NE = (GH * GW + 255) / 256;
    uint8_t v[NE][CN];
#pragma unroll
    for (int k = 0; k < NE; k++) {
      const int i = t + 256 * k, r = i / GW, c = i - r * GW;
#pragma unroll
      for (int j = 0; j < CN; j++) v[k][j] = 0;
      if (i < GH * GW) {
        const uint8_t* p = G + (long long)refl1(y0 - 4 + r, h) * pitch + (long long)refl1(x0 - 4 + c, w) * CN;
#pragma unroll
        for (int j = 0; j < CN; j++) v[k][j] = p[j];
      }
    }
#pragma unroll
    for (int k = 0; k < NE; k++) {
      const int i = t + 256 * k, r = i / GW, c = i - r * GW;
      if (i < GH * GW)
        g[r][c] = CN == 1 ? v[k][0] : (uint8_t)((v[k][0] * 1868 + v[k][1] * 9617 + v[k][2] * 4899 + (1 << 13)) >> 14);
    }
  }
  __syncthreads();
  // horizontal taps, 4 outputs per item from the row's bytes c .. c + 7 (two dwords): output k
  // is v_dot4(bytes k .. k + 3, (k0, k1, k2, k1)) + k0 * byte k + 4 (the taps are < 256 and
  // sum to 257: a sum is <= 65535 and fits 16 bits)
  {
    const uint32_t tp = (uint32_t)k0 | (uint32_t)k1 << 8 | (uint32_t)k2 << 16 | (uint32_t)k1 << 24;
    for (Walk2<BW / 4> q(t); q.r < GH; q.next()) {
      const uint32_t d0 = *(const uint32_t*)&g[q.r][4 * q.c], d1 = *(const uint32_t*)&g[q.r][4 * q.c + 4];
      const uint32_t o0 = __builtin_amdgcn_udot4(d0, tp, (d1 & 0xffu) * k0, false);
      const uint32_t o1 = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d1, d0, 1), tp, ((d1 >> 8) & 0xffu) * k0, false);
      const uint32_t o2 = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d1, d0, 2), tp, ((d1 >> 16) & 0xffu) * k0, false);
      const uint32_t o3 = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d1, d0, 3), tp, (d1 >> 24) * k0, false);
      *(uint2*)&hs[q.r][4 * q.c] = make_uint2(o0 | o1 << 16, o2 | o3 << 16);
    }
  }
  __syncthreads();
  for (Walk2<BW / 4> q(t); q.r < BH; q.next()) {  // blur at (x0 - 2 + c, y0 - 2 + r), 4 per item
    const int r = q.r, c4 = 4 * q.c;
    uint2 a[5];
#pragma unroll
    for (int i = 0; i < 5; i++) a[i] = *(const uint2*)&hs[r + i][c4];
    uint32_t pk = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int sh = 16 * (k & 1);
      auto H = [&](int i) { return (int)(((k < 2 ? a[i].x : a[i].y) >> sh) & 0xffffu); };
      const int sm = k0 * (H(0) + H(4)) + k1 * (H(1) + H(3)) + k2 * H(2);
      pk |= (uint32_t)min((sm + (1 << 15)) >> 16, 255) << (8 * k);
    }
    *(uint32_t*)&bl[r][c4] = pk;
    const int y = y0 - 2 + r;
    if (r >= 2 && r < BH - 2 && y < h) {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int c = c4 + k, x = x0 - 2 + c;
        if (c >= 2 && c < BW - 2 && x < w) blur[fo + (long long)y * w + x] = (uint8_t)(pk >> (8 * k));
      }
    }
  }
  __syncthreads();
  for (Walk2<CW> q(t); q.r < CH; q.next()) {  // code at (x0 - 1 + c, y0 - 1 + r)
    const int r = q.r, c = q.c;
    const int a = bl[r][c], b = bl[r][c + 1], cc = bl[r][c + 2];
    const int d = bl[r + 1][c], e = bl[r + 1][c + 2];
    const int gg = bl[r + 2][c], hh = bl[r + 2][c + 1], k = bl[r + 2][c + 2];
    const int gx = (cc - a) + 2 * (e - d) + (k - gg);
    const int gy = (gg - a) + 2 * (hh - b) + (k - cc);
    const int ax = abs(gx), ay = abs(gy), sm = ax + ay;
    const int tz = sm > LN_GRAD_TH + 1 ? sm : 0;             // threshold(TOZERO, 81)
    const int qv = __float2int_rn(fmul((float)tz, 0.25f));   // saturate_cast<short>(v * 0.25f)
    const uint16_t cv = (uint16_t)(qv | (ax < ay ? LN_HORIZ : 0));
    cd[r][c] = cv;
    const int x = x0 - 1 + c, y = y0 - 1 + r;
    if (r >= 1 && r < CH - 1 && c >= 1 && c < CW - 1 && x < w && y < h) {
      const long long o = fo + (long long)y * w + x;
      dxo[o] = (int16_t)gx;
      dyo[o] = (int16_t)gy;
      code[o] = cv;
    }
  }
  __syncthreads();
  // anchors (:1683-1693): the candidates (odd x <= w - 2, odd y <= h - 2) of the tile, as one
  // 16-bit row mask per candidate column; k_line_anchors orders them
  for (int i = t; i < (LF_TW / 2) * (LF_TH / 2); i += 256) {
    const int cl = i & (LF_TW / 2 - 1), jb = i / (LF_TW / 2);
    const int r = 2 + 2 * jb, c = 2 + 2 * cl;  // cd index of (x0 + 1 + 2 cl, y0 + 1 + 2 jb)
    if (x0 + c - 1 <= w - 2 && y0 + r - 1 <= h - 2) {
      const int cv = cd[r][c], gv = cv & 0x7fff;
      const bool an = (cv & LN_HORIZ)
                          ? (gv >= (cd[r - 1][c] & 0x7fff) + LN_ANCHOR_TH && gv >= (cd[r + 1][c] & 0x7fff) + LN_ANCHOR_TH)
                          : (gv >= (cd[r][c - 1] & 0x7fff) + LN_ANCHOR_TH && gv >= (cd[r][c + 1] & 0x7fff) + LN_ANCHOR_TH);
      if (an) atomicOr(&am[cl], 1u << jb);
    }
  }
  for (Walk2<LF_TW> q(t); q.r < LF_TH; q.next()) {  // move words of the tile (see lm_nibble)
    const int r = q.r, c = q.c, x = x0 + c, y = y0 + r;
    if (x >= w || y >= h) continue;
    const int cv = cd[r + 1][c + 1];
    int m = 0;
    if (cv & 0x7fff) {
      // the walk compares gImg_ read as unsigned char (gValue1..3, :1643): the code's low byte;
      // a neighbour outside the plane is never read (the border stops that direction)
      auto gb = [&](int dx, int dy) { return (int)(uint8_t)cd[r + 1 + dy][c + 1 + dx]; };
      // a step onto a non-edge pixel ends the walk there (the pixel is not taken): that step is
      // stored as the border's (0, 0), so the walk never reads a non-edge pixel's word
      auto to_edge = [&](int nb) {
        if (nb == LM_STOP) return nb;
        const int dx = (nb & 3) - 1, dy = (nb >> 2) - 1;
        return (cd[r + 1 + dy][c + 1 + dx] & 0x7fff) ? nb : LM_STOP;
      };
      if (cv & LN_HORIZ) {  // st 0, 1: LEFT; st 2, 3: RIGHT
        const int rt = (x == w - 1 || y == 0 || y == h - 1) ? 3 : ln_pick(gb(1, -1), gb(1, 0), gb(1, 1));
        const int lf = (x == 0 || y == 0 || y == h - 1) ? 3 : ln_pick(gb(-1, -1), gb(-1, 0), gb(-1, 1));
        const int nl = to_edge(lm_nibble(true, 0, lf)), nr = to_edge(lm_nibble(true, 1, rt));
        m = nl | nl << 4 | nr << 8 | nr << 12;
      } else {  // st 0, 2: UP; st 1, 3: DOWN
        const int dn = (x == 0 || x == w - 1 || y == h - 1) ? 3 : ln_pick(gb(1, 1), gb(0, 1), gb(-1, 1));
        const int up = (x == 0 || x == w - 1 || y == 0) ? 3 : ln_pick(gb(1, -1), gb(0, -1), gb(-1, -1));
        const int nu = to_edge(lm_nibble(false, 0, up)), nd = to_edge(lm_nibble(false, 1, dn));
        m = nu | nd << 4 | nu << 8 | nd << 12;
      }
    }
    moves[(long long)f * MP * h + (long long)y * MP + x] = (uint16_t)m;
  }
  __syncthreads();
  if (t < LF_TW / 2)
    amask[((long long)f * gridDim.y + blockIdx.y) * (gridDim.x * (LF_TW / 2)) + blockIdx.x * (LF_TW / 2) + t] =
        (uint16_t)am[t];
}

// ---------------------------------------------------------------- anchors
// The reference's scan order is column-major (w outer, h inner, step 2, :1683-1693). k_line_maps
// leaves one 16-bit row mask per (candidate column, 32-row band); here a thread per candidate
// column (x = 1 + 2 k, blockDim.x columns per pass) counts its column, a block scan of the
// counts in column order places every column, and the column's anchors are written in row order.
__global__ __launch_bounds__(512) void k_line_anchors(const uint16_t* __restrict__ amask, int W, int H, int nty,
                                                      int ncp, uint32_t* __restrict__ anchors, int acap,
                                                      int* __restrict__ nanchor, uint32_t* __restrict__ pl_reset = nullptr,
                                                      int* __restrict__ ctl_reset = nullptr) {
  __shared__ int wsum[8], base;
  const int f = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const uint16_t* AM = amask + (long long)f * nty * ncp;
  uint32_t* A = anchors + (long long)f * acap;
  const int nw = (W - 2 + 1) / 2;
  if (t == 0) base = 0;
  __syncthreads();
  for (int k0 = 0; k0 < nw; k0 += blockDim.x) {
    const int col = k0 + t, x = 1 + 2 * col;
    int c = 0;
    if (col < nw) {
      int ty = 0;
      for (; ty + 8 <= nty; ty += 8) {  // eight masks in flight
        uint32_t m[8];
#pragma unroll
        for (int u = 0; u < 8; u++) m[u] = AM[(long long)(ty + u) * ncp + col];
#pragma unroll
        for (int u = 0; u < 8; u++) c += __popc(m[u]);
      }
      for (; ty < nty; ty++) c += __popc((uint32_t)AM[(long long)ty * ncp + col]);
    }
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
      for (int ty = 0; ty < nty; ty++)
        for (uint32_t m = AM[(long long)ty * ncp + col]; m; m &= m - 1) {
          const int y = ty * LF_TH + 1 + 2 * __builtin_ctz(m);
          if (o < acap) A[o] = (uint32_t)x | ((uint32_t)y << 16);
          o++;
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
  // k_lines_fused's length words (pending) and control words, single frames
  if (pl_reset)
    for (int i = t; i < 2 * min(base, acap); i += blockDim.x) pl_reset[i] = 0xFFFFFFFFu;
  if (ctl_reset && t < 4) ctl_reset[t] = 0;
}

// ---------------------------------------------------------------- edge drawing
// The walk reads the move words through a 128 x 64 tile of them in LDS (16 KB), reloaded
// (centred on the step's pixel) when the pixel leaves it: one round of 16 aligned 16-byte loads
// per lane. (No move word is read outside the plane: the border steps stop the walk.)
constexpr int LE_TW = 128, LE_TH = 64;
struct MoveTile {
  uint16_t* t;  // LDS [LE_TH][LE_TW]
  int x0, y0;   // origin in the plane (x0 = -LE_TW: empty)
};
__device__ __forceinline__ void tile_load(const uint16_t* __restrict__ M, int MP, int H, MoveTile& T, int x, int y) {
  T.x0 = min(max((x - LE_TW / 2) & ~7, 0), max(MP - LE_TW, 0));
  T.y0 = min(max(y - LE_TH / 2, 0), max(H - LE_TH, 0));
  const int lane = lane_id();
  uint4 v[16];
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int id = lane + 64 * k, r = id >> 4, c = (id & 15) * 8;
    v[k] = make_uint4(0u, 0u, 0u, 0u);
    if (T.y0 + r < H && T.x0 + c < MP) v[k] = *(const uint4*)(M + (long long)(T.y0 + r) * MP + T.x0 + c);
  }
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int id = lane + 64 * k, r = id >> 4, c = (id & 15) * 8;
    *(uint4*)(T.t + r * LE_TW + c) = v[k];
  }
}

// one walk from (x, y) leaving in direction dir: its pixels appended (packed y << 16 | x) to
// P[off..], off being the reference's running offF / offS and cap its edgePixelArraySize;
// false on overflow. The whole wave runs the walk with uniform (scalar) values, lane 0 writes.
// The direction rule (:1746-2000): a Horizontal pixel keeps a horizontal lastDir, else turns
// RIGHT if x > lastX (the previous pixel's x), LEFT otherwise. A RIGHT step always has x >
// lastX and a LEFT step never, so on a Horizontal pixel the walk goes RIGHT exactly when its
// last step increased x -- and on a Vertical one DOWN exactly when the last step increased y.
// The walk's state is those two bits (px, py), initialised from dir (an anchor's first step
// leaves along dir: its own direction).
// a 4-byte store another CU reads without an acquire (WT: written through, sc1; MI355X_MICROARCH
// "Valid forms"), or a plain one
template <bool WT>
__device__ __forceinline__ void st_wt(uint32_t* p, uint32_t v) {
  if (WT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
template <bool WT>
__device__ __forceinline__ uint32_t ld_wt(const uint32_t* p) {
  if (WT) return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return *p;
}
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

template <bool WT = false>
__device__ __forceinline__ bool ed_walk_st(const uint16_t* __restrict__ M, int W, int MP, int H, uint32_t* bits,
                                           MoveTile& T, int x, int y, int st, uint32_t* __restrict__ P, uint32_t& off,
                                           uint32_t cap) {
  // st bit 1: the last step increased x (px), bit 0: it increased y (py) (see lm_nibble)
  if ((unsigned)(x - T.x0) >= (unsigned)LE_TW || (unsigned)(y - T.y0) >= (unsigned)LE_TH) tile_load(M, MP, H, T, x, y);
  // the pixel as its packed record (x | y << 16), its edge-map index, its tile offset (bytes)
  // and its tile coordinates packed like the record, all advanced by the step. The step's
  // increments of each, and the next state's nibble shift, are read from per-nibble tables in
  // lane k of a VGPR (v_readlane with the nibble as the lane): four reads instead of a decode.
  const int lane = lane_id(), ndx = (lane & 3) - 1, ndy = ((lane >> 2) & 3) - 1;
  const int t_pk = ndx + ndy * 65536, t_idx = ndx + ndy * W, t_off = 2 * (ndx + ndy * LE_TW);
  const int t_sh = 4 * ((lane & 2) | ((lane >> 3) & 1));
  int pk = x | y << 16, idx = y * W + x, tp = (x - T.x0) | (y - T.y0) << 16;
  const uint8_t* tw = (const uint8_t*)T.t + 2 * ((y - T.y0) * LE_TW + (x - T.x0));  // the pixel's word in the tile
  int sh = 4 * st;
  static_assert(LE_TW == 128 && LE_TH == 64, "the tile test mask");
  constexpr int kOut = (int)0xFFC0FF80u;  // tp outside [0, 128) x [0, 64) (a negative coordinate sets the high bits)
  // one loop exit (separate exits for the stop and the overflow cost the compiler's exit
  // bookkeeping on every step): the walk ends at a marked or non-edge pixel (stop != 0), or
  // with the pixel arrays full (an overflow: the reference returns -1)
  uint32_t* Pw = P + off;  // the next pixel record
  int rem = (int)(cap - off) - 1;  // records left after this one (< 0: the arrays are full)
  while (true) {
    const int mw = __builtin_amdgcn_readfirstlane((int)*(const uint16_t*)tw);
    const uint32_t bw = (uint32_t)__builtin_amdgcn_readfirstlane((int)bits[idx >> 5]);
    const uint32_t bit = 1u << (idx & 31);
    // marked (a walk reaches only edge pixels: a step onto a non-edge one is stored as (0, 0)),
    // or off >= cap (cap < 2^31)
    if (__builtin_expect(((bw & bit) | ((uint32_t)rem >> 31)) != 0, 0)) break;
    // every lane stores the same word to the same address (no per-step exec-mask switch;
    // the wave is the only writer of the frame's edge map)
    bits[idx >> 5] = bw | bit;
    st_wt<WT>(Pw++, (uint32_t)pk);
    rem--;
    const int nib = (mw >> sh) & 15;  // (0, 0) at the border: the pixel is marked, the walk stops next
    const int dpk = __builtin_amdgcn_readlane(t_pk, nib);
    pk += dpk;
    tp += dpk;
    idx += __builtin_amdgcn_readlane(t_idx, nib);
    tw += __builtin_amdgcn_readlane(t_off, nib);
    sh = __builtin_amdgcn_readlane(t_sh, nib);
    if (__builtin_expect((tp & kOut) != 0, 0)) {  // left the tile
      const int xx = pk & 0xffff, yy = pk >> 16;
      tile_load(M, MP, H, T, xx, yy);
      tp = (xx - T.x0) | (yy - T.y0) << 16;
      tw = (const uint8_t*)T.t + 2 * ((yy - T.y0) * LE_TW + (xx - T.x0));
    }
  }
  // stopped at a marked pixel (true), or the arrays are full there (an overflow)
  const bool stop = (bits[idx >> 5] >> (idx & 31)) & 1u;
  off = cap - 1 - (uint32_t)rem;
  return stop;
}
__device__ __forceinline__ bool ed_walk(const uint16_t* __restrict__ M, int W, int MP, int H, uint32_t* bits,
                                        MoveTile& T, int x, int y, int dir, uint32_t* __restrict__ P, uint32_t& off,
                                        uint32_t cap) {
  return ed_walk_st(M, W, MP, H, bits, T, x, y, dir == LN_RIGHT ? 2 : (dir == LN_DOWN ? 1 : 0), P, off, cap);
}

// EdgeDrawing's anchor loop (:1695-2327), one wave per frame. Anchors are taken 64 at a time
// (one per lane, with their code word (direction)); the ones an earlier walk has marked are dropped by one
// ballot after each walk, so an anchor costs no round trip of its own. Both parts of a chain
// go to P1 / P2 at the reference's running offsets offF / offS (a short chain's pixels are
// overwritten by the next walk, as there); chain e is P1[fS[e], fS[e + 1]) reversed, then
// P2[sS[e] + 1, sS[e + 1]) (the second part without its copy of the anchor), and it starts at
// fS[e] + sS[e] - e in the assembled chain array Q. STREAM (k_edge_lines): each kept chain is
// published to the workgroup's line waves as soon as it is complete (*pub = chains complete,
// release); the walk's pixel stores are made visible to them first. Returns the number of
// chains, or -1 where the reference returns -1.
template <bool STREAM>
__device__ int ed_walker(const uint16_t* __restrict__ M, const uint16_t* __restrict__ C, int W, int H, int MP,
                         const uint32_t* __restrict__ A, int na,
                         int acap, uint32_t* __restrict__ P1, uint32_t* __restrict__ P2, int pcap, int ecap,
                         uint32_t* bits, uint32_t* fS, uint32_t* sS, MoveTile& T, int* pub) {
  const int lane = lane_id();
  const int nb = (W * H + 31) / 32;
  for (int i = lane; i < nb; i += 64) bits[i] = 0;
  if (lane == 0) {
    fS[0] = 0;
    sS[0] = 0;
  }
  uint32_t b1 = 0, b2 = 0;  // offF / offS after the last kept chain
  int ne = 0;               // offPS
  bool fail = na > acap;    // anchorsSize > edgePixelArraySize (acap is that size)
  for (int a0 = 0; a0 < na && !fail; a0 += 64) {
    const int a = a0 + lane;
    const uint32_t ap = a < na ? A[a] : 0u;
    const int ax = (int)(ap & 0xffffu), ay = (int)(ap >> 16), aidx = ay * W + ax;
    const int acv = a < na ? (int)C[(long long)ay * W + ax] : 0;  // the anchor's code (its direction)
    uint64_t pend = ballot(a < na);
    while (true) {
      pend &= ~ballot(((bits[aidx >> 5] >> (aidx & 31)) & 1u) != 0);  // edgeImg_[anchor] set: skipped
      if (!pend) break;
      const int k = __builtin_ctzll(pend);
      pend &= pend - 1;
      if (ne > ecap) {  // offPS > maxNumOfEdge
        fail = true;
        break;
      }
      const int x = __builtin_amdgcn_readlane(ax, k), y = __builtin_amdgcn_readlane(ay, k);
      const bool horiz = (__builtin_amdgcn_readlane(acv, k) & LN_HORIZ) != 0;
      uint32_t o1 = b1, o2 = b2;
      if (!ed_walk(M, W, MP, H, bits, T, x, y, horiz ? LN_RIGHT : LN_DOWN, P1, o1, (uint32_t)pcap)) {
        fail = true;
        break;
      }
      const int idx = y * W + x;
      if (lane == 0) bits[idx >> 5] &= ~(1u << (idx & 31));  // the second part walks the anchor again
      if (!ed_walk(M, W, MP, H, bits, T, x, y, horiz ? LN_LEFT : LN_UP, P2, o2, (uint32_t)pcap)) {
        fail = true;
        break;
      }
      if ((int)((o1 - b1) + (o2 - b2)) < LN_MIN_LEN + 1) continue;  // short edge: dropped, its pixels stay marked
      b1 = o1;
      b2 = o2;
      ne++;
      if (ne <= ecap + 1 && lane == 0) {  // the end of chain ne - 1 = the start of the next
        fS[ne] = b1;
        sS[ne] = b2;
      }
      if (STREAM) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // the chain's pixels and bounds first
        if (lane == 0) __hip_atomic_store(pub, ne, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  }
  if (ne > ecap) fail = true;
  return fail ? -1 : ne;
}

__global__ __launch_bounds__(64) void k_edge_draw(const uint16_t* __restrict__ moves, const uint16_t* __restrict__ code,
                                                  int W, int H, int MP,
                                                  const uint32_t* __restrict__ anchors, const int* __restrict__ nanchor,
                                                  int acap, uint32_t* __restrict__ p1, uint32_t* __restrict__ p2,
                                                  int pcap, uint32_t* __restrict__ chains, uint32_t* __restrict__ sid,
                                                  int ecap, int* __restrict__ nedge, uint32_t* __restrict__ gstarts) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_ed[];
  const int f = blockIdx.x, lane = threadIdx.x;
  const int nb = (W * H + 31) / 32, nbp = (nb + 3) & ~3, ep = (ecap + 2 + 3) & ~3;
  uint32_t* bits = lds_ed;
  // the kept chains' offF / offS starts (the reference's fS / sS): in LDS after the bitmap, or in
  // global memory (gstarts, frames whose bitmap + starts exceed the LDS; edge_draw_lds)
  uint32_t* fS = gstarts ? gstarts + (long long)f * 2 * ep : bits + nbp;
  uint32_t* sS = fS + ep;
  MoveTile T{(uint16_t*)(bits + nbp + (gstarts ? 0 : 2 * ep)), -LE_TW, -LE_TH};
  uint32_t* P1 = p1 + (long long)f * pcap;
  uint32_t* P2 = p2 + (long long)f * pcap;
  uint32_t* Q = chains + (long long)f * 2 * pcap;
  uint32_t* S = sid + (long long)f * (ecap + 1);
  const int ne = ed_walker<false>(moves + (long long)f * MP * H, code + (long long)f * W * H, W, H, MP, anchors + (long long)f * acap, nanchor[f],
                                  acap, P1, P2, pcap, ecap, bits, fS, sS, T, nullptr);
  if (ne < 0) {
    if (lane == 0) nedge[f] = -1;
    return;
  }
  __syncthreads();  // lane 0's P1 / P2 stores complete, fS / sS visible
  for (int e = lane; e <= ne; e += 64) S[e] = fS[e] + sS[e] - (uint32_t)e;
  const uint32_t b1 = fS[ne], b2 = sS[ne];
  int e = 0;
  for (uint32_t t = lane; t < b1; t += 64) {  // part 1 of chain e, reversed
    while (fS[e + 1] <= t) e++;
    Q[fS[e] + sS[e] - (uint32_t)e + fS[e + 1] - 1 - t] = P1[t];
  }
  e = 0;
  for (uint32_t t = lane; t < b2; t += 64) {  // part 2 without its first pixel (the anchor)
    while (sS[e + 1] <= t) e++;
    if (t > sS[e]) Q[fS[e + 1] + t - (uint32_t)e - 1] = P2[t];
  }
  if (lane == 0) nedge[f] = ne;
}

// ---------------------------------------------------------------- speculative edge drawing
// The latency path (a single frame, EAO_LINES_SPEC): EdgeDrawing split into a parallel and a
// sequential phase that give the walks of ed_walker exactly.
//
// A walk step depends only on the pixel and the two-bit state (the move words), and the edge map
// enters a walk only as its stop test. So the walk of anchor a in direction d, run with no marks
// but its own (ls_walk: stopping where it would revisit one of its own pixels, or at a stop step),
// visits p0, p1, ..., p(k-1); the reference's walk, run after all earlier walks (and, for the
// second part, after the anchor's first part), visits the prefix p0 .. p(i-1) where p(i) is the first
// pixel those earlier walks marked (or k): no pixel before that prefix's end is marked, so the two
// walks take the same steps up to it. Phase 1 (k_walk_spec) computes every (anchor, direction)
// path in parallel, one wave per walk, up to LS_CAP pixels; phase 2 (k_walk_merge) replays the
// anchor loop of ed_walker in order on one wave, taking each part as that prefix, found 64 pixels
// at a time against the LDS edge bitmap (a ballot of the marked ones; the pixels before the first
// are marked and recorded in one round), and continues a path cut at LS_CAP with the sequential
// ed_walk from its stored position and state.
__device__ __forceinline__ uint32_t px_x(uint32_t p) { return p & 0xffffu; }
__device__ __forceinline__ uint32_t px_y(uint32_t p) { return p >> 16; }
constexpr int LS_CAP = 256;          // pixels stored per speculative walk
#define LS_FENCE() __asm__ volatile("" ::: "memory")  // compiler order of one wave's LDS accesses
constexpr uint16_t LS_SEEN = 0xFFFF;  // a tile word no pixel has (nibble 15 never occurs): visited

// ed_walk with the initial state given (a capped speculative walk's continuation)
__device__ __forceinline__ int ls_state(int dir) { return dir == LN_RIGHT ? 2 : (dir == LN_DOWN ? 1 : 0); }

// Phase 1, one walk by one wave: the path with own marks only, kept as visited marks in the wave's
// private move tile (a visited pixel's word becomes LS_SEEN, which is the stop test); when the tile
// moves, the pixels of the path so far that fall in the new tile are marked again from the LDS copy
// of the path. Writes the pixels (packed x | y << 16) to out[0 .. n), returns n | (capped << 31) and,
// for a capped walk, the next pixel and state in *next (pixel | st << 30).
template <bool WT = false>
__device__ __forceinline__ uint32_t ls_walk(const uint16_t* __restrict__ M, int MP, int H, MoveTile& T, uint32_t* path,
                                            int x, int y, int st, uint32_t* __restrict__ out, uint32_t* next) {
  const int lane = lane_id(), ndx = (lane & 3) - 1, ndy = ((lane >> 2) & 3) - 1;
  const int t_pk = ndx + ndy * 65536, t_off = 2 * (ndx + ndy * LE_TW);
  const int t_sh = 4 * ((lane & 2) | ((lane >> 3) & 1));
  tile_load(M, MP, H, T, x, y);
  int pk = x | y << 16, tp = (x - T.x0) | (y - T.y0) << 16;
  uint8_t* tw = (uint8_t*)T.t + 2 * ((y - T.y0) * LE_TW + (x - T.x0));
  int sh = 4 * st;
  constexpr int kOut = (int)0xFFC0FF80u;
  int n = 0;
  bool capped = false;
  while (true) {
    const int mw = __builtin_amdgcn_readfirstlane((int)*(const uint16_t*)tw);
    if (mw == (int)LS_SEEN) break;  // a revisit of the walk's own pixel
    if (n == LS_CAP) {
      capped = true;
      break;
    }
    *(uint16_t*)tw = LS_SEEN;  // every lane: the same word (the wave's own tile)
    path[n] = (uint32_t)pk;
    st_wt<WT>(&out[n], (uint32_t)pk);
    n++;
    const int nib = (mw >> sh) & 15;  // LM_STOP: the walk finds its own pixel next
    const int dpk = __builtin_amdgcn_readlane(t_pk, nib);
    pk += dpk;
    tp += dpk;
    tw += __builtin_amdgcn_readlane(t_off, nib);
    sh = __builtin_amdgcn_readlane(t_sh, nib);
    if (__builtin_expect((tp & kOut) != 0, 0)) {  // left the tile: reload it and mark the path again
      const int xx = pk & 0xffff, yy = pk >> 16;
      tile_load(M, MP, H, T, xx, yy);
      LS_FENCE();
      for (int j = lane; j < n; j += 64) {
        const uint32_t q = path[j];
        const int qx = (int)(q & 0xffffu) - T.x0, qy = (int)(q >> 16) - T.y0;
        if ((unsigned)qx < (unsigned)LE_TW && (unsigned)qy < (unsigned)LE_TH) T.t[qy * LE_TW + qx] = LS_SEEN;
      }
      LS_FENCE();
      tp = (xx - T.x0) | (yy - T.y0) << 16;
      tw = (uint8_t*)T.t + 2 * ((yy - T.y0) * LE_TW + (xx - T.x0));
    }
  }
  if (capped && lane == 0) st_wt<WT>(next, (uint32_t)pk | (uint32_t)(sh >> 2) << 30);
  return (uint32_t)n | (capped ? 0x80000000u : 0u);
}

// Phase 1: walk w = 2 a + d of frame f (a the anchor in scan order, d 0 its first part -- RIGHT or
// DOWN --, 1 its second -- LEFT or UP --), one wave per walk, the walks of all frames grid-strided.
// LDS per wave: the move tile and the path's LDS copy.
__global__ __launch_bounds__(64) void k_walk_spec(const uint16_t* __restrict__ moves, const uint16_t* __restrict__ code,
                                                  int W, int H, int MP, const uint32_t* __restrict__ anchors,
                                                  const int* __restrict__ nanchor, int acap,
                                                  uint32_t* __restrict__ ps, uint32_t* __restrict__ pl,
                                                  uint32_t* __restrict__ pe) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_ls[];
  const int f = blockIdx.y;
  const int na = min(nanchor[f], acap);
  MoveTile T{(uint16_t*)lds_ls, -LE_TW, -LE_TH};
  uint32_t* path = lds_ls + LE_TW * LE_TH / 2;
  const uint16_t* M = moves + (long long)f * MP * H;
  const uint16_t* C = code + (long long)f * W * H;
  for (int w = blockIdx.x; w < 2 * na; w += gridDim.x) {
    const uint32_t ap = anchors[(long long)f * acap + (w >> 1)];
    const int x = (int)(ap & 0xffffu), y = (int)(ap >> 16);
    const bool horiz = (C[(long long)y * W + x] & LN_HORIZ) != 0;
    const int dir = (w & 1) == 0 ? (horiz ? LN_RIGHT : LN_DOWN) : (horiz ? LN_LEFT : LN_UP);
    const long long wi = (long long)f * 2 * acap + w;
    const uint32_t r = ls_walk(M, MP, H, T, path, x, y, ls_state(dir), ps + wi * LS_CAP, pe + wi);
    if (lane_id() == 0) pl[wi] = r;
    LS_FENCE();
  }
}

// Phase 2's pixel records go through an LDS ring to a second wave that stores them to P1 / P2: the
// merging wave then issues no global stores, so waiting for its look-ahead loads never waits for
// store completions too (the vector-memory counter retires loads and stores in one order).
constexpr int LS_RING = 2048;  // records: (part << 31 | index into P1 / P2, pixel)
struct LsRing {
  uint2* r;
  int *wpos, *rpos;
  int rseen;  // the writer's position as last read (re-read only when the ring may be full)
};

// The ring writer stores 64 records per instruction. A short edge the merge drops leaves records at
// positions the next walk records again (its start is not advanced), and both can fall in one
// 64-record chunk: two lanes storing to one address in one instruction, whose winner the hardware
// does not order. A record is stored only if no later record of its chunk has the same target
// (the later one is the merge's final word for that position).
__device__ __forceinline__ bool ring_last_in_chunk(uint32_t key, bool valid) {
  const int lane = lane_id();
  // a later record can target an earlier one's position only after a restart: a record at or
  // below the highest earlier position of its part in the chunk (exclusive prefix maxima, one
  // per part). Chunks without one -- nearly all -- store every record.
  const bool rec = valid && !(key & 0x40000000u);  // pixel records (markers have bit 30)
  const int pos = (int)(key & 0x7fffffffu), part = (int)(key >> 31);
  int m1 = rec && part == 0 ? pos : -1, m2 = rec && part == 1 ? pos : -1;
  int p1 = __shfl_up(m1, 1, 64), p2 = __shfl_up(m2, 1, 64);
  if (lane == 0) p1 = p2 = -1;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int t1 = __shfl_up(p1, d, 64), t2 = __shfl_up(p2, d, 64);
    if (lane >= d) {
      p1 = max(p1, t1);
      p2 = max(p2, t2);
    }
  }
  if (!ballot(rec && pos <= (part == 0 ? p1 : p2))) return valid;
  bool later = false;
  for (int d = 1; d < 64; d++) {
    const uint32_t o = (uint32_t)__shfl((int)key, min(lane + d, 63), 64);
    const bool ov = __shfl((int)valid, min(lane + d, 63), 64) != 0;
    later |= lane + d < 64 && ov && o == key;
  }
  return valid && !later;
}

// Phase 2, one part of an anchor's chain: the prefix of walk wi not yet marked, recorded at
// P[off..] (part: P1 / P2) and marked, 64 pixels per round; a path cut at LS_CAP goes on with
// ed_walk from its stored next pixel and state (whose stores go straight to P). False on overflow
// (the reference's -1), as ed_walk. p is the lane's pixel of the first round, loaded ahead by the
// caller; each round loads the next one's before it tests its own.
template <bool WT = false>
__device__ __forceinline__ bool ls_part(const uint16_t* __restrict__ M, int W, int MP, int H, uint32_t* bits,
                                        MoveTile& T, const uint32_t* __restrict__ ps, uint32_t len, uint32_t nextw,
                                        uint32_t p, uint32_t* __restrict__ P, uint32_t part, uint32_t& off, uint32_t cap,
                                        LsRing& R, int& w, bool have_mk0 = false, uint64_t mk0 = 0) {
  const int lane = lane_id();
  const bool capped = (len >> 31) != 0;
  len &= 0x7fffffffu;
  for (uint32_t c0 = 0; c0 < len; c0 += 64) {
    const uint32_t i = c0 + (uint32_t)lane;
    const bool in = i < len;
    const uint32_t pn = i + 64 < len ? ld_wt<WT>(ps + i + 64) : 0u;  // the next round's pixel, in flight
    const int idx = (int)(p >> 16) * W + (int)(p & 0xffffu);
    // the first round's marked pixels may come tested already (mk0: read after every earlier mark)
    uint64_t mk;
    if (have_mk0 && c0 == 0) mk = mk0;
    else mk = ballot(in && ((bits[idx >> 5] >> (idx & 31)) & 1u));
    const uint32_t take = mk ? (uint32_t)__builtin_ctzll(mk) : min(64u, len - c0);  // pixels recorded this round
    if (take > cap - off) return false;  // the arrays fill before the walk stops
    while (w + 64 - R.rseen > LS_RING) {  // the ring may be full: look where the writer is
      R.rseen = __hip_atomic_load(R.rpos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (w + 64 - R.rseen > LS_RING) __builtin_amdgcn_s_sleep(1);
    }
    if ((uint32_t)lane < take) {
      atomicOr(&bits[idx >> 5], 1u << (idx & 31));
      R.r[(w + lane) & (LS_RING - 1)] = make_uint2(part << 31 | (off + lane), p);
    }
    w += (int)take;
    // the new write position after the records: relaxed, behind a compiler fence only -- one wave's
    // LDS operations complete in order, and a workgroup-scope release would wait for every vector
    // memory operation in flight (the look-ahead's path loads: ~1 us per anchor)
    LS_FENCE();
    if (lane == 0) __hip_atomic_store(R.wpos, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    off += take;
    if (mk) return true;  // stopped at a marked pixel
    p = pn;
  }
  if (!capped) return true;  // stopped where the speculative walk stopped (its own revisit)
  const int nx = (int)(nextw & 0xffffu), ny = (int)((nextw >> 16) & 0x3fffu), st = (int)(nextw >> 30);
  return ed_walk_st<WT>(M, W, MP, H, bits, T, nx, ny, st, P, off, cap);
}

// Phase 2: ed_walker's anchor loop over the speculative walks (wave 0), the records stored by wave 1
// from the ring, then the chain assembly of k_edge_draw by both. LDS as k_edge_draw (the tile serves
// the capped walks' continuations) plus the ring. The first round of both parts of the next pending
// anchor is loaded while the current one is merged (used when that anchor is still the next one
// after the current walk's marks).
__global__ __launch_bounds__(128) void k_walk_merge(const uint16_t* __restrict__ moves, int W, int H, int MP,
                                                    const uint32_t* __restrict__ anchors,
                                                    const int* __restrict__ nanchor, int acap,
                                                    const uint32_t* __restrict__ ps, const uint32_t* __restrict__ pl,
                                                    const uint32_t* __restrict__ pe, uint32_t* __restrict__ p1,
                                                    uint32_t* __restrict__ p2, int pcap, uint32_t* __restrict__ chains,
                                                    uint32_t* __restrict__ sid, int ecap, int* __restrict__ nedge,
                                                    uint32_t* __restrict__ gstarts, int* __restrict__ diag) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_ed[];
  __shared__ int s_w, s_r, s_done, s_ne;
  const int f = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nb = (W * H + 31) / 32, nbp = (nb + 3) & ~3, ep = (ecap + 2 + 3) & ~3;
  uint32_t* bits = lds_ed;
  uint32_t* fS = gstarts ? gstarts + (long long)f * 2 * ep : bits + nbp;
  uint32_t* sS = fS + ep;
  uint16_t* tile = (uint16_t*)(bits + nbp + (gstarts ? 0 : 2 * ep));
  LsRing R{(uint2*)(tile + LE_TW * LE_TH), &s_w, &s_r, 0};
  uint32_t* P1 = p1 + (long long)f * pcap;
  uint32_t* P2 = p2 + (long long)f * pcap;
  if (threadIdx.x == 0) s_w = s_r = s_done = 0;
  __syncthreads();
  if (wave == 0) {
    MoveTile T{tile, -LE_TW, -LE_TH};
    const uint16_t* M = moves + (long long)f * MP * H;
    const uint32_t* A = anchors + (long long)f * acap;
    const long long w0 = (long long)f * 2 * acap;
    const int na = nanchor[f];
    for (int i = lane; i < nb; i += 64) bits[i] = 0;
    if (lane == 0) {
      fS[0] = 0;
      sS[0] = 0;
    }
    uint32_t b1 = 0, b2 = 0;
    int ne = 0, w = 0;
    bool fail = na > acap;
    for (int a0 = 0; a0 < na && !fail; a0 += 64) {
      const int a = a0 + lane;
      const uint32_t ap = a < na ? A[a] : 0u;
      const int aidx = (int)(ap >> 16) * W + (int)(ap & 0xffffu);
      // both parts' lengths and continuation words of this lane's anchor, loaded ahead
      const uint32_t l1 = a < na ? pl[w0 + 2 * a] : 0u, l2 = a < na ? pl[w0 + 2 * a + 1] : 0u;
      const uint32_t e1 = a < na ? pe[w0 + 2 * a] : 0u, e2 = a < na ? pe[w0 + 2 * a + 1] : 0u;
      // lane's pixel of the first round of both parts of walk pair k (anchor a0 + k)
      auto first = [&](int k, uint32_t& q1, uint32_t& q2) {
        const long long wk = w0 + 2 * (a0 + k);
        const uint32_t n1 = (uint32_t)__builtin_amdgcn_readlane((int)l1, k) & 0x7fffffffu;
        const uint32_t n2 = (uint32_t)__builtin_amdgcn_readlane((int)l2, k) & 0x7fffffffu;
        q1 = (uint32_t)lane < n1 ? ps[wk * LS_CAP + lane] : 0u;
        q2 = (uint32_t)lane < n2 ? ps[(wk + 1) * LS_CAP + lane] : 0u;
      };
      uint64_t pend = ballot(a < na) & ~ballot(((bits[aidx >> 5] >> (aidx & 31)) & 1u) != 0);
      int k = pend ? __builtin_ctzll(pend) : -1;
      uint32_t c1 = 0, c2 = 0;
      if (k >= 0) first(k, c1, c2);
      while (k >= 0) {
        pend &= pend - 1;
        const int kn = pend ? __builtin_ctzll(pend) : -1;  // the next pending anchor as things stand
        uint32_t n1 = 0, n2 = 0;
        if (kn >= 0) first(kn, n1, n2);
        if (ne > ecap) {  // offPS > maxNumOfEdge
          fail = true;
          break;
        }
        const long long wk = w0 + 2 * (a0 + k);
        uint32_t o1 = b1, o2 = b2;
        if (!ls_part(M, W, MP, H, bits, T, ps + wk * LS_CAP, (uint32_t)__builtin_amdgcn_readlane((int)l1, k),
                     (uint32_t)__builtin_amdgcn_readlane((int)e1, k), c1, P1, 0u, o1, (uint32_t)pcap, R, w)) {
          fail = true;
          break;
        }
        const int idx = __builtin_amdgcn_readlane(aidx, k);
        if (lane == 0) bits[idx >> 5] &= ~(1u << (idx & 31));  // the second part walks the anchor again
        LS_FENCE();
        if (!ls_part(M, W, MP, H, bits, T, ps + (wk + 1) * LS_CAP, (uint32_t)__builtin_amdgcn_readlane((int)l2, k),
                     (uint32_t)__builtin_amdgcn_readlane((int)e2, k), c2, P2, 1u, o2, (uint32_t)pcap, R, w)) {
          fail = true;
          break;
        }
        if ((int)((o1 - b1) + (o2 - b2)) >= LN_MIN_LEN + 1) {  // else a short edge: dropped, its pixels stay marked
          b1 = o1;
          b2 = o2;
          ne++;
          if (ne <= ecap + 1 && lane == 0) {
            fS[ne] = b1;
            sS[ne] = b2;
          }
        }
        pend &= ~ballot(((bits[aidx >> 5] >> (aidx & 31)) & 1u) != 0);  // anchors this walk marked: skipped
        k = pend ? __builtin_ctzll(pend) : -1;
        if (k >= 0 && k == kn) {
          c1 = n1;
          c2 = n2;
        } else if (k >= 0) {
          first(k, c1, c2);
        }
      }
    }
    if (ne > ecap) fail = true;
    if (lane == 0) {
      s_ne = fail ? -1 : ne;
      __hip_atomic_store(&s_done, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  } else {
    // the writer: ring records to P1 / P2 until the merge is done and the ring drained
    int r = 0;
    while (true) {
      const int d = __hip_atomic_load(&s_done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
      const int w = __hip_atomic_load(&s_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        LS_FENCE();
      if (r < w) {
        for (int c0 = r; c0 < w; c0 += 64) {
          const int i = c0 + lane;
          const uint2 e = i < w ? R.r[i & (LS_RING - 1)] : make_uint2(0u, 0u);
          if (!ring_last_in_chunk(e.x, i < w)) continue;
          if (diag && ((e.x & 0x7fffffffu) >= (uint32_t)pcap || px_x(e.y) >= (uint32_t)W || px_y(e.y) >= (uint32_t)H))
            atomicOr(diag, 1);  // a record out of range (checking mode: not stored)
          else
            ((e.x >> 31) ? P2 : P1)[e.x & 0x7fffffffu] = e.y;
        }
        r = w;
        LS_FENCE();
        if (lane == 0) __hip_atomic_store(&s_r, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else if (d) {
        break;
      } else {
        __builtin_amdgcn_s_sleep(2);
      }
    }
  }
  __syncthreads();  // the records in P1 / P2 (both waves' stores), fS / sS visible
  const int ne = s_ne;
  if (ne < 0) {
    if (threadIdx.x == 0) nedge[f] = -1;
    return;
  }
  const int t0 = threadIdx.x, nt = blockDim.x;
  uint32_t* Q = chains + (long long)f * 2 * pcap;
  uint32_t* S = sid + (long long)f * (ecap + 1);
  for (int e = t0; e <= ne; e += nt) S[e] = fS[e] + sS[e] - (uint32_t)e;
  const uint32_t c1 = fS[ne], c2 = sS[ne];
  if (diag && threadIdx.x == 0) {  // checking mode: the chain starts in order and in range
    bool bad = c1 > (uint32_t)pcap || c2 > (uint32_t)pcap;
    for (int k = 0; k < ne && !bad; k++) bad = fS[k] > fS[k + 1] || sS[k] >= sS[k + 1];
    if (bad) atomicOr(diag, 2);
  }
  int e = 0;
  for (uint32_t t = t0; t < c1; t += nt) {  // part 1 of chain e, reversed
    while (fS[e + 1] <= t) e++;
    Q[fS[e] + sS[e] - (uint32_t)e + fS[e + 1] - 1 - t] = P1[t];
  }
  e = 0;
  for (uint32_t t = t0; t < c2; t += nt) {  // part 2 without its first pixel (the anchor)
    while (sS[e + 1] <= t) e++;
    if (t > sS[e]) Q[fS[e + 1] + t - (uint32_t)e - 1] = P2[t];
  }
  if (threadIdx.x == 0) nedge[f] = ne;
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

// EDline on one chain (:2380-2906): Q[s0, end) -> the chain's kept lines as records of 6
// words at L[s0 + 6 k] (L[s0, end) is the chain's own scratch), their count in CNT[e]; one wave
__device__ void ed_chain_lines(int e, uint32_t s0, uint32_t end, const uint32_t* __restrict__ Q, uint32_t* __restrict__ L,
                               const uint16_t* __restrict__ C, const int16_t* __restrict__ DX,
                               const int16_t* __restrict__ DY, int W, int H, double logNT, float min_length,
                               int* __restrict__ CNT) {
  const int lane = lane_id();
  auto horiz_at = [&](uint32_t i) { return (C[px_y(Q[i]) * W + px_x(Q[i])] & LN_HORIZ) != 0; };
  uint32_t s = s0;
  uint32_t offL = s;
  int nl = 0;
  double le2[2] = {0, 0};
  float ata[4], atv[2];
  while (end > s + LN_MIN_LEN) {
    double fitErr = 0;
    while (end > s + LN_MIN_LEN) {
      const bool h0 = horiz_at(s);
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
    const bool horiz = horiz_at(s);
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
          L[s0 + 6 * nl + lane] = __float_as_uint(v);
        }
        nl++;
      }
    } else {
      offL = lineStart;
    }
  }
  if (lane == 0) CNT[e] = nl;
}

// the chains' lines in chain order: a block scan of the per-chain counts; a chain's thread
// copies its records (lines past cap are counted, not stored, as the reference's nl). The whole
// workgroup; returns the line count.
__device__ int ed_place_lines(int ne, const uint32_t* __restrict__ S, const uint32_t* __restrict__ L,
                              const int* __restrict__ CNT, float* __restrict__ O, int cap) {
  __shared__ int wsum[16], carry;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
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
  return carry;
}

// ---------------------------------------------------------------- fused single-frame lines
// k_lines_fused: k_walk_spec, k_walk_merge and k_edlines_par of one frame as one launch whose
// phases overlap (the default for single frames; EAO_LINES_ONE_LAUNCH=0 restores the three launches). Workgroup 0: the merge (wave 0,
// ls_part as k_walk_merge) and the ring writer (wave 1); the other workgroups: every wave first
// computes speculative walks (grid-strided in anchor order, so the merge finds the walks of its next
// anchors done long before it reaches them: each walk's length word is released last, and the merge
// acquires the words of its next 64 anchors before their paths), then takes chains as the merge
// completes them and runs EDline on each (k_edlines_par's work, now beside the merge instead of
// after it). A completed chain reaches the ring as two marker records (its fS / sS starts, bit 30 of
// the index word); the writer stores them with the chain's pixels and releases the count of
// complete chains to the chip. k_line_anchors resets the length words and the control words.
constexpr uint32_t LS_PENDING = 0xFFFFFFFFu;  // pl of a walk not written yet (no length word has it)
constexpr uint32_t LS_MARK = 0x40000000u;      // ring record: a chain start (bit 29: sS, else fS), low bits the chain
constexpr int LF_WAVES = 4;
constexpr int LF_STAGE = 64 * 128;  // staged words per chunk: 64 anchors x 2 walks x 64 pixels
// control words per frame: [0] chains complete, [1] next chain to take, [2] 0 running / 1 done / -1 failed,
// [3] next walk to take
constexpr int LF_CTL = 4;

__device__ __forceinline__ void ls_ring_space(LsRing& R, int w, int need) {
  while (w + need - R.rseen > LS_RING) {
    R.rseen = __hip_atomic_load(R.rpos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (w + need - R.rseen > LS_RING) __builtin_amdgcn_s_sleep(1);
  }
}

__global__ __launch_bounds__(64 * LF_WAVES) void k_lines_fused(
    const uint16_t* __restrict__ moves, const uint16_t* __restrict__ code, const int16_t* __restrict__ dxi,
    const int16_t* __restrict__ dyi, int W, int H, int MP, const uint32_t* __restrict__ anchors,
    const int* __restrict__ nanchor, int acap, uint32_t* __restrict__ ps, uint32_t* __restrict__ pl,
    uint32_t* __restrict__ pe, uint32_t* __restrict__ p1, uint32_t* __restrict__ p2, int pcap,
    uint32_t* __restrict__ chains, uint32_t* __restrict__ sid, int ecap, int* __restrict__ nedge,
    uint32_t* __restrict__ gstarts, int* __restrict__ ctl, uint32_t* __restrict__ lscratch,
    uint32_t* __restrict__ ccount, float min_length, int* __restrict__ diag, unsigned long long* __restrict__ prof) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_lf[];
  __shared__ int s_w, s_r, s_done, s_ne, s_stage, s_cons;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nb = (W * H + 31) / 32, nbp = (nb + 3) & ~3, ep = (ecap + 2 + 3) & ~3;
  uint32_t* fS = gstarts;
  uint32_t* sS = gstarts + ep;
  uint32_t* P1 = p1;
  uint32_t* P2 = p2;
  const int na = nanchor[0];
  if (threadIdx.x == 0) s_w = s_r = s_done = s_stage = s_cons = 0;
  __syncthreads();
  if (blockIdx.x == 0 && wave < 3) {
    uint32_t* bits = lds_lf;
    uint16_t* tile = (uint16_t*)(bits + nbp);
    LsRing R{(uint2*)(tile + LE_TW * LE_TH), &s_w, &s_r, 0};
    // the stager's double buffer: per chunk of 64 anchors, both walks' first 64 pixels and the
    // anchors' (length, length, continuation, continuation, edge-map index) words
    uint32_t* stg = (uint32_t*)(R.r + LS_RING);
    uint32_t* meta = stg + 2 * LF_STAGE;
    if (wave == 2) {
      // the stager (wave 2): waits for the walks of chunk c, loads their first rounds and copies
      // them to LDS slot c & 1, so the merge wave issues no global loads for them (its vector-memory
      // waits -- in order -- would otherwise wait for these loads: ~1 us per anchor)
      const int nae = min(na, acap);
      for (int a0 = 0, c = 0; a0 < nae; a0 += 64, c++) {
        while (__hip_atomic_load(&s_cons, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < c - 1) {
          if (__hip_atomic_load(&s_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return;
          __builtin_amdgcn_s_sleep(1);
        }
        const int a = a0 + lane;
        uint32_t l1 = 0, l2 = 0;
        while (true) {
          l1 = a < nae ? ld_wt<true>(&pl[2 * a]) : 0u;
          l2 = a < nae ? ld_wt<true>(&pl[2 * a + 1]) : 0u;
          if (!ballot(l1 == LS_PENDING || l2 == LS_PENDING)) break;
          if (__hip_atomic_load(&s_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return;
          __builtin_amdgcn_s_sleep(1);
        }
        const uint32_t e1 = a < nae ? ld_wt<true>(&pe[2 * a]) : 0u, e2 = a < nae ? ld_wt<true>(&pe[2 * a + 1]) : 0u;
        const uint32_t ap = a < nae ? anchors[a] : 0u;
        uint32_t* st = stg + (c & 1) * LF_STAGE;
        uint32_t* mt = meta + (c & 1) * 64 * 5;
        mt[5 * lane + 0] = l1;
        mt[5 * lane + 1] = l2;
        mt[5 * lane + 2] = e1;
        mt[5 * lane + 3] = e2;
        mt[5 * lane + 4] = (ap >> 16) * (uint32_t)W + (ap & 0xffffu);
        for (int j0 = 0; j0 < 64 && a0 + j0 < nae; j0 += 8) {  // 16 loads in flight per lane
          uint32_t q[16];
#pragma unroll
          for (int j = 0; j < 8; j++) {
            const int k = j0 + j;
            const uint32_t n1 = (uint32_t)__builtin_amdgcn_readlane((int)l1, k) & 0x7fffffffu;
            const uint32_t n2 = (uint32_t)__builtin_amdgcn_readlane((int)l2, k) & 0x7fffffffu;
            const long long wk = 2 * (long long)(a0 + k);
            q[2 * j] = a0 + k < nae && (uint32_t)lane < n1 ? ld_wt<true>(ps + wk * LS_CAP + lane) : 0u;
            q[2 * j + 1] = a0 + k < nae && (uint32_t)lane < n2 ? ld_wt<true>(ps + (wk + 1) * LS_CAP + lane) : 0u;
          }
#pragma unroll
          for (int j = 0; j < 8; j++) {
            st[(j0 + j) * 128 + lane] = q[2 * j];
            st[(j0 + j) * 128 + 64 + lane] = q[2 * j + 1];
          }
        }
        LS_FENCE();  // the slot's words before its count (one wave's LDS operations complete in order)
        if (lane == 0) __hip_atomic_store(&s_stage, c + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      return;
    }
    if (wave == 0) {
      MoveTile T{tile, -LE_TW, -LE_TH};
      for (int i = lane; i < nb; i += 64) bits[i] = 0;
      LS_FENCE();
      uint32_t b1 = 0, b2 = 0;
      int ne = 0, w = 0;
      bool fail = na > acap;
      // profiling (prof != null): anchors merged; wall-clock ticks in the two parts, the
      // pending-set update, the chunk starts (waits for the stager), the whole merge
      int pn_anchor = 0;
      unsigned long long pt_p1 = 0, pt_p2 = 0, pt_pend = 0, pt_chunk = 0, pt_wait = 0;
      const unsigned long long pt_start = prof ? wall_clock64() : 0;
      int c = 0;
      for (int a0 = 0; a0 < na && !fail; a0 += 64, c++) {
        const unsigned long long tc0 = prof ? wall_clock64() : 0;
        const int a = a0 + lane;
        // the chunk's walks, staged in LDS by wave 2 (their paths and words were stored sc1 and
        // drained before their length words, and loaded sc1 there)
        while (__hip_atomic_load(&s_stage, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <= c) __builtin_amdgcn_s_sleep(1);
        LS_FENCE();
        const uint32_t* st = stg + (c & 1) * LF_STAGE;
        const uint32_t* mt = meta + (c & 1) * 64 * 5;
        const uint32_t l1 = mt[5 * lane + 0], l2 = mt[5 * lane + 1], e1 = mt[5 * lane + 2], e2 = mt[5 * lane + 3];
        const int aidx = (int)mt[5 * lane + 4];
        auto first = [&](int k, uint32_t& q1, uint32_t& q2) {
          q1 = st[k * 128 + lane];
          q2 = st[k * 128 + 64 + lane];
        };
        uint64_t pend = ballot(a < na) & ~ballot(((bits[aidx >> 5] >> (aidx & 31)) & 1u) != 0);
        int k = pend ? __builtin_ctzll(pend) : -1;
        uint32_t c1 = 0, c2 = 0;
        bool have1 = false;  // part 1's first-round marks of anchor k tested already (mk1)
        uint64_t mk1 = 0;
        if (k >= 0) first(k, c1, c2);
        if (prof) pt_chunk += wall_clock64() - tc0;
        while (k >= 0) {
          if (prof) {  // the anchor's first-round pixels arriving (profiling: drained here, timed)
            const unsigned long long tw = wall_clock64();
            vm_drain();
            pt_wait += wall_clock64() - tw;
          }
          const unsigned long long ta = prof ? wall_clock64() : 0;
          pn_anchor++;
          pend &= pend - 1;
          const int kn = pend ? __builtin_ctzll(pend) : -1;
          uint32_t n1 = 0, n2 = 0;
          if (kn >= 0) first(kn, n1, n2);
          if (ne > ecap) {
            fail = true;
            break;
          }
          const long long wk = 2 * (long long)(a0 + k);
          const uint32_t L1 = (uint32_t)__builtin_amdgcn_readlane((int)l1, k), L2 = (uint32_t)__builtin_amdgcn_readlane((int)l2, k);
          uint32_t o1 = b1, o2 = b2;
          if (!ls_part<true>(moves, W, MP, H, bits, T, ps + wk * LS_CAP, L1, (uint32_t)__builtin_amdgcn_readlane((int)e1, k), c1,
                             P1, 0u, o1, (uint32_t)pcap, R, w, have1, mk1)) {
            fail = true;
            break;
          }
          const unsigned long long tb = prof ? wall_clock64() : 0;
          const int idx = __builtin_amdgcn_readlane(aidx, k);
          if (lane == 0) atomicAnd(&bits[idx >> 5], ~(1u << (idx & 31)));  // no return: no wait
          LS_FENCE();
          if (!ls_part<true>(moves, W, MP, H, bits, T, ps + (wk + 1) * LS_CAP, L2, (uint32_t)__builtin_amdgcn_readlane((int)e2, k),
                             c2, P2, 1u, o2, (uint32_t)pcap, R, w)) {
            fail = true;
            break;
          }
          const unsigned long long tcc = prof ? wall_clock64() : 0;
          if (prof) {
            pt_p1 += tb - ta;
            pt_p2 += tcc - tb;
          }
          // a capped walk's continuation stored its pixels itself (sc1): drained before the chain's
          // markers reach the writer, whose count then covers them
          if (((L1 | L2) >> 31) != 0) vm_drain();
          if ((int)((o1 - b1) + (o2 - b2)) >= LN_MIN_LEN + 1) {
            b1 = o1;
            b2 = o2;
            ne++;
            if (ne <= ecap + 1) {  // the chain's end: its starts through the ring (the writer publishes)
              ls_ring_space(R, w, 2);
              if (lane < 2) R.r[(w + lane) & (LS_RING - 1)] = make_uint2(LS_MARK | (lane ? 0x20000000u : 0u) | (uint32_t)ne, lane ? b2 : b1);
              w += 2;
              LS_FENCE();
              if (lane == 0) __hip_atomic_store(R.wpos, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
          }
          // the anchors this walk marked, and -- in the same LDS round trip -- the first-round marks of
          // the next candidate's part 1, valid when it is still the next pending anchor
          const uint32_t ln1 = kn >= 0 ? (uint32_t)__builtin_amdgcn_readlane((int)l1, kn) & 0x7fffffffu : 0u;
          const int nidx = (int)(n1 >> 16) * W + (int)(n1 & 0xffffu);
          const bool am = ((bits[aidx >> 5] >> (aidx & 31)) & 1u) != 0;
          const bool nm = (uint32_t)lane < ln1 && ((bits[nidx >> 5] >> (nidx & 31)) & 1u);
          pend &= ~ballot(am);
          const uint64_t nmk = ballot(nm);
          k = pend ? __builtin_ctzll(pend) : -1;
          have1 = false;
          if (k >= 0 && k == kn) {
            c1 = n1;
            c2 = n2;
            have1 = true;
            mk1 = nmk;
          } else if (k >= 0) {
            first(k, c1, c2);
          }
          if (prof) pt_pend += wall_clock64() - tcc;
        }
        LS_FENCE();  // the slot's reads done: wave 2 may refill it
        if (lane == 0) __hip_atomic_store(&s_cons, c + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      if (ne > ecap) fail = true;
      if (prof && lane == 0) {
        atomicAdd(&prof[0], (unsigned long long)pn_anchor);
        atomicAdd(&prof[3], pt_p1);
        atomicAdd(&prof[4], pt_p2);
        atomicAdd(&prof[5], pt_pend);
        atomicAdd(&prof[6], pt_chunk);
        atomicAdd(&prof[7], wall_clock64() - pt_start);
        atomicAdd(&prof[8], (unsigned long long)na);
        atomicAdd(&prof[9], (unsigned long long)ne);
        atomicAdd(&prof[10], 1ull);
        atomicAdd(&prof[11], pt_wait);
      }
      if (lane == 0) {
        s_ne = fail ? -1 : ne;
        __hip_atomic_store(&s_done, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    } else {
      // the writer: ring records to P1 / P2 and chain starts to fS / sS; after each batch that
      // completed chains, the count released to the chip
      if (lane == 0) {
        st_wt<true>(fS, 0u);
        st_wt<true>(sS, 0u);
      }
      int r = 0;
      while (true) {
        const int d = __hip_atomic_load(&s_done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        const int w = __hip_atomic_load(&s_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        LS_FENCE();
        if (r < w) {
          int pub = 0;
          for (int c0 = r; c0 < w; c0 += 64) {
            const int i = c0 + lane;
            const uint2 e = i < w ? R.r[i & (LS_RING - 1)] : make_uint2(0u, 0u);
            // (markers' words are unique: bit 30 set, the chain count below it)
            if (!ring_last_in_chunk(e.x, i < w)) continue;
            if (e.x & LS_MARK) {
              const int c = (int)(e.x & 0x1fffffffu);
              st_wt<true>(((e.x & 0x20000000u) ? sS : fS) + c, e.y);
              pub = max(pub, c);
            } else if (diag && ((e.x & 0x7fffffffu) >= (uint32_t)pcap || px_x(e.y) >= (uint32_t)W || px_y(e.y) >= (uint32_t)H)) {
              atomicOr(diag, 1);
            } else {
              st_wt<true>(((e.x >> 31) ? P2 : P1) + (e.x & 0x7fffffffu), e.y);
            }
          }
          r = w;
          LS_FENCE();
          if (lane == 0) __hip_atomic_store(&s_r, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          pub = wave_max_int(pub);
          if (pub > 0) {
            vm_drain();  // the chains' pixels and starts (sc1), then their count
            if (lane == 0) st_wt<true>((uint32_t*)&ctl[0], (uint32_t)pub);
          }
        } else if (d) {
          break;
        } else {
          __builtin_amdgcn_s_sleep(2);
        }
      }
      const int ne = s_ne;
      if (lane == 0) {
        nedge[0] = ne;  // for k_lines_place (the next launch)
        vm_drain();
        st_wt<true>((uint32_t*)&ctl[2], (uint32_t)(ne < 0 ? -1 : 1));
      }
    }
    return;
  }
  // ---- speculative walks (workgroups >= 1), then EDline on the completed chains (every wave)
  if (blockIdx.x > 0) {
    uint8_t* base = (uint8_t*)lds_lf + (size_t)wave * (sizeof(uint16_t) * LE_TW * LE_TH + 4 * LS_CAP);
    MoveTile T{(uint16_t*)base, -LE_TW, -LE_TH};
    uint32_t* path = (uint32_t*)(base + sizeof(uint16_t) * LE_TW * LE_TH);
    // walks are claimed in anchor order from a counter, not assigned by workgroup: whichever
    // workgroups are resident do every walk the merge waits for, so the launch progresses with any
    // number of them on the chip (others of its kind, or other work, may hold the rest of the CUs)
    const int nw2 = 2 * min(na, acap);
    for (;;) {
      int w = 0;
      if (lane == 0) w = __hip_atomic_fetch_add(&ctl[3], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      w = __shfl(w, 0, 64);
      if (w >= nw2) break;
      const uint32_t ap = anchors[w >> 1];
      const int x = (int)(ap & 0xffffu), y = (int)(ap >> 16);
      const bool horiz = (code[(long long)y * W + x] & LN_HORIZ) != 0;
      const int dir = (w & 1) == 0 ? (horiz ? LN_RIGHT : LN_DOWN) : (horiz ? LN_LEFT : LN_UP);
      const uint32_t r = ls_walk<true>(moves, MP, H, T, path, x, y, ls_state(dir), ps + (long long)w * LS_CAP, pe + w);
      vm_drain();  // the path and continuation word (sc1) before the length word
      if (lane == 0) st_wt<true>(&pl[w], r);
      LS_FENCE();
    }
  }
  const double logNT = 2.0 * (log10((double)W) + log10((double)H));
  int* CNT = (int*)ccount;
  while (true) {
    int e = 0;
    if (lane == 0) e = __hip_atomic_fetch_add(&ctl[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    e = __shfl(e, 0, 64);
    int st = 0, rd = 0;
    while (true) {  // chain e complete, or the merge over
      st = (int)ld_wt<true>((const uint32_t*)&ctl[2]);
      rd = (int)ld_wt<true>((const uint32_t*)&ctl[0]);
      if (rd > e || st != 0) break;
      // a few us between polls: ~100 waiting waves must not load the fabric the frame's other
      // kernels (the drop-in's extraction and matching beside the lines) depend on
      __builtin_amdgcn_s_sleep(127);
    }
    if (st < 0 || rd <= e) break;
    const uint32_t f0 = ld_wt<true>(fS + e), f1 = ld_wt<true>(fS + e + 1), s0 = ld_wt<true>(sS + e),
                   s1 = ld_wt<true>(sS + e + 1);
    const uint32_t q0 = f0 + s0 - (uint32_t)e, q1 = f1 + s1 - (uint32_t)e - 1;
    if (diag && (f1 < f0 || s1 <= s0 || f1 > (uint32_t)pcap || s1 > (uint32_t)pcap)) {
      atomicOr(diag, 8);
      if (lane == 0) CNT[e] = 0;
      continue;
    }
    for (uint32_t i = lane; i < f1 - f0; i += 64) chains[q0 + i] = ld_wt<true>(P1 + f1 - 1 - i);
    for (uint32_t i = lane + 1; i < s1 - s0; i += 64) chains[q0 + (f1 - f0) + i - 1] = ld_wt<true>(P2 + s0 + i);
    if (lane == 0) sid[e] = q0;
    ed_chain_lines(e, q0, q1, chains, lscratch, code, dxi, dyi, W, H, logNT, min_length, CNT);
  }
}

// one workgroup of LN_WAVES waves per frame: chains Q / S -> lines out [cap][6] (sx, sy, ex, ey,
// angle, length); chains are independent: wave w takes chains w, w + nw, ...
__global__ __launch_bounds__(64 * LN_WAVES) void k_edlines(const uint16_t* __restrict__ code,
                                                          const int16_t* __restrict__ dxi,
                                                          const int16_t* __restrict__ dyi, int W, int H,
                                                          const uint32_t* __restrict__ chains,
                                                          const uint32_t* __restrict__ sid,
                                                          const int* __restrict__ nedge, int pcap, int ecap,
                                                          uint32_t* __restrict__ lscratch,
                                                          uint32_t* __restrict__ ccount, float min_length,
                                                          float* __restrict__ out, int* __restrict__ nout, int cap) {
  const int f = blockIdx.x, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const long long fo = (long long)f * W * H;
  const uint32_t* Q = chains + (long long)f * 2 * pcap;
  const uint32_t* S = sid + (long long)f * (ecap + 1);
  uint32_t* L = lscratch + (long long)f * 2 * pcap;
  int* CNT = (int*)(ccount + (long long)f * (ecap + 1));  // lines kept per chain
  const int ne = nedge[f];
  if (ne < 0) {  // the whole workgroup
    if (threadIdx.x == 0) nout[f] = -1;
    return;
  }
  const double logNT = 2.0 * (log10((double)W) + log10((double)H));
  for (int e = wave; e < ne; e += nw)
    ed_chain_lines(e, S[e], S[e + 1], Q, L, code + fo, dxi + fo, dyi + fo, W, H, logNT, min_length, CNT);
  __syncthreads();
  const int n = ed_place_lines(ne, S, L, CNT, out + (long long)f * cap * 6, cap);
  if (threadIdx.x == 0) nout[f] = n;
}

// the latency path's EDline: one wave per chain over the whole chip (chains are independent), then
// the placement in chain order by one workgroup per frame. (Staging chains of <= 3072 pixels in LDS
// gained nothing, 136 -> 139 us, and the build that did faulted intermittently: DESIGN.md section 9.)
__global__ __launch_bounds__(64) void k_edlines_par(const uint16_t* __restrict__ code, const int16_t* __restrict__ dxi,
                                                   const int16_t* __restrict__ dyi, int W, int H,
                                                   const uint32_t* __restrict__ chains, const uint32_t* __restrict__ sid,
                                                   const int* __restrict__ nedge, int pcap, int ecap,
                                                   uint32_t* __restrict__ lscratch, uint32_t* __restrict__ ccount,
                                                   float min_length, int* __restrict__ diag) {
  const int f = blockIdx.y, lane = threadIdx.x;
  const int ne = nedge[f];
  const long long fo = (long long)f * W * H;
  const uint32_t* Q = chains + (long long)f * 2 * pcap;
  const uint32_t* S = sid + (long long)f * (ecap + 1);
  uint32_t* L = lscratch + (long long)f * 2 * pcap;
  int* CNT = (int*)(ccount + (long long)f * (ecap + 1));
  const double logNT = 2.0 * (log10((double)W) + log10((double)H));
  for (int e = blockIdx.x; e < ne; e += gridDim.x) {
    const uint32_t s0 = S[e], s1 = S[e + 1];
    if (diag) {  // checking mode: the chain in range, its pixels in the image (else skipped)
      bool bad = s1 < s0 || s1 > 2u * (uint32_t)pcap;
      for (uint32_t i = s0 + lane; i < s1 && !bad; i += 64) {
        const uint32_t p = Q[i];
        if (px_x(p) >= (uint32_t)W || px_y(p) >= (uint32_t)H) atomicOr(diag, 16);
      }
      if (bad) atomicOr(diag, 8);
      if (bad || __hip_atomic_load(diag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 24) {
        if (lane == 0) CNT[e] = 0;
        continue;
      }
    }
    ed_chain_lines(e, s0, s1, Q, L, code + fo, dxi + fo, dyi + fo, W, H, logNT, min_length, CNT);
  }
}
__global__ __launch_bounds__(256) void k_lines_place(const uint32_t* __restrict__ sid, const int* __restrict__ nedge,
                                                     int pcap, int ecap, const uint32_t* __restrict__ lscratch,
                                                     const uint32_t* __restrict__ ccount, float* __restrict__ out,
                                                     int* __restrict__ nout, int cap) {
  const int f = blockIdx.x;
  const int ne = nedge[f];
  if (ne < 0) {
    if (threadIdx.x == 0) nout[f] = -1;
    return;
  }
  const int n = ed_place_lines(ne, sid + (long long)f * (ecap + 1), lscratch + (long long)f * 2 * pcap,
                               (const int*)(ccount + (long long)f * (ecap + 1)), out + (long long)f * cap * 6, cap);
  if (threadIdx.x == 0) nout[f] = n;
}

// EdgeDrawing + EDline of a frame in one workgroup: wave 0 walks (ed_walker<true>) and publishes
// each kept chain; the other LE_WAVES - 1 waves take the published chains in order (an LDS
// ticket), assemble each into Q and run EDline on it while the walk goes on, so a frame costs
// its walk plus the last chains' lines instead of the walk plus all of EDline. Four waves: EDline
// needs ~250 VGPRs, so two workgroups per CU (the LDS allows two) hold 2 waves per SIMD, and all
// 405 frames of a step run in one round over the 256 CUs (8 waves: one workgroup per CU, two
// rounds, 9.9 ms against 6.5 ms per 405 frames; r04_ab_lines.txt).
constexpr int LE_WAVES = 4;
__global__ __launch_bounds__(64 * LE_WAVES) void k_edge_lines(
    const uint16_t* __restrict__ moves, int W, int H, int MP, const uint32_t* __restrict__ anchors,
    const int* __restrict__ nanchor, int acap, uint32_t* __restrict__ p1, uint32_t* __restrict__ p2, int pcap,
    uint32_t* __restrict__ chains, uint32_t* __restrict__ sid, int ecap, int* __restrict__ nedge,
    const uint16_t* __restrict__ code, const int16_t* __restrict__ dxi, const int16_t* __restrict__ dyi,
    uint32_t* __restrict__ lscratch, uint32_t* __restrict__ ccount, float min_length, float* __restrict__ out,
    int* __restrict__ nout, int cap, uint32_t* __restrict__ gstarts) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_ed[];
  __shared__ int pub, ticket, state;  // chains published, next chain to take, 0 walking / 1 done / -1 failed
  const int f = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nb = (W * H + 31) / 32, nbp = (nb + 3) & ~3, ep = (ecap + 2 + 3) & ~3;
  uint32_t* bits = lds_ed;
  // chain starts in LDS, or in global memory (gstarts) for large frames (k_edge_draw); the line
  // waves read them after the walker's release on pub, like the chain pixels P1 / P2
  uint32_t* fS = gstarts ? gstarts + (long long)f * 2 * ep : bits + nbp;
  uint32_t* sS = fS + ep;
  uint16_t* tile = (uint16_t*)(bits + nbp + (gstarts ? 0 : 2 * ep));
  const long long fo = (long long)f * W * H;
  uint32_t* P1 = p1 + (long long)f * pcap;
  uint32_t* P2 = p2 + (long long)f * pcap;
  uint32_t* Q = chains + (long long)f * 2 * pcap;
  uint32_t* S = sid + (long long)f * (ecap + 1);
  uint32_t* L = lscratch + (long long)f * 2 * pcap;
  int* CNT = (int*)(ccount + (long long)f * (ecap + 1));
  if (threadIdx.x == 0) {
    pub = 0;
    ticket = 0;
    state = 0;
  }
  __syncthreads();
  if (wave == 0) {
    MoveTile T{tile, -LE_TW, -LE_TH};
    const int ne = ed_walker<true>(moves + (long long)f * MP * H, code + fo, W, H, MP, anchors + (long long)f * acap, nanchor[f],
                                   acap, P1, P2, pcap, ecap, bits, fS, sS, T, &pub);
    if (lane == 0) {
      nedge[f] = ne;
      __hip_atomic_store(&state, ne < 0 ? -1 : 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  } else {
    const double logNT = 2.0 * (log10((double)W) + log10((double)H));
    while (true) {
      int e = 0;
      if (lane == 0) e = atomicAdd(&ticket, 1);
      e = __shfl(e, 0, 64);
      int st = 0;
      while (true) {  // chain e published, or the walk over
        st = __hip_atomic_load(&state, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (__hip_atomic_load(&pub, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) > e || st != 0) break;
        __builtin_amdgcn_s_sleep(4);
      }
      if (st < 0 || __hip_atomic_load(&pub, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= e) break;
      const uint32_t f0 = fS[e], f1 = fS[e + 1], s0 = sS[e], s1 = sS[e + 1];
      const uint32_t q0 = f0 + s0 - (uint32_t)e, q1 = f1 + s1 - (uint32_t)e - 1;
      for (uint32_t i = lane; i < f1 - f0; i += 64) Q[q0 + i] = P1[f1 - 1 - i];
      for (uint32_t i = lane + 1; i < s1 - s0; i += 64) Q[q0 + (f1 - f0) + i - 1] = P2[s0 + i];
      if (lane == 0) S[e] = q0;
      ed_chain_lines(e, q0, q1, Q, L, code + fo, dxi + fo, dyi + fo, W, H, logNT, min_length, CNT);
    }
  }
  __syncthreads();
  if (state < 0) {
    if (threadIdx.x == 0) nout[f] = -1;
    return;
  }
  const int n = ed_place_lines(pub, S, L, CNT, out + (long long)f * cap * 6, cap);
  if (threadIdx.x == 0) nout[f] = n;
}

// ================================================================ host
struct LineEngine {
  int dev = 0, W = 0, H = 0, B = 0;
  int acap = 0, pcap = 0, ecap = 0;
  int MP = 0;  // the move words' row pitch in pixels (a multiple of 16)
  bool fused = true;  // k_edge_lines (EAO_LINES_FUSED=0: k_edge_draw, then k_edlines)
  bool gstarts = false;  // the chains' fS / sS starts in global memory (d_starts), not LDS
  bool spec = true;      // single frames through the speculative walk (EAO_LINES_SPEC=0: k_edge_lines)
  uint32_t *d_ps = nullptr, *d_pl = nullptr, *d_pe = nullptr;  // its paths / lengths / continuations (one frame)
  uint32_t* d_starts = nullptr;
  int* d_lctl = nullptr;           // k_lines_fused's control words
  unsigned long long* d_lprof = nullptr;  // its merge counters (EAO_LINES_PROF=1: printed at destroy)
  uint32_t* d_lstarts = nullptr;   // k_lines_fused's chain starts (fS / sS)
  int k[3] = {0, 0, 0};
  hipStream_t stream = nullptr;
  uint8_t* d_blur = nullptr;
  int16_t *d_dx = nullptr, *d_dy = nullptr;
  uint16_t* d_code = nullptr;
  uint16_t* d_moves = nullptr;
  uint16_t* d_amask = nullptr;  // [frame][row band][candidate column] anchor row masks
  uint32_t *d_anch = nullptr, *d_p1 = nullptr, *d_p2 = nullptr, *d_chain = nullptr, *d_sid = nullptr,
           *d_lscr = nullptr, *d_ccnt = nullptr;
  int *d_nanch = nullptr, *d_nedge = nullptr;
  uint8_t* d_img = nullptr;  // [H][W * 4]: one host frame of up to 4 channels
  float* d_lines = nullptr;
  int* d_nlines = nullptr;
  int* h_n = nullptr;  // pinned: the single-frame line count (and, checking, the diagnostic word)
  int pending_cap = -1;  // eao_lines_detect_color_start's cap while its outputs are not taken (-1: none)
  HostStage stage_in, stage_out;  // single-frame staging: the pinned image in, count + lines back
  ~LineEngine() {
    if (d_lprof) {
      unsigned long long h[16] = {0};
      if (hipMemcpy(h, d_lprof, sizeof h, hipMemcpyDeviceToHost) == hipSuccess && h[10]) {
        const double n = (double)h[10], us = 0.01;  // wall clock 100 MHz
        fprintf(stderr,
                "k_lines_fused merge per call (%llu calls): anchors %.0f (of %.0f), chains %.0f | us: pixels-arrive "
                "wait %.1f part1 %.1f part2 %.1f pend %.1f chunk starts %.1f total %.1f\n",
                h[10], h[0] / n, h[8] / n, h[9] / n, h[11] * us / n, h[3] * us / n, h[4] * us / n, h[5] * us / n,
                h[6] * us / n, h[7] * us / n);
      }
      (void)hipFree(d_lprof);
    }
    void* p[] = {d_blur, d_dx,   d_dy,    d_code,  d_moves, d_amask, d_anch,  d_p1,   d_p2,    d_chain,
                 d_sid,  d_lscr, d_ccnt,  d_nanch, d_nedge, d_img,   d_lines, d_nlines, d_starts,
                 d_ps,   d_pl,   d_pe,   d_lctl, d_lstarts};
    for (void* q : p)
      if (q) (void)hipFree(q);
    if (h_n) (void)hipHostFree(h_n);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

// getGaussianKernel(5, 1, CV_32F) -> the 8U fixed-point taps (cvRound(k * 256)): 14, 63, 103, 63, 14 --
// each < 256 and summing to 257 (<= 257), which k_line_maps' byte dot products and 16-bit row sums rely on
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

// k_edge_draw's dynamic LDS: the edge bitmap, the chains' fS / sS starts (unless they are kept in
// global memory: gstarts), the move tile
static size_t edge_draw_lds(int W, int H, int ecap, bool gstarts) {
  return ((size_t)((((W * H + 31) / 32) + 3) & ~3) + (gstarts ? 0 : 2 * (size_t)((ecap + 2 + 3) & ~3))) * 4 +
         sizeof(uint16_t) * LE_TW * LE_TH;
}
constexpr size_t kLdsMax = 160 * 1024;

}  // namespace eao

using namespace eao;
struct eao_lines {
  LineEngine e;
};

static bool lines_check() {
  static const bool on = [] { const char* v = getenv("EAO_LINES_CHECK"); return v && v[0] == '1'; }();
  return on;
}

extern "C" {

int eao_lines_create(int device, int width, int height, int max_batch, eao_lines** out) {
  if (!out) return EAO_E_ARG;
  *out = nullptr;
  if (width < 8 || height < 8 || width > 8192 || height > 8192 || max_batch < 1) return EAO_E_ARG;
  if (!eao_device_ok(device)) {
    set_error("no usable gfx950 device (the engine has no CPU fallback)");
    return EAO_E_NODEVICE;
  }
  // the same dynamic LDS k_edge_draw is launched with (edge bitmap, chain starts, move tile);
  // EdgeDrawing's arrays: edgePixelArraySize = pixels / 5, maxNumOfEdge = that / 20. Frames whose
  // chain starts do not fit beside the bitmap keep the starts in global memory (up to ~1.18 M px)
  if (edge_draw_lds(width, height, width * height / 5 / 20, true) > kLdsMax) {
    set_error("eao_lines_create: the per-frame edge bitmap and move tile exceed the LDS");
    return EAO_E_CAPACITY;
  }
  eao_lines* L = new eao_lines();
  LineEngine& e = L->e;
  e.dev = device;
  e.W = width;
  e.H = height;
  e.B = max_batch;
  e.pcap = width * height / 5;
  e.MP = (width + 15) & ~15;
  if (const char* v = getenv("EAO_LINES_FUSED")) e.fused = v[0] != '0';
  if (const char* v = getenv("EAO_LINES_SPEC")) e.spec = v[0] != '0';
  e.acap = e.pcap;
  e.ecap = e.pcap / 20;
  e.gstarts = edge_draw_lds(width, height, e.ecap, false) > kLdsMax;
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
  // the engine's stream at the highest priority (EAO_LINES_PRI=0: default priority): its own hardware
  // queue, so a single frame's one long launch (k_lines_fused) does not hold the matcher's or the
  // extractor's launches of the same frame behind it in a shared queue
  static const bool lines_pri = [] {
    const char* v = getenv("EAO_LINES_PRI");
    return !(v && v[0] == '0');
  }();
  int lo_pri = 0, hi_pri = 0;
  if (hipSetDevice(device) != hipSuccess || hipDeviceGetStreamPriorityRange(&lo_pri, &hi_pri) != hipSuccess ||
      hipStreamCreateWithPriority(&e.stream, hipStreamNonBlocking, lines_pri ? hi_pri : 0) != hipSuccess ||
      hipMalloc(&e.d_blur, px) != hipSuccess || hipMalloc(&e.d_dx, px * 2) != hipSuccess ||
      hipMalloc(&e.d_dy, px * 2) != hipSuccess || hipMalloc(&e.d_code, px * 2) != hipSuccess ||
      hipMalloc(&e.d_moves, sizeof(uint16_t) * e.MP * height * max_batch) != hipSuccess ||
      hipMalloc(&e.d_amask, (size_t)((width + LF_TW - 1) / LF_TW) * (LF_TW / 2) * ((height + LF_TH - 1) / LF_TH) * 2 *
                                max_batch) != hipSuccess ||
      hipMalloc(&e.d_anch, (size_t)e.acap * 4 * max_batch) != hipSuccess ||
      hipMalloc(&e.d_p1, (size_t)e.pcap * 4 * max_batch) != hipSuccess ||
      hipMalloc(&e.d_p2, (size_t)e.pcap * 4 * max_batch) != hipSuccess ||
      hipMalloc(&e.d_chain, (size_t)e.pcap * 8 * max_batch) != hipSuccess ||
      hipMalloc(&e.d_lscr, (size_t)e.pcap * 8 * max_batch) != hipSuccess ||
      hipMalloc(&e.d_sid, (size_t)(e.ecap + 1) * 4 * max_batch) != hipSuccess ||
      hipMalloc(&e.d_ccnt, (size_t)(e.ecap + 1) * 4 * max_batch) != hipSuccess ||
      (e.gstarts && hipMalloc(&e.d_starts, (size_t)2 * ((e.ecap + 2 + 3) & ~3) * 4 * max_batch) != hipSuccess) ||
      hipMalloc(&e.d_nanch, 4 * (size_t)max_batch) != hipSuccess ||
      hipMalloc(&e.d_nedge, 4 * (size_t)max_batch) != hipSuccess ||
      hipMalloc(&e.d_img, (size_t)width * height * 4 + 16) != hipSuccess ||  // + the staging kernel's 16 B rounding
      hipMalloc(&e.d_lines, sizeof(float) * 6 * 4096) != hipSuccess || hipMalloc(&e.d_nlines, 8) != hipSuccess ||
      hipHostMalloc((void**)&e.h_n, 2 * sizeof(int), 0) != hipSuccess) {
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
  const dim3 bg((W + LF_TW - 1) / LF_TW, (H + LF_TH - 1) / LF_TH, nframes);
  const long long fs = (long long)pitch * H;
  // inner tiles stage their rows with aligned 4-byte loads when the layout allows it
  const int vec = (pitch % 4 == 0 && fs % 4 == 0 && ((uintptr_t)d_img & 3) == 0) ? 1 : 0;
  if (channels == 1)
    hipLaunchKernelGGL(k_line_maps<1>, bg, dim3(256), 0, s, d_img, pitch, fs, W, H, e.MP, e.k[0], e.k[1], e.k[2], vec,
                       e.d_blur, e.d_dx, e.d_dy, e.d_code, e.d_moves, e.d_amask);
  else if (channels == 3)
    hipLaunchKernelGGL(k_line_maps<3>, bg, dim3(256), 0, s, d_img, pitch, fs, W, H, e.MP, e.k[0], e.k[1], e.k[2], vec,
                       e.d_blur, e.d_dx, e.d_dy, e.d_code, e.d_moves, e.d_amask);
  else
    hipLaunchKernelGGL(k_line_maps<4>, bg, dim3(256), 0, s, d_img, pitch, fs, W, H, e.MP, e.k[0], e.k[1], e.k[2], vec,
                       e.d_blur, e.d_dx, e.d_dy, e.d_code, e.d_moves, e.d_amask);
  // single frames: spec / merge / EDline in one launch (EAO_LINES_ONE_LAUNCH=0: the three kernels;
  // n: the workgroups beside the merge's)
  static const int fused_blocks = [] {
    const char* v = getenv("EAO_LINES_ONE_LAUNCH");
    return v ? atoi(v) : 64;  // workgroups beside the merge's; 0 = off
  }();
  const size_t lf_merge = edge_draw_lds(W, H, e.ecap, true) + 8 * LS_RING + 4 * (2 * (size_t)LF_STAGE + 2 * 64 * 5);
  const size_t lf_walk = (size_t)LF_WAVES * (sizeof(uint16_t) * LE_TW * LE_TH + 4 * LS_CAP);
  const size_t lf_lds = std::max(lf_merge, lf_walk);
  const bool fused = nframes == 1 && e.spec && fused_blocks > 0 && lf_lds <= kLdsMax - 64;
  if (fused && !e.d_lctl) {
    const size_t nw = (size_t)2 * e.acap;
    EAO_HIP_CHECK(hipMalloc(&e.d_lctl, sizeof(int) * LF_CTL));
    if (const char* v = getenv("EAO_LINES_PROF"))
      if (v[0] == '1') {
        EAO_HIP_CHECK(hipMalloc(&e.d_lprof, 16 * sizeof(unsigned long long)));
        EAO_HIP_CHECK(hipMemset(e.d_lprof, 0, 16 * sizeof(unsigned long long)));
      }
    EAO_HIP_CHECK(hipMalloc(&e.d_lstarts, (size_t)2 * ((e.ecap + 2 + 3) & ~3) * 4));
    if (!e.d_ps) {
      EAO_HIP_CHECK(hipMalloc(&e.d_ps, nw * LS_CAP * 4));
      EAO_HIP_CHECK(hipMalloc(&e.d_pl, nw * 4));
      EAO_HIP_CHECK(hipMalloc(&e.d_pe, nw * 4));
    }
  }
  hipLaunchKernelGGL(k_line_anchors, dim3(nframes), dim3(512), 0, s, e.d_amask, W, H, (int)bg.y, (int)bg.x * (LF_TW / 2),
                     e.d_anch, e.acap, e.d_nanch, fused ? e.d_pl : nullptr, fused ? e.d_lctl : nullptr);
  if (fused) {
    int* diag = lines_check() && d_counts == e.d_nlines ? e.d_nlines + 1 : nullptr;
    if (diag) EAO_HIP_CHECK(hipMemsetAsync(diag, 0, 4, s));
    // one workgroup of lf_lds per CU; progress needs only workgroup 0 (dispatched first) and one
    // other resident: walks and chains are claimed from counters, in order
    hipLaunchKernelGGL(k_lines_fused, dim3(1 + std::min(fused_blocks, 192)), dim3(64 * LF_WAVES), lf_lds, s, e.d_moves,
                       e.d_code, e.d_dx, e.d_dy, W, H, e.MP, e.d_anch, e.d_nanch, e.acap, e.d_ps, e.d_pl, e.d_pe, e.d_p1,
                       e.d_p2, e.pcap, e.d_chain, e.d_sid, e.ecap, e.d_nedge, e.d_lstarts, e.d_lctl, e.d_lscr, e.d_ccnt,
                       min_length, diag, e.d_lprof);
    hipLaunchKernelGGL(k_lines_place, dim3(1), dim3(256), 0, s, e.d_sid, e.d_nedge, e.pcap, e.ecap, e.d_lscr,
                       e.d_ccnt, d_lines, d_counts, cap);
  } else if (nframes == 1 && e.spec && edge_draw_lds(W, H, e.ecap, e.gstarts) + 8 * LS_RING <= kLdsMax - 64) {
    // the latency path: every anchor's two walks in parallel, the in-order merge on one wave, EDline
    // a wave per chain, the placement (k_walk_spec .. k_lines_place)
    if (!e.d_ps) {
      const size_t nw = (size_t)2 * e.acap;
      EAO_HIP_CHECK(hipMalloc(&e.d_ps, nw * LS_CAP * 4));
      EAO_HIP_CHECK(hipMalloc(&e.d_pl, nw * 4));
      EAO_HIP_CHECK(hipMalloc(&e.d_pe, nw * 4));
    }
    // development switches: EAO_LINES_DEBUG_SYNC=1 checks every kernel of this path on its own;
    // EAO_LINES_CHECK=1 range-checks the
    // merge's records and the chains (a diagnostic word beside the count, eao_lines_detect_color)
    static const bool dbg = [] { const char* v = getenv("EAO_LINES_DEBUG_SYNC"); return v && v[0] == '1'; }();
    int* diag = lines_check() && d_counts == e.d_nlines ? e.d_nlines + 1 : nullptr;
    if (diag) EAO_HIP_CHECK(hipMemsetAsync(diag, 0, 4, s));
    auto dsync = [&](const char* k) -> int {
      if (!dbg) return EAO_OK;
      const hipError_t r = hipStreamSynchronize(s);
      if (r != hipSuccess) {
        set_error(std::string(k) + ": " + hipGetErrorString(r));
        return EAO_E_HIP;
      }
      return EAO_OK;
    };
    hipLaunchKernelGGL(k_walk_spec, dim3(4096, 1), dim3(64), sizeof(uint16_t) * LE_TW * LE_TH + 4 * LS_CAP, s,
                       e.d_moves, e.d_code, W, H, e.MP, e.d_anch, e.d_nanch, e.acap, e.d_ps, e.d_pl, e.d_pe);
    if (int rc = dsync("k_walk_spec")) return rc;
    hipLaunchKernelGGL(k_walk_merge, dim3(1), dim3(128), edge_draw_lds(W, H, e.ecap, e.gstarts) + 8 * LS_RING, s,
                       e.d_moves, W, H,
                       e.MP, e.d_anch, e.d_nanch, e.acap, e.d_ps, e.d_pl, e.d_pe, e.d_p1, e.d_p2, e.pcap, e.d_chain,
                       e.d_sid, e.ecap, e.d_nedge, e.d_starts, diag);
    if (int rc = dsync("k_walk_merge")) return rc;
    hipLaunchKernelGGL(k_edlines_par, dim3(1024, 1), dim3(64), 0, s, e.d_code, e.d_dx, e.d_dy, W, H, e.d_chain,
                       e.d_sid, e.d_nedge, e.pcap, e.ecap, e.d_lscr, e.d_ccnt, min_length, diag);
    if (int rc = dsync("k_edlines_par")) return rc;
    hipLaunchKernelGGL(k_lines_place, dim3(1), dim3(256), 0, s, e.d_sid, e.d_nedge, e.pcap, e.ecap, e.d_lscr,
                       e.d_ccnt, d_lines, d_counts, cap);
    if (int rc = dsync("k_lines_place")) return rc;
  } else if (e.fused) {
    hipLaunchKernelGGL(k_edge_lines, dim3(nframes), dim3(64 * LE_WAVES), edge_draw_lds(W, H, e.ecap, e.gstarts), s,
                       e.d_moves, W, H, e.MP, e.d_anch, e.d_nanch, e.acap, e.d_p1, e.d_p2, e.pcap, e.d_chain, e.d_sid,
                       e.ecap, e.d_nedge, e.d_code, e.d_dx, e.d_dy, e.d_lscr, e.d_ccnt, min_length, d_lines, d_counts,
                       cap, e.d_starts);
  } else {
    hipLaunchKernelGGL(k_edge_draw, dim3(nframes), dim3(64), edge_draw_lds(W, H, e.ecap, e.gstarts), s, e.d_moves,
                       e.d_code, W, H, e.MP, e.d_anch, e.d_nanch, e.acap, e.d_p1, e.d_p2, e.pcap, e.d_chain, e.d_sid,
                       e.ecap, e.d_nedge, e.d_starts);
    hipLaunchKernelGGL(k_edlines, dim3(nframes), dim3(64 * LN_WAVES), 0, s, e.d_code, e.d_dx, e.d_dy, W, H,
                       e.d_chain, e.d_sid, e.d_nedge, e.pcap, e.ecap, e.d_lscr, e.d_ccnt, min_length, d_lines, d_counts,
                       cap);
  }
  EAO_HIP_CHECK(hipGetLastError());
  return EAO_OK;
}

int eao_lines_detect_batch_device(eao_lines* L, const uint8_t* d_gray, int nframes, int pitch, float min_length,
                                  float* d_lines, int32_t* d_counts, int cap, void* stream) {
  return eao_lines_detect_color_batch_device(L, d_gray, nframes, pitch, 1, min_length, d_lines, d_counts, cap, stream);
}

// single calls: the count (and the checking word) and min(count, cap) lines written by the GPU straight
// into the handle's pinned buffers, behind the kernels on the engine's stream. A DMA copy would queue on
// the copy engine behind this frame's 0.5 ms line launch, and with it every other engine's transfers
// of the same frame (the drop-in's matching waited there: profiles/r06_dropin_copy_engine.txt).
__global__ __launch_bounds__(256) void k_lines_out(const int* __restrict__ dn, const float* __restrict__ dl, int cap,
                                                   int nw, int* __restrict__ hn, float* __restrict__ hl) {
  const int n = dn[0];
  if (threadIdx.x < nw) hn[threadIdx.x] = dn[threadIdx.x];
  const int k = 6 * max(0, min(n, cap));
  for (int i = threadIdx.x; i < k; i += blockDim.x) hl[i] = dl[i];
}

__global__ __launch_bounds__(256) void k_lines_stage(const uint4* __restrict__ src, uint4* __restrict__ dst, int n16) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256) dst[i] = src[i];
}

int eao_lines_detect_color_start(eao_lines* L, const uint8_t* img, int pitch, int channels, float min_length,
                                 int cap) {
  if (!L || !img || cap < 0) return EAO_E_ARG;
  LineEngine& e = L->e;
  if ((channels != 1 && channels != 3 && channels != 4) || pitch < e.W * channels) return EAO_E_ARG;
  if (e.pending_cap >= 0) {
    set_error("eao_lines_detect_color_start: the previous frame's lines are not taken (eao_lines_detect_finish)");
    return EAO_E_STATE;
  }
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  hipStream_t s = e.stream;
  const int row = e.W * channels;
  // the frame through pinned staging (one DMA copy); the count and every line slot back into
  // pinned memory behind the kernels, one synchronisation
  EAO_HIP_CHECK(e.stage_in.reserve((size_t)row * e.H));
  if (pitch == row) {
    e.stage_in.put(img, (size_t)row * e.H);
  } else {
    const size_t o = e.stage_in.put(nullptr, (size_t)row * e.H);
    for (int y = 0; y < e.H; y++) std::memcpy(e.stage_in.h + o + (size_t)y * row, img + (size_t)y * pitch, row);
  }
  // the pinned frame into HBM by a copy kernel (16 B per lane over 120 workgroups, ~50 GB/s) by default:
  // a copy-engine transfer would queue behind the other engines' transfers of the frame, and the maps
  // kernel reading the frame in place over PCIe ran 58 us against 16 us from HBM (its tiles' loads are
  // latency-bound there). EAO_LINES_IN=dma: one DMA copy; =pcie: the maps kernel reads in place (A/B)
  static const int in_mode = [] {
    const char* v = getenv("EAO_LINES_IN");
    return !v ? 0 : v[0] == 'd' ? 1 : v[0] == 'p' ? 2 : 0;
  }();
  const uint8_t* src = e.d_img;
  if (in_mode == 1) {
    EAO_HIP_CHECK(hipMemcpyAsync(e.d_img, e.stage_in.h, (size_t)row * e.H, hipMemcpyHostToDevice, s));
  } else if (in_mode == 2) {
    src = e.stage_in.h;
  } else {
    const int n16 = (int)(((size_t)row * e.H + 15) >> 4);  // stage_in: 16-aligned with slack; d_img: + 16 B
    hipLaunchKernelGGL(k_lines_stage, dim3(std::min(240, (n16 + 255) / 256)), dim3(256), 0, s,
                       (const uint4*)e.stage_in.h, (uint4*)e.d_img, n16);
    EAO_HIP_CHECK(hipGetLastError());
  }
  int rc = eao_lines_detect_color_batch_device(L, src, 1, row, channels, min_length, e.d_lines, e.d_nlines, 4096, s);
  if (rc) return rc;
  const size_t lb = sizeof(float) * 6 * (size_t)std::min(std::max(cap, 0), 4096);
  EAO_HIP_CHECK(e.stage_out.reserve(lb));
  static const bool dma_out = [] {
    const char* v = getenv("EAO_LINES_DMA_OUT");  // 1: the DMA copies back (A/B)
    return v && v[0] == '1';
  }();
  if (dma_out) {
    EAO_HIP_CHECK(hipMemcpyAsync(e.h_n, e.d_nlines, lines_check() ? 8 : 4, hipMemcpyDeviceToHost, s));
    if (lb) EAO_HIP_CHECK(hipMemcpyAsync(e.stage_out.h, e.d_lines, lb, hipMemcpyDeviceToHost, s));
  } else {
    hipLaunchKernelGGL(k_lines_out, dim3(1), dim3(256), 0, s, e.d_nlines, e.d_lines,
                       std::min(std::max(cap, 0), 4096), lines_check() ? 2 : 1, e.h_n, (float*)e.stage_out.h);
    EAO_HIP_CHECK(hipGetLastError());
  }
  e.pending_cap = std::min(std::max(cap, 0), 4096);
  return EAO_OK;
}

int eao_lines_detect_finish(eao_lines* L, float* lines, int* n_out) {
  if (!L || !n_out) return EAO_E_ARG;
  LineEngine& e = L->e;
  if (e.pending_cap < 0) {
    set_error("eao_lines_detect_finish: no frame started (eao_lines_detect_color_start)");
    return EAO_E_STATE;
  }
  const int cap = e.pending_cap;
  e.pending_cap = -1;
  if (cap && !lines) return EAO_E_ARG;
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  EAO_HIP_CHECK(hipStreamSynchronize(e.stream));
  const int n = *e.h_n;
  if (lines_check() && e.h_n[1]) {
    set_error("eao_lines_detect: checking mode found out-of-range records or chains (diag 0x" +
              std::to_string(e.h_n[1]) + ": 1 merge record, 2 chain starts, 8 chain span, 16 chain pixel)");
    return EAO_E_HIP;
  }
  if (n < 0) {
    set_error("eao_lines_detect: edge arrays overflowed (the reference's EdgeDrawing -1)");
    return EAO_E_CAPACITY;
  }
  *n_out = n;
  const int k = n < cap ? n : cap;
  if (k > 0) std::memcpy(lines, e.stage_out.h, sizeof(float) * 6 * k);
  return n > cap ? EAO_E_CAPACITY : EAO_OK;
}

int eao_lines_detect_color(eao_lines* L, const uint8_t* img, int pitch, int channels, float min_length, float* lines,
                           int cap, int* n_out) {
  if (!L || !img || !n_out || cap < 0 || (cap && !lines)) return EAO_E_ARG;
  *n_out = 0;
  const int rc = eao_lines_detect_color_start(L, img, pitch, channels, min_length, cap);
  if (rc) return rc;
  return eao_lines_detect_finish(L, lines, n_out);
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
