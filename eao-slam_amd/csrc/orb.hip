// orb.hip -- ORB extraction on gfx950: the MI355X replacement of
// ORBextractor::operator() (reference src/ORBextractor.cc:1043-1105).
//
// Pipeline per batch of frames (all HBM-resident, one stream):
//   k_resize_tile x7  level l from level l-1 (cv::resize INTER_LINEAR 8U, fixed
//                     point, ORBextractor.cc:1120), one workgroup per band of 8 rows
//   k_fast_band   x1  one 4-wave workgroup per (band of cells <= 258 px, frame):
//                     band ROI staged in LDS, packed-f16 FAST strength swept
//                     down 62-column strips, in-cell 3x3 NMS by DPP, iniTh with
//                     minTh retry for empty cells (ORBextractor.cc:789-829)
//   k_distribute  x1  one wave per (level, frame): DistributeOctTree with
//                     the reference's list order (ORBextractor.cc:539-763)
//   k_describe    x1  one wave per selected keypoint: the raw 43x43 patch in LDS,
//                     IC_Angle on it, the 7x7 sigma-2 blur (REFLECT_101) fused --
//                     horizontal sums of the patch, vertical sums at the 512
//                     rBRIEF taps only -- 256-bit descriptor, final scaling
//                     (:77-147, :1076-1104; blur :1085-1086)
// Bit-exactness: integer paths are exact; float paths use __f*_rn intrinsics
// and -ffp-contract=off so every rounding matches the oracle.
#include <hip/hip_runtime.h>

#include <cstdint>

#include <cstdlib>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "common.h"
#include "orb.h"

namespace eao {


__constant__ int c_pattern[1024] = {
#include "orb_pattern.inc"
};

// ---------------------------------------------------------------- resize
// Row-band tiles: one workgroup makes RESIZE_TR whole output rows (a thread per column,
// stepping by 256 across the row). A thread walks its column down the band and keeps the
// last two source rows' horizontal sums in registers, so a source row is read once per
// band instead of once per output row that uses it (rows are shared ~1.67x at scale 1.2),
// whole rows keep the reads line-aligned, and the rows a band reads stay in one XCD's L2.
// Same fixed-point arithmetic as OpenCV's INTER_LINEAR 8U resize (tables on the host).
constexpr int RESIZE_TR = 8;
__global__ __launch_bounds__(256) void k_resize_tile(const uint8_t* __restrict__ src, int spitch,
                                                     long long sstride, uint8_t* __restrict__ dst,
                                                     int dpitch, long long dstride, int dw, int dh,
                                                     const int* __restrict__ xofs,
                                                     const short* __restrict__ ialpha, int xmax,
                                                     const int* __restrict__ yrows,
                                                     const short* __restrict__ ibeta) {
  const int dy0 = blockIdx.y * RESIZE_TR;
  const int f = blockIdx.z;
  const uint8_t* sf = src + f * sstride;
  uint8_t* df = dst + f * dstride;
  const int dy1 = min(dy0 + RESIZE_TR, dh);
  for (int dx = threadIdx.x; dx < dw; dx += blockDim.x) {
    const int sx = xofs[dx];
    const bool two = dx < xmax;
    const int a0 = two ? ialpha[2 * dx] : 2048, a1 = two ? ialpha[2 * dx + 1] : 0;
    auto hsum = [&](int r) {
      const uint8_t* q = sf + (long long)r * spitch + sx;
      return two ? q[0] * a0 + q[1] * a1 : q[0] * 2048;
    };
    int ra = -1, rb = -1, ha = 0, hb = 0;  // the last two source rows and their horizontal sums
    for (int dy = dy0; dy < dy1; dy++) {
      const int r0 = yrows[2 * dy], r1 = yrows[2 * dy + 1];
      int d0, d1;
      if (r0 == rb) d0 = hb; else if (r0 == ra) d0 = ha; else d0 = hsum(r0);
      if (r1 == rb) d1 = hb; else if (r1 == ra) d1 = ha; else d1 = hsum(r1);
      ra = r0; ha = d0;
      rb = r1; hb = d1;
      const int v = (d0 * ibeta[2 * dy] + d1 * ibeta[2 * dy + 1] + (1 << 21)) >> 22;
      df[(long long)dy * dpitch + dx] = (uint8_t)min(max(v, 0), 255);
    }
  }
}

// LDS-staged resize (the production path): one workgroup per (tile of tr output rows, frame).
//   1. the tile's source rows [ys0, ys1] are staged in LDS with 16-byte loads (row stride sw16 =
//      the source width rounded up to 16), all of them in flight;
//   2. a work item = (group of 4 output columns, segment of RESIZE_RS rows): the item keeps its
//      4 columns' x offsets and coefficients and its rows' source rows and coefficients in
//      registers, walks its rows keeping the last two source rows' horizontal sums (a source row
//      is summed once per item, not per output row), taps are LDS byte reads, and the 4 outputs go
//      out as one dword store (level planes are 64-byte pitched, so the store is aligned; columns
//      past dw repeat the last column's coefficients into the plane's pitch padding, which nothing
//      reads).
// Latency: the kernel is a chain of memory round trips per workgroup, so every load is issued up
// front -- ys0 / ys1 are recomputed from scale_y (the host's float expression, bit-identical) instead
// of read from the row table, and the first item's table entries are loaded together with the
// staging loads, before the barrier.
// Items are numbered column-group-fastest, so a wave's stores cover 256 contiguous bytes.
// Arithmetic identical to k_resize_tile (OpenCV INTER_LINEAR 8U, ORBextractor.cc:1120).
constexpr int RESIZE_RS = 4;
constexpr int RESIZE_IPT = 4;  // items per thread of a k_resize_lds tile (OrbEngine::plan)
__device__ __forceinline__ int resize_src_row(int dy, double scale_y, int sh, int k) {
  const float fy = (float)((dy + 0.5) * scale_y - 0.5);  // OrbEngine::plan's resize_yrows
  return min(max((int)floorf(fy) + k, 0), sh - 1);
}
// an item's table entries, packed: x offsets; coefficient pairs a0 | a1 << 16 (a1 = 0 past xmax)
// and b0 | b1 << 16 (all in [0, 2048]); source rows r0 | r1 << 16
struct ResizeItem {
  int sx[4], a[4], r[RESIZE_RS], b[RESIZE_RS];
};
__device__ __forceinline__ void resize_item_load(ResizeItem& I, int g, int e0, int e1, int dw, int xmax,
                                                 const int* __restrict__ xofs, const short* __restrict__ ialpha,
                                                 const int* __restrict__ yrows, const short* __restrict__ ibeta) {
#pragma unroll
  for (int u = 0; u < 4; u++) {
    const int dx = min(4 * g + u, dw - 1);
    I.sx[u] = xofs[dx];
    const int pa = *(const int*)(ialpha + 2 * dx);  // the (a0, a1) pair: 4-byte aligned
    I.a[u] = dx < xmax ? pa : 2048;
  }
#pragma unroll
  for (int k = 0; k < RESIZE_RS; k++) {
    const int dy = min(e0 + k, e1 - 1);
    const int2 yr = *(const int2*)(yrows + 2 * dy);
    I.r[k] = yr.x | (yr.y << 16);
    I.b[k] = *(const int*)(ibeta + 2 * dy);
  }
}
// the rows [e0, e1) of an item from a source image in LDS (row r at img + (r - ys0) * stride, one
// readable byte past every row): the last two source rows' horizontal sums kept; put(dy, w) takes
// the 4 output bytes of row dy. `one` is 1: a kernel argument where the compiler would otherwise
// merge a tap pair into one unaligned ds_read_u16 (k_pyr_tail: 2.5x slower)
template <class Put>
__device__ __forceinline__ void resize_item_rows(const ResizeItem& I, const unsigned char* img, int ys0, int stride,
                                                 int e0, int e1, int one, Put put) {
  auto hsum = [&](int r, int (&h)[4]) {
    const unsigned char* row = img + (r - ys0) * stride;
#pragma unroll
    for (int u = 0; u < 4; u++) h[u] = row[I.sx[u]] * (I.a[u] & 0xffff) + row[I.sx[u] + one] * (I.a[u] >> 16);
  };
  int ra = -1, rb = -1, ha[4], hb[4];
#pragma unroll
  for (int k = 0; k < RESIZE_RS; k++) {
    const int dy = e0 + k;
    if (dy >= e1) break;
    const int r0 = I.r[k] & 0xffff, r1 = I.r[k] >> 16;
    int d0[4], d1[4];
    if (r0 == rb) {
#pragma unroll
      for (int u = 0; u < 4; u++) d0[u] = hb[u];
    } else if (r0 == ra) {
#pragma unroll
      for (int u = 0; u < 4; u++) d0[u] = ha[u];
    } else {
      hsum(r0, d0);
    }
    if (r1 == rb) {
#pragma unroll
      for (int u = 0; u < 4; u++) d1[u] = hb[u];
    } else {
      hsum(r1, d1);
    }
    uint32_t w = 0;
#pragma unroll
    for (int u = 0; u < 4; u++) {
      // no saturation: 0 <= v <= 255 already (taps >= 0, a0 + a1 <= 2049, b0 + b1 <= 2049:
      // v <= (255 * 2049^2 + 2^21) >> 22 = 255), and the clamp made the compiler pack two
      // bytes with v_ashr_pk_u8_i32, whose result's upper half is not zero on gfx950: the
      // v_lshl_or of bytes 2 / 3 then OR'ed stale bits into them (round-5 miscompile)
      const uint32_t v = (uint32_t)(d0[u] * (I.b[k] & 0xffff) + d1[u] * (I.b[k] >> 16) + (1 << 21)) >> 22;
      w |= v << (8 * u);
      ha[u] = d0[u];
      hb[u] = d1[u];
    }
    ra = r0;
    rb = r1;
    put(dy, w);
  }
}

template <bool VEC>
__global__ __launch_bounds__(1024) void k_resize_lds(const uint8_t* __restrict__ src, int spitch, long long sstride,
                                                     uint8_t* __restrict__ dst, int dpitch, long long dstride,
                                                     int sw, int sh, int dw, int dh, int tr, double scale_y,
                                                     const int* __restrict__ xofs, const short* __restrict__ ialpha,
                                                     int xmax, const int* __restrict__ yrows,
                                                     const short* __restrict__ ibeta) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int dy0 = blockIdx.x * tr, f = blockIdx.y;
  const int dy1 = min(dy0 + tr, dh);
  const int ys0 = resize_src_row(dy0, scale_y, sh, 0), ys1 = resize_src_row(dy1 - 1, scale_y, sh, 1);
  const int nrows = ys1 - ys0 + 1;
  const int sw16 = (sw + 15) & ~15;
  const uint8_t* sf = src + f * sstride + (long long)ys0 * spitch;
  const int tid = threadIdx.x, nb = blockDim.x;
  const int G = (dw + 3) >> 2;
  const int nseg = (dy1 - dy0 + RESIZE_RS - 1) / RESIZE_RS;
  const int nit = G * nseg;
  ResizeItem I;
  auto seg_rows = [&](int it, int& g, int& e0, int& e1) {
    const int seg = it / G;
    g = it - seg * G;
    e0 = dy0 + seg * RESIZE_RS;
    e1 = min(e0 + RESIZE_RS, dy1);
  };
  int g = 0, e0 = 0, e1 = 0;
  if (tid < nit) {  // the first item's tables: in flight with the staging loads
    seg_rows(tid, g, e0, e1);
    resize_item_load(I, g, e0, e1, dw, xmax, xofs, ialpha, yrows, ibeta);
  }
  if (VEC) {
    const int cpr = sw16 >> 4, nc = nrows * cpr;
    int c = tid;
    for (; c + 3 * nb < nc; c += 4 * nb) {
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int cc = c + u * nb, r = cc / cpr, k = cc - r * cpr;
        v[u] = *(const uint4*)(sf + (long long)r * spitch + 16 * k);
      }
#pragma unroll
      for (int u = 0; u < 4; u++) ((uint4*)smem)[c + u * nb] = v[u];
    }
    if (c < nc) {  // the rest: at most three loads per thread, all in flight
      uint4 v[3];
#pragma unroll
      for (int u = 0; u < 3; u++) {
        const int cc = c + u * nb, r = cc / cpr, k = cc - r * cpr;
        v[u] = *(const uint4*)(sf + (long long)(cc < nc ? r : 0) * spitch + 16 * (cc < nc ? k : 0));
      }
#pragma unroll
      for (int u = 0; u < 3; u++)
        if (c + u * nb < nc) ((uint4*)smem)[c + u * nb] = v[u];
    }
  } else {
    for (int c = tid; c < nrows * sw16; c += nb) {
      const int r = c / sw16, k = c - r * sw16;
      smem[c] = k < sw ? sf[(long long)r * spitch + k] : 0;
    }
  }
  __syncthreads();
  uint8_t* df = dst + f * dstride;
  for (int it = tid; it < nit; it += nb) {
    if (it != tid) {
      seg_rows(it, g, e0, e1);
      resize_item_load(I, g, e0, e1, dw, xmax, xofs, ialpha, yrows, ibeta);
    }
    resize_item_rows(I, smem, ys0, sw16, e0, e1, 1,
                     [&](int dy, uint32_t w) { *(uint32_t*)(df + (long long)dy * dpitch + 4 * g) = w; });
  }
}

// The pyramid's small levels in one launch (OrbEngine::plan's tail_a): one workgroup per frame
// makes levels [a, nl) from level a - 1, whose plane is staged in LDS; each level is computed
// from the previous level's LDS image (items of 4 columns x RESIZE_RS rows, column-group fastest,
// as k_resize_lds) and stored to its plane and, for the next level, into the other LDS image
// (images ping-pong between offsets 0 and img_b; one readable byte past each). The levels' resize
// tables (contiguous from level a: nx column and ny row entries) are staged in LDS at tab_b with the
// source image. Launched per level, these levels were latency: 62 us of the 640x480 pyramid's
// 0.30 ms for 15 % of its bytes.
__global__ __launch_bounds__(1024) void k_pyr_tail(uint8_t* __restrict__ pyr, long long pstride,
                                                   const LevelDev* __restrict__ lv, int a, int nl, int img_b,
                                                   int tab_b, int nx, int ny, int one, const int* __restrict__ xofs,
                                                   const short* __restrict__ ialpha, const int* __restrict__ yrows,
                                                   const short* __restrict__ ibeta) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, nb = blockDim.x;
  uint8_t* pf = pyr + (long long)blockIdx.x * pstride;
  const int tx0 = lv[a].tab_x, ty0 = lv[a].tab_y;
  int* sX = (int*)(smem + tab_b);
  int* sIA = sX + nx;  // (a0, a1) pairs
  int2* sY = (int2*)(sIA + nx);
  int* sIB = (int*)(sY + ny);  // (b0, b1) pairs
  // a workgroup's time is its chain of memory round trips: every staging load (tables and image,
  // up to 8 16-byte chunks per thread) is issued before the first LDS store
  int cs = 0;  // the current image's row stride
  {
    const LevelDev S = lv[a - 1];
    cs = (S.w + 15) & ~15;
    const int cpr = cs >> 4, nc = S.h * cpr;
    const uint8_t* sp = pf + S.plane_off;
    const bool hx = tid < nx, hy = tid < ny;
    const int tX = hx ? xofs[tx0 + tid] : 0, tA = hx ? *(const int*)(ialpha + 2 * (tx0 + tid)) : 0;
    const int2 tY = hy ? *(const int2*)(yrows + 2 * (ty0 + tid)) : make_int2(0, 0);
    const int tB = hy ? *(const int*)(ibeta + 2 * (ty0 + tid)) : 0;
    for (int c = tid; c < nc; c += 8 * nb) {
      uint4 v[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int cc = min(c + u * nb, nc - 1), r = cc / cpr, k = cc - r * cpr;
        v[u] = *(const uint4*)(sp + (long long)r * S.pitch + 16 * k);
      }
#pragma unroll
      for (int u = 0; u < 8; u++)
        if (c + u * nb < nc) ((uint4*)smem)[c + u * nb] = v[u];
    }
    if (hx) {
      sX[tid] = tX;
      sIA[tid] = tA;
    }
    if (hy) {
      sY[tid] = tY;
      sIB[tid] = tB;
    }
    for (int i = nb + tid; i < nx; i += nb) {  // (levels wider than a workgroup)
      sX[i] = xofs[tx0 + i];
      sIA[i] = *(const int*)(ialpha + 2 * (tx0 + i));
    }
    for (int i = nb + tid; i < ny; i += nb) {
      sY[i] = *(const int2*)(yrows + 2 * (ty0 + i));
      sIB[i] = *(const int*)(ibeta + 2 * (ty0 + i));
    }
  }
  __syncthreads();
  unsigned char* cur = smem;
  unsigned char* nxt = smem + img_b;
  for (int l = a; l < nl; l++) {
    const LevelDev L = lv[l];
    const int ds = (L.w + 15) & ~15;
    const int G = (L.w + 3) >> 2, nit = G * ((L.h + RESIZE_RS - 1) / RESIZE_RS);
    uint8_t* dp = pf + L.plane_off;
    const bool keep = l + 1 < nl;
    for (int it = tid; it < nit; it += nb) {
      const int seg = it / G, g = it - seg * G;
      const int e0 = seg * RESIZE_RS, e1 = min(e0 + RESIZE_RS, L.h);
      ResizeItem I;
      resize_item_load(I, g, e0, e1, L.w, L.xmax, sX + (L.tab_x - tx0), (const short*)(sIA + (L.tab_x - tx0)),
                       (const int*)(sY + (L.tab_y - ty0)), (const short*)(sIB + (L.tab_y - ty0)));
      resize_item_rows(I, cur, 0, cs, e0, e1, one, [&](int dy, uint32_t w) {
        *(uint32_t*)(dp + (long long)dy * L.pitch + 4 * g) = w;
        if (keep) *(uint32_t*)(nxt + dy * ds + 4 * g) = w;
      });
    }
    __syncthreads();
    unsigned char* t = cur;
    cur = nxt;
    nxt = t;
    cs = ds;
  }
}

// ---------------------------------------------------------------- FAST
// FAST corner strength of a pixel (cv::FAST-9/16 + cornerScore<16>, ORBextractor.cc:809-815):
// with A = min over the 16 arcs of 9 ring pixels of the arc's max and B = max over the arcs
// of the arc's min, S = max(0, v - A, B - v). The pixel is a FAST-9 corner at threshold th
// iff S > th, and cornerScore<16> at that threshold is then S - 1 (its a0 starts at th < S),
// so one strength map serves both the iniTh pass and the minTh retry.

// gfx950 packed 3-input f16 minimum / maximum (two pixels per instruction)
__device__ __forceinline__ uint32_t pk_min3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_pk_minimum3_f16 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
__device__ __forceinline__ uint32_t pk_max3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_pk_maximum3_f16 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

// The FAST strength (above) for the two vertically adjacent pixels p (low half) and
// p + RS (high half) at once. A ring byte b is carried as the 16-bit pattern 0x00bb, an f16
// subnormal: the kernels run with f16 denormals preserved (float_denorm_mode_16_64 = 3) and
// subnormals order as their integer patterns, so f16 minimum / maximum order the bytes exactly
// and the 3- then 9-wide arc windows run on both rows per instruction (one v_lshl_or per ring
// pair; an exponent bias would cost a second op). The arc bounds A, B come out as the byte
// values, so S = max(0, v - A, B - v) is taken on their low bytes as integers.
// Returns S(row) | S(row + 1) << 16.
template <int RS>
__device__ __forceinline__ uint32_t fast_strength_pair(const uint8_t* p) {
  constexpr int off[16] = {3 * RS,  3 * RS + 1,  2 * RS + 2,  RS + 3,  3,  -RS + 3,  -2 * RS + 2,  -3 * RS + 1,
                           -3 * RS, -3 * RS - 1, -2 * RS - 2, -RS - 3, -3, RS - 3,   2 * RS - 2,  3 * RS - 1};
  uint32_t q[16];
#pragma unroll
  for (int k = 0; k < 16; k++) q[k] = (uint32_t)p[off[k]] | ((uint32_t)p[off[k] + RS] << 16);
  uint32_t mn3[16], mx3[16];
#pragma unroll
  for (int k = 0; k < 16; k++) {
    mn3[k] = pk_min3(q[k], q[(k + 1) & 15], q[(k + 2) & 15]);
    mx3[k] = pk_max3(q[k], q[(k + 1) & 15], q[(k + 2) & 15]);
  }
  uint32_t A = 0x00ff00ffu, B = 0u;  // 255, 0
#pragma unroll
  for (int k = 0; k < 16; k += 2) {
    const uint32_t a0 = pk_max3(mx3[k], mx3[(k + 3) & 15], mx3[(k + 6) & 15]);
    const uint32_t a1 = pk_max3(mx3[k + 1], mx3[(k + 4) & 15], mx3[(k + 7) & 15]);
    const uint32_t b0 = pk_min3(mn3[k], mn3[(k + 3) & 15], mn3[(k + 6) & 15]);
    const uint32_t b1 = pk_min3(mn3[k + 1], mn3[(k + 4) & 15], mn3[(k + 7) & 15]);
    A = pk_min3(A, a0, a1);
    B = pk_max3(B, b0, b1);
  }
  const int v0 = p[0], v1 = p[RS];
  const int s0 = max(0, max(v0 - (int)(A & 0xff), (int)(B & 0xff) - v0));
  const int s1 = max(0, max(v1 - (int)((A >> 16) & 0xff), (int)((B >> 16) & 0xff) - v1));
  return (uint32_t)s0 | ((uint32_t)s1 << 16);
}

// ROI row strides of k_fast_band: a band is at most RS - 30 px wide (16-byte alignment
// slack of the staging loads). Rows of cells are split into bands of balanced width
// <= FAST_BAND_W, so the narrow stride serves 640x480 and 1920x1080 alike; its smaller
// LDS block (RS * (2 bh - 6) bytes) lifts the resident waves per CU.
constexpr int FAST_RS_NARROW = 288;
constexpr int FAST_RS = 544;
constexpr int FAST_BAND_W = FAST_RS_NARROW - 30;

// lane l <- lane l-1 (right = false) or l+1 (right = true) across the whole
// wave (GFX9 DPP wave_shr:1 / wave_shl:1); the missing end lane reads 0
__device__ __forceinline__ int wave_from_left(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, true); }
__device__ __forceinline__ int wave_from_right(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x130, 0xF, 0xF, true); }

// One workgroup per (row of cells, frame), ORBextractor.cc:789-829 per cell:
// FAST-9 at iniTh with in-cell 3x3 non-max suppression (neighbours outside the
// cell's detection window count as 0, Q15), retry at minTh only when the cell
// found nothing; corners emitted row-major per cell.
//   1. the band ROI is staged in LDS with 16-byte loads;
//   2. each wave sweeps 64-column strips down the band (62 output columns, the
//      two end lanes are halo): a lane computes the FAST strength S of its
//      column row by row, keeps three rows in registers and gets the left /
//      right neighbours by DPP wave shifts, so the suppression costs a few
//      VALU ops instead of nine LDS reads. keep(t) <=> S > t, S >= 2 and S
//      beats the largest in-window neighbour whenever that one exceeds t;
//      keep(iniTh) == keep(minTh) && S > iniTh, so one byte per pixel
//      (S if kept at minTh, else 0) encodes both passes;
//   3. one wave per cell emits the kept pixels row-major (ballot + popcount),
//      the iniTh set, or the minTh set when the cell has no iniTh corner.
template <int RS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6, 8))) void k_fast_band(const uint8_t* __restrict__ frames, int fpitch,
                                                   long long fstride, const uint8_t* __restrict__ pyr,
                                                   long long pstride, const LevelDev* __restrict__ levels,
                                                   const BandDev* __restrict__ bands,
                                                   const CellDev* __restrict__ cells, int iniTh, int minTh,
                                                   uint32_t* __restrict__ cand, long long cand_stride,
                                                   int* __restrict__ cell_cnt, int ncells, int vec_ok,
                                                   int xcd_order) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ int16_t bnd[64];  // cell detection-window starts (band coords), then the end
  // xcd_order: the (band, frame) work in a bijective XCD-aware order -- workgroups are dealt
  // to the 8 XCDs round-robin, so XCD x takes a contiguous eighth of the bands of consecutive
  // frames and the halo rows two vertically adjacent bands share are read through one L2
  int bi = blockIdx.x, f = blockIdx.y;
  if (xcd_order) {
    const int n = gridDim.x * gridDim.y, P = blockIdx.y * gridDim.x + blockIdx.x;
    const int x = P & 7, q = n >> 3, r = n & 7;
    const int lg = x * q + min(x, r) + (P >> 3);
    bi = lg % gridDim.x;
    f = lg / gridDim.x;
  }
  const BandDev B = bands[bi];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const LevelDev& L = levels[B.level];
  const uint8_t* img;
  int pitch;
  if (B.level == 0) {
    img = frames + f * fstride;
    pitch = fpitch;
  } else {
    img = pyr + f * pstride + L.plane_off;
    pitch = L.pitch;
  }
  const int bw = B.x1 - B.x0, bh = B.y1 - B.y0;
  // ROI column c lives at smem[r * RS + sh + c] (16-byte aligned row starts)
  const int ax0 = vec_ok ? (B.x0 & ~15) : B.x0, sh = B.x0 - ax0;
  uint8_t* roi = smem + sh;
  // kept strengths of the detection rows / columns [3, bh - 3) x [3, bw - 3) only,
  // addressed F[r * RS + x] (so the block needs RS * (2 bh - 6) bytes of LDS)
  uint8_t* F = smem + RS * bh - (3 * RS + 3);
  if (vec_ok) {
    const int nvec = (sh + bw + 15) >> 4;
    for (int idx = t; idx < bh * nvec; idx += 256) {
      const int r = idx / nvec, v = idx - r * nvec;
      *(uint4*)(smem + r * RS + 16 * v) = *(const uint4*)(img + (long long)(B.y0 + r) * pitch + ax0 + 16 * v);
    }
  } else {
    for (int r = t >> 6; r < bh; r += 4)
      for (int c = lane; c < bw; c += 64) roi[r * RS + c] = img[(long long)(B.y0 + r) * pitch + B.x0 + c];
  }
  for (int k = t; k <= B.ncells; k += 256) {
    const CellDev c = cells[B.cell_begin + min(k, B.ncells - 1)];
    bnd[k] = (int16_t)(k < B.ncells ? c.x0 + 3 - B.x0 : c.x1 - 3 - B.x0);
  }
  __syncthreads();
  const int thi = min(max(iniTh, 0), 255), tlo = min(max(minTh, 0), 255);
  const int y0 = 3, y1 = bh - 3;  // detection rows (every cell of the band)
  for (int k = wv; 3 + 62 * k < bw - 3; k += 4) {
    const int x = 2 + 62 * k + lane;  // lane 0 / 63: halo columns
    const bool inx = x >= 3 && x < bw - 3;
    const bool outl = inx && lane >= 1 && lane <= 62;
    int lo = 0, hi = 0;  // the detection window of x's cell
    if (inx) {
      int q = 0;
      while (q + 1 < B.ncells && bnd[q + 1] <= x) q++;
      lo = bnd[q];
      hi = bnd[q + 1];
    }
    const bool okl = x - 1 >= lo, okr = x + 1 < hi;
    // strengths of rows a and a + 1 of this column (one packed evaluation),
    // thresholded at minTh (rows >= y1 read as 0), with the in-window left /
    // right neighbours. Row a + 1 = y1 reads one ROI row past the band, which
    // is still inside the LDS allocation (the F area) and is masked.
    auto strengths = [&](int a, bool two, uint32_t& spa, uint32_t& spb) {
      spa = spb = 0;
      if (!(inx && a < y1)) return;
      spa = fast_strength_pair<RS>(roi + a * RS + x);
      if (two) spb = fast_strength_pair<RS>(roi + (a + 2) * RS + x);
    };
    auto pair_from = [&](uint32_t sp, int a, int (&Sv)[2], int (&Lv)[2], int (&Rv)[2]) {
      int s0 = (int)(sp & 0xffffu), s1 = (int)(sp >> 16);
      s0 = s0 > tlo ? s0 : 0;
      s1 = (s1 > tlo && a + 1 < y1) ? s1 : 0;
      const int l0 = wave_from_left(s0), r0 = wave_from_right(s0);
      const int l1 = wave_from_left(s1), r1 = wave_from_right(s1);
      Sv[0] = s0;
      Sv[1] = s1;
      Lv[0] = okl ? l0 : 0;
      Lv[1] = okl ? l1 : 0;
      Rv[0] = okr ? r0 : 0;
      Rv[1] = okr ? r1 : 0;
    };
    int Sc = 0, Lc = 0, Rc = 0;
    int mp = 0;  // neighbour-row max of row r-1 (row y0-1 is outside every window)
    // finalise row r (held in Sc/Lc/Rc) once row r + 1 is known
    auto fin = [&](int r, int Sn, int Ln, int Rn) {
      const int mn = max(max(Ln, Sn), Rn);
      const int M = max(max(mp, mn), max(Lc, Rc));
      const bool keep = Sc > tlo && Sc >= 2 && (M <= tlo || Sc > M);
      if (outl) F[r * RS + x] = (uint8_t)(keep ? Sc : 0);
      mp = max(max(Lc, Sc), Rc);
      Sc = Sn;
      Lc = Ln;
      Rc = Rn;
    };
    if (y0 < y1) {
      int S2[2], L2[2], R2[2];
      uint32_t sa, sb;
      strengths(y0, false, sa, sb);
      pair_from(sa, y0, S2, L2, R2);
      Sc = S2[0];
      Lc = L2[0];
      Rc = R2[0];
      fin(y0, S2[1], L2[1], R2[1]);
      // two row pairs per trip: their strength evaluations are independent, so the
      // LDS reads and VALU chains of one hide the latencies of the other
      for (int a = y0 + 2; a <= y1; a += 4) {
        int S4[2], L4[2], R4[2];
        strengths(a, a + 2 < y1, sa, sb);
        pair_from(sa, a, S2, L2, R2);
        pair_from(sb, a + 2, S4, L4, R4);
        fin(a - 1, S2[0], L2[0], R2[0]);
        if (a < y1) fin(a, S2[1], L2[1], R2[1]);
        if (a + 2 <= y1) {
          fin(a + 1, S4[0], L4[0], R4[0]);
          if (a + 2 < y1) fin(a + 2, S4[1], L4[1], R4[1]);
        }
      }
    }
  }
  __syncthreads();
#ifdef EAO_FAST_ABL_EMIT
  return;
#endif
  // ---- emission, one wave per cell, one lane per detection row: the lane counts
  // its row's kept pixels (F > iniTh, F > 0), the cell takes the iniTh set or -- when
  // that is empty -- the minTh set (ORBextractor.cc:812), an exclusive wave scan of the
  // row counts places every row, and each lane writes its row's corners in column
  // order: the cell's candidates come out row-major as cv::FAST emits them
  const int nr = y1 - y0;  // <= 64 (host checks)
  for (int cc = wv; cc < B.ncells; cc += 4) {
    const int ci = B.cell_begin + cc;
    const CellDev c = cells[ci];
    const int wx0 = bnd[cc], ww = bnd[cc + 1] - wx0;
    uint32_t* out = cand + f * cand_stride + c.slot;
    const int r = y0 + lane;
    const uint8_t* row = F + r * RS + wx0;
    int ci_ = 0, cm = 0;
    if (lane < nr)
      for (int x = 0; x < ww; x++) {
        const int v = row[x];
        ci_ += v > thi ? 1 : 0;
        cm += v > 0 ? 1 : 0;
      }
    const bool use_ini = wave_sum(ci_) > 0;
    const int th = use_ini ? thi : 0;
    const int cnt = use_ini ? ci_ : cm;
    int pre = cnt;  // inclusive scan over the lanes (rows)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(pre, o, 64);
      if (lane >= o) pre += u;
    }
    const int n = __shfl(pre, 63, 64);
    int k = pre - cnt;
    if (lane < nr && cnt > 0)
      for (int x = 0; x < ww; x++) {
        const int v = row[x];
        if (v > th) {
          // FAST coordinates are relative to the cell ROI (ORBextractor.cc:821-826)
          if (k < c.cap) out[k] = pack_kp(x + 3 + c.j * L.wCell, r + c.i * L.hCell, v - 1);
          k++;
        }
      }
    if (lane == 0) cell_cnt[f * ncells + ci] = n;
  }
}

// ---------------------------------------------------------------- frame input
// cvtColor(..., CV_{RGB,BGR}[A]2GRAY) on 8-bit data (src/Tracking.cc:349-362), the
// OpenCV 3.2 scalar RGB2Gray<uchar>: gray = (s0*c0 + s1*G2Y + s2*c2 + 2^13) >> 14
// with (c0, c2) = (R2Y, B2Y) for the RGB codes and (B2Y, R2Y) for the BGR codes
// (R2Y 4899, G2Y 9617, B2Y 1868). TUM3's Camera.RGB: 1 applies the RGB code to
// imread's BGR bytes. One thread per 16 output pixels of a frame
// (rows flattened): 16-byte stores, 16-byte loads when the rows allow it; HBM-bound.
__global__ __launch_bounds__(256) void k_gray(const uint8_t* __restrict__ src, int w, int h, int spitch,
                                              long long sstride, int cn, int c0, int c2,
                                              uint8_t* __restrict__ dst, int dpitch, long long dstride,
                                              int vec_ok) {
  constexpr int G2Y = 9617, HALF = 1 << 13;
  const int f = blockIdx.y, t = threadIdx.x;
  const uint8_t* S = src + f * sstride;
  uint8_t* D = dst + f * dstride;
  if (vec_ok && w % 16 == 0 && spitch == w * cn && dpitch == w) {
    // dense frame: the block's 256 x 16 pixels are one contiguous run of
    // 256 * 16 * cn source bytes -- staged through LDS with coalesced 16-byte
    // loads, converted, stored as 16-byte words
    __shared__ uint4 stage[256 * 4];
    const long long px0 = (long long)blockIdx.x * 4096, npx = (long long)w * h;
    const int nv = cn * 256;  // 16-byte words of the run
    const uint4* sv = (const uint4*)(S + px0 * cn);
    const long long words_left = (npx - px0) * cn / 16;
    for (int k = t; k < nv; k += 256)
      if (k < words_left) stage[k] = sv[k];
    __syncthreads();
    if (px0 + 16 * t >= npx) return;
    const uint32_t* in = (const uint32_t*)stage + t * 4 * cn;
    auto byte = [&](int i) -> int { return (int)((in[i >> 2] >> (8 * (i & 3))) & 0xffu); };
    uint32_t out[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const int b = i * cn;
      const int g = (byte(b) * c0 + byte(b + 1) * G2Y + byte(b + 2) * c2 + HALF) >> 14;
      out[i >> 2] |= (uint32_t)g << (8 * (i & 3));
    }
    *(uint4*)(D + px0 + 16 * t) = make_uint4(out[0], out[1], out[2], out[3]);
    return;
  }
  // general pitches / ragged widths: 16 pixels of one row per thread
  const int chunks = (w + 15) >> 4;
  const int idx = blockIdx.x * blockDim.x + t;
  if (idx >= chunks * h) return;
  const int y = idx / chunks, x0 = 16 * (idx - y * chunks);
  const uint8_t* s = S + (long long)y * spitch + (long long)x0 * cn;
  uint8_t* d = D + (long long)y * dpitch + x0;
  for (int i = 0; i < 16 && x0 + i < w; i++) {
    const uint8_t* q = s + i * cn;
    d[i] = (uint8_t)((q[0] * c0 + q[1] * G2Y + q[2] * c2 + HALF) >> 14);
  }
}

int color_to_gray(const uint8_t* d_src, int nframes, int w, int h, int spitch, int cn, int rgb, uint8_t* d_dst,
                  int dpitch, hipStream_t s) {
  if (nframes < 1 || w < 1 || h < 1 || (cn != 3 && cn != 4) || spitch < w * cn || dpitch < w) {
    set_error("eao_color_to_gray_batch_device: bad arguments");
    return EAO_E_ARG;
  }
  constexpr int R2Y = 4899, B2Y = 1868;
  const int c0 = rgb ? R2Y : B2Y, c2 = rgb ? B2Y : R2Y;
  const int vec_ok = ((uintptr_t)d_src % 16 == 0 && spitch % 16 == 0 && (uintptr_t)d_dst % 16 == 0 &&
                      dpitch % 16 == 0) ? 1 : 0;
  const int chunks = (w + 15) / 16;
  dim3 g((unsigned)(((long long)chunks * h + 255) / 256), nframes);  // 4096 px per block (dense path)
  hipLaunchKernelGGL(k_gray, g, dim3(256), 0, s, d_src, w, h, spitch, (long long)spitch * h, cn, c0, c2, d_dst,
                     dpitch, (long long)dpitch * h, vec_ok);
  EAO_HIP_CHECK(hipGetLastError());
  return EAO_OK;
}

// ---------------------------------------------------------------- quadtree
// One wave per (level, frame). Node list order is kept explicitly in an
// ordered slot array with push-front semantics; ties in the final-phase sort
// are broken by node creation id.
struct QNode {
  int16_t x0, y0, x1, y1;
  int beg, cnt;
  int id;
  int pos;
  uint8_t buf, nomore, alive, pad;
};

// QCAP: nodes alive at once (N + 4*nIni + margin), chosen per extractor from
// {256, 512, 1024} so the LDS footprint -- and with it the number of
// concurrently resident (level, frame) quadtrees -- follows the feature quota
constexpr int QCAP_MAX = 1024;

template <int QCAP>
struct QShared {
  static constexpr int QOS = 5 * QCAP;  // order array (one pass pushes <= 4*QCAP)
  QNode node[QCAP];
  int16_t order[QOS];
  int16_t freel[QCAP];
  int16_t vcur[QCAP];
  int16_t vprev[QCAP];
  unsigned long long skey[QCAP];
};

__device__ __forceinline__ int child_of(uint32_t k, int mx, int my) {
  const int x = kp_x(k), y = kp_y(k);
  return x < mx ? (y < my ? 0 : 2) : (y < my ? 1 : 3);
}

// the quadtree of one (level, frame) over n keys already in B0, ping-ponging with B1: global
// memory (LK false) or the workgroup's dynamic LDS (LK true, single frames: every divide's key
// reads and partition writes are then LDS round trips instead of L2 ones -- the walk is a chain
// of ~140 dependent divides at level 0)
template <int QCAP, bool LK>
__device__ __forceinline__ void dist_tree(QShared<QCAP>& S, uint32_t* B0, uint32_t* B1, int n, const LevelDev& L,
                                          uint32_t* __restrict__ S_out, int* __restrict__ sel_cnt_out, int lane) {
  constexpr int QOS = QShared<QCAP>::QOS;
  // a select, not an array: the pointers keep their address space (ds_* on the LDS path)
  auto bufs = [&](int b) -> uint32_t* { return b ? B1 : B0; };
  const int N = L.nfeat;
  // ---- free list
  for (int i = lane; i < QCAP; i += 64) {
    S.freel[i] = (int16_t)(QCAP - 1 - i);
    S.node[i].alive = 0;
  }
  __syncthreads();
  int nfree = QCAP;
  int next_id = 0;
  int alive = 0;
  int head = QOS;  // list occupies order[head .. QOS)
  bool overflow = false;

  auto alloc = [&]() -> int {
    if (nfree == 0) {
      overflow = true;
      return -1;
    }
    return S.freel[--nfree];
  };

  // ---- initial nodes (ORBextractor.cc:543-585)
  const int nIni = L.nIni;
  const float hX = L.hX;
  {
    // stable partition of keys by initial node, B0 -> B1
    int base = 0;
    int slots[16];
    for (int i = 0; i < nIni && i < 16; i++) {
      int cnt = 0;
      for (int c0 = 0; c0 < n; c0 += 64) {
        const int idx = c0 + lane;
        bool in = false;
        if (idx < n) in = (int)((float)kp_x(B0[idx]) / hX) == i;
        const uint64_t m = ballot(in);
        if (in) B1[base + cnt + popc64(m & lanes_below())] = B0[idx];
        cnt += popc64(m);
      }
      const int id = next_id++;
      slots[i] = -1;
      if (cnt > 0) {
        const int s = alloc();
        slots[i] = s;
        if (lane == 0 && s >= 0) {
          QNode& q = S.node[s];
          q.x0 = (int16_t)(int)(hX * (float)i);
          q.x1 = (int16_t)(int)(hX * (float)(i + 1));
          q.y0 = 0;
          q.y1 = (int16_t)(L.maxBY - L.minBY);
          q.beg = base;
          q.cnt = cnt;
          q.id = id;
          q.buf = 1;
          q.nomore = cnt == 1;
          q.alive = 1;
        }
        alive++;
      }
      base += cnt;
    }
    // push_back order: list = [ini0, ini1, ...] at the tail of order[]
    head = QOS - alive;
    int p = head;
    for (int i = 0; i < nIni && i < 16; i++)
      if (slots[i] >= 0) {
        if (lane == 0) {
          S.order[p] = (int16_t)slots[i];
          S.node[slots[i]].pos = p;
        }
        p++;
      }
    __syncthreads();
  }

  int nvcur = 0;
  int nToExpand = 0;

  // divide node s: partition its keys into the other buffer, push children
  // to the front (n1..n4), record children with >1 keys in vcur.
  auto divide = [&](int s) {
    const QNode q = S.node[s];
    const int hx = (int)ceilf((float)(q.x1 - q.x0) / 2);
    const int hy = (int)ceilf((float)(q.y1 - q.y0) / 2);
    const int mx = q.x0 + hx, my = q.y0 + hy;
    const uint32_t* src = bufs(q.buf) + q.beg;
    uint32_t* dst = bufs(q.buf ^ 1) + q.beg;
    // keys are read in groups of RK * 64 with all RK loads in flight
    // together; a node of <= RK * 64 keys keeps them in registers for the
    // scatter pass, larger nodes read each group again
    constexpr int RK = 8;
    uint32_t kr[RK];
    int chr[RK];
    auto load = [&](int base) {
#pragma unroll
      for (int j = 0; j < RK; j++) {
        const int idx = base + 64 * j + lane;
        kr[j] = idx < q.cnt ? src[idx] : 0u;
      }
#pragma unroll
      for (int j = 0; j < RK; j++) chr[j] = base + 64 * j + lane < q.cnt ? child_of(kr[j], mx, my) : 4;
    };
    int cnt4[4] = {0, 0, 0, 0};
    for (int base = 0; base < q.cnt; base += 64 * RK) {
      load(base);
#pragma unroll
      for (int j = 0; j < RK; j++)
        if (base + 64 * j < q.cnt) {
#pragma unroll
          for (int c = 0; c < 4; c++) cnt4[c] += popc64(ballot(chr[j] == c));
        }
    }
    int off4[4] = {0, cnt4[0], cnt4[0] + cnt4[1], cnt4[0] + cnt4[1] + cnt4[2]};
    int run4[4] = {0, 0, 0, 0};
    for (int base = 0; base < q.cnt; base += 64 * RK) {
      if (q.cnt > 64 * RK) load(base);
#pragma unroll
      for (int j = 0; j < RK; j++)
        if (base + 64 * j < q.cnt) {
#pragma unroll
          for (int c = 0; c < 4; c++) {
            const uint64_t m = ballot(chr[j] == c);
            if (chr[j] == c) dst[off4[c] + run4[c] + popc64(m & lanes_below())] = kr[j];
            run4[c] += popc64(m);
          }
        }
    }
    const int16_t rx0[4] = {q.x0, (int16_t)mx, q.x0, (int16_t)mx};
    const int16_t ry0[4] = {q.y0, q.y0, (int16_t)my, (int16_t)my};
    const int16_t rx1[4] = {(int16_t)mx, q.x1, (int16_t)mx, q.x1};
    const int16_t ry1[4] = {(int16_t)my, (int16_t)my, q.y1, q.y1};
    for (int c = 0; c < 4; c++) {
      if (cnt4[c] == 0) continue;
      const int ns = alloc();
      const int id = next_id++;
      head--;
      if (ns >= 0 && lane == 0) {
        QNode& d = S.node[ns];
        d.x0 = rx0[c];
        d.y0 = ry0[c];
        d.x1 = rx1[c];
        d.y1 = ry1[c];
        d.beg = q.beg + off4[c];
        d.cnt = cnt4[c];
        d.id = id;
        d.buf = q.buf ^ 1;
        d.nomore = cnt4[c] == 1;
        d.alive = 1;
        d.pos = head;
        S.order[head] = (int16_t)ns;
      }
      alive++;
      if (cnt4[c] > 1) {
        nToExpand++;
        if (lane == 0 && ns >= 0) S.vcur[nvcur] = (int16_t)ns;
        nvcur++;
      }
    }
    // erase the parent
    if (lane == 0) {
      S.order[q.pos] = -1;
      S.node[s].alive = 0;
      S.freel[nfree] = (int16_t)s;
    }
    nfree++;
    alive--;
    __syncthreads();
  };

  // move live entries of order[head..QOS) to the tail, preserving order
  auto compact = [&]() {
    int w = 0;
    for (int c0 = head; c0 < QOS; c0 += 64) {
      const int idx = c0 + lane;
      const int v = idx < QOS ? S.order[idx] : -1;
      const uint64_t m = ballot(v >= 0);
      const int p = w + popc64(m & lanes_below());
      // write into vprev as a staging area (reused; vprev is free here)
      if (v >= 0) S.skey[p] = (unsigned long long)v;
      w += popc64(m);
    }
    __syncthreads();
    head = QOS - w;
    for (int i = lane; i < w; i += 64) {
      const int s = (int)S.skey[i];
      S.order[head + i] = (int16_t)s;
      S.node[s].pos = head + i;
    }
    __syncthreads();
  };

  bool finish = false;
  while (!finish && !overflow) {
    const int prevSize = alive;
    nToExpand = 0;
    nvcur = 0;
    const int end = QOS;
    // walk the list in order, 64 positions at a time: the nodes to divide
    // are found by ballot (divide only writes positions < head and its own,
    // so the flags read for later positions of the chunk stay valid)
    for (int c0 = head; c0 < end && !overflow; c0 += 64) {
      const int i = c0 + lane;
      const int s = i < end ? (int)S.order[i] : -1;
      uint64_t m = ballot(s >= 0 && !S.node[s >= 0 ? s : 0].nomore);
      while (m) {
        const int b = __builtin_ctzll(m);
        m &= m - 1;
        divide(__builtin_amdgcn_readlane(s, b));
        if (overflow) break;
      }
    }
    compact();
    if (alive >= N || alive == prevSize) {
      finish = true;
    } else if (alive + nToExpand * 3 > N) {
      while (!finish && !overflow) {
        const int prev2 = alive;
        const int nv = nvcur;
        for (int i = lane; i < nv; i += 64) S.vprev[i] = S.vcur[i];
        __syncthreads();
        nvcur = 0;
        // sort vprev by (size, id) ascending: bitonic over P = next pow2.
        // key = size << 32 | id << 11 | slot (ids unique, slot < QCAP=2^11)
        int P = 1;
        while (P < nv) P <<= 1;
        for (int i = lane; i < P; i += 64) {
          if (i < nv) {
            const int sl = S.vprev[i];
            const QNode& q = S.node[sl];
            S.skey[i] = ((unsigned long long)(uint32_t)q.cnt << 32) |
                        ((unsigned long long)(uint32_t)q.id << 11) | (unsigned long long)sl;
          } else
            S.skey[i] = ~0ull;
        }
        __syncthreads();
        for (int k = 2; k <= P; k <<= 1) {
          for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = lane; i < P; i += 64) {
              const int ixj = i ^ j;
              if (ixj > i) {
                const unsigned long long a = S.skey[i], b = S.skey[ixj];
                const bool up = (i & k) == 0;
                if ((a > b) == up) {
                  S.skey[i] = b;
                  S.skey[ixj] = a;
                }
              }
            }
            __syncthreads();
          }
        }
        for (int i = lane; i < nv; i += 64) S.vprev[i] = (int16_t)(S.skey[i] & 0x7ffu);
        __syncthreads();
        for (int j = nv - 1; j >= 0; j--) {
          const int s = S.vprev[j];
          divide(s);
          if (overflow) break;
          if (alive >= N) break;
        }
        compact();
        if (alive >= N || alive == prev2) finish = true;
      }
    }
  }
  // ---- retain the best keypoint per node (largest score, first in the
  // node's key order on ties), in list order: one node per lane, 64 nodes
  // at a time, outputs placed by ballot prefix (final nodes hold few keys)
  int outn = 0;
  for (int c0 = head; c0 < QOS; c0 += 64) {
    const int i = c0 + lane;
    const int s = i < QOS ? S.order[i] : -1;
    uint32_t bk = 0;
    if (s >= 0) {
      const int cnt = S.node[s].cnt;
      const uint32_t* src = bufs(S.node[s].buf) + S.node[s].beg;
      int best_s = -1;
      for (int idx = 0; idx < cnt; idx++) {
        const uint32_t k = src[idx];
        if (kp_s(k) > best_s) {
          best_s = kp_s(k);
          bk = k;
        }
      }
    }
    const uint64_t m = ballot(s >= 0);
    const int p = outn + popc64(m & lanes_below());
    if (s >= 0 && p < L.sel_cap) S_out[p] = bk;
    outn += popc64(m);
  }
  if (lane == 0) *sel_cnt_out = overflow ? -1 : min(outn, L.sel_cap);
}

// lds_keys > 0: the keys of a (level, frame) with n <= lds_keys are distributed in the dynamic
// LDS (2 x lds_keys words), larger ones in qbuf
template <int QCAP>
__global__ __launch_bounds__(64) void k_distribute(const uint32_t* __restrict__ cand,
                                                   long long cand_stride,
                                                   const int* __restrict__ cell_cnt, int ncells,
                                                   const LevelDev* __restrict__ levels,
                                                   const CellDev* __restrict__ cells,
                                                   uint32_t* __restrict__ qbuf, long long qstride,
                                                   uint32_t* __restrict__ sel, long long sel_stride,
                                                   int* __restrict__ sel_cnt, int nlevels, int lds_keys) {
  __shared__ QShared<QCAP> S;
  extern __shared__ uint32_t qk_lds[];
  // grid (frames, levels): workgroups are dispatched x fastest, so every frame's level-0
  // quadtree (the longest walk) starts first and the shorter levels fill in behind it
  const int l = blockIdx.y, f = blockIdx.x, lane = threadIdx.x;
  const LevelDev& L = levels[l];
  const uint32_t* C = cand + f * cand_stride;
  uint32_t* S_out = sel + f * sel_stride + L.sel_off;
  int* sc = sel_cnt + f * nlevels + l;
  // the cells' counts 64 at a time (one lane per cell: independent loads, not a chain of
  // scalar ones over the level's ~340 cells)
  auto cell_count = [&](int k) -> int {
    return k < L.cell_count ? min(cell_cnt[f * ncells + L.cell_begin + k], cells[L.cell_begin + k].cap) : 0;
  };
  int n = 0;
  for (int k0 = 0; k0 < L.cell_count; k0 += 64) n += wave_sum(cell_count(k0 + lane));
  if (n == 0) {
    if (lane == 0) *sc = 0;
    return;
  }
  // ---- gather candidates in vToDistributeKeys order (cells row-major): per 64 cells, an
  // exclusive scan of their counts places each cell, and the wave copies the group's keys as
  // one flat range (a key finds its cell by binary search over the scan, staged in LDS)
  auto gather = [&](uint32_t* B0) {
    int* gpre = (int*)S.skey;  // free until the tree's first compaction
    int* gslot = gpre + 64;
    int o = 0;
    for (int k0 = 0; k0 < L.cell_count; k0 += 64) {
      const int k = k0 + lane;
      const int cnt = cell_count(k);
      int pre = cnt;  // inclusive scan
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int u = __shfl_up(pre, d, 64);
        if (lane >= d) pre += u;
      }
      gpre[lane] = pre - cnt;
      gslot[lane] = k < L.cell_count ? cells[L.cell_begin + k].slot : 0;
      const int tot = __shfl(pre, 63, 64);
      __syncthreads();
      for (int t = lane; t < tot; t += 64) {
        int lo = 0;  // last cell with gpre <= t
#pragma unroll
        for (int step = 32; step > 0; step >>= 1)
          if (gpre[lo + step] <= t) lo += step;
        B0[o + t] = C[gslot[lo] + (t - gpre[lo])];
      }
      o += tot;
      __syncthreads();
    }
  };
  if (n <= lds_keys) {
    gather(qk_lds);
    dist_tree<QCAP, true>(S, qk_lds, qk_lds + lds_keys, n, L, S_out, sc, lane);
  } else {
    // ping-pong halves of this (frame, level): [2 cand_off, 2 cand_off + 2 cand_cap) of the frame area
    uint32_t* B0 = qbuf + f * qstride + 2 * (long long)L.cand_off;
    gather(B0);
    dist_tree<QCAP, false>(S, B0, B0 + L.cand_cap, n, L, S_out, sc, lane);
  }
}

// ---------------------------------------------------------------- quadtree, single frames
// k_distribute_mw: the same DistributeOctTree as k_distribute, NW waves per (level, frame), for
// launches of a few frames (the drop-in's single calls), where one wave's chain of ~140 divides
// per level-0 tree is the latency. The divides of a pass (every expandable node of the list), and
// the candidates of one final-phase round, depend only on their own node: they are counted in
// parallel (a wave per node), one wave places them -- children's ids, list positions, expandable
// list and the point where the final phase reaches N, all exclusive scans over the divides in the
// sequential order --, and they are partitioned in parallel. The sequential pool bound (QCAP nodes
// alive; overflow -> -1) is evaluated on the same scans; the physical pool has room for the
// parents still held while their children are written.
template <int QCAP>
struct QSharedMW {
  static constexpr int QOS = 5 * QCAP;
  static constexpr int PC = 2 * QCAP + 64;  // physical node slots (< 4096: 12 bits in the sort key)
  QNode node[PC];
  int16_t order[QOS];
  int16_t freel[PC];
  int16_t vcur[QCAP];
  int16_t vprev[QCAP];
  int16_t dv[QCAP];  // the round's divides in the sequential order (slots)
  unsigned long long skey[QCAP];
  int dcnt[QCAP][4];  // per divide: keys per child
  int dch[QCAP];      // per divide: children of the earlier divides
  int dex[QCAP];      // per divide: expandable children of the earlier divides
  int ctl[16];
};

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

template <int QCAP, int NW>
__device__ __forceinline__ void dist_tree_mw(QSharedMW<QCAP>& S, uint32_t* B0, uint32_t* B1, int n,
                                             const LevelDev& L, uint32_t* __restrict__ S_out,
                                             int* __restrict__ sel_cnt_out) {
  constexpr int QOS = QSharedMW<QCAP>::QOS, PC = QSharedMW<QCAP>::PC, NT = 64 * NW;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  auto bufs = [&](int b) -> uint32_t* { return b ? B1 : B0; };
  const int N = L.nfeat;
  for (int i = tid; i < PC; i += NT) {
    S.freel[i] = (int16_t)(PC - 1 - i);
    S.node[i].alive = 0;
  }
  // ---- initial nodes (ORBextractor.cc:543-585): a stable partition of the keys by initial node,
  // B0 -> B1, each wave over one contiguous range of keys
  const int nIni = min(L.nIni, 16);
  const float hX = L.hX;
  int* icnt = &S.dcnt[0][0];  // [NW][16]
  const int per = ((n + NW - 1) / NW + 63) & ~63;
  const int r0 = min(n, wv * per), r1 = min(n, r0 + per);
  for (int i = 0; i < nIni; i++) {
    int cnt = 0;
    for (int c0 = r0; c0 < r1; c0 += 64) {
      const int idx = c0 + lane;
      const bool in = idx < r1 && (int)((float)kp_x(B0[idx]) / hX) == i;
      cnt += popc64(ballot(in));
    }
    if (lane == 0) icnt[wv * 16 + i] = cnt;
  }
  __syncthreads();
  {
    int base = 0;
    for (int i = 0; i < nIni; i++) {
      int off = base;
      for (int w = 0; w < NW; w++) {
        if (w == wv) break;
        off += icnt[w * 16 + i];
      }
      for (int c0 = r0; c0 < r1; c0 += 64) {
        const int idx = c0 + lane;
        const bool in = idx < r1 && (int)((float)kp_x(B0[idx]) / hX) == i;
        const uint64_t m = ballot(in);
        if (in) B1[off + popc64(m & lanes_below())] = B0[idx];
        off += popc64(m);
      }
      for (int w = 0; w < NW; w++) base += icnt[w * 16 + i];
    }
  }
  if (tid == 0) {
    int base = 0, alive = 0, nfp = PC;
    int slots[16];
    for (int i = 0; i < nIni; i++) {
      int cnt = 0;
      for (int w = 0; w < NW; w++) cnt += icnt[w * 16 + i];
      slots[i] = -1;
      if (cnt > 0) {
        const int s = S.freel[--nfp];
        slots[i] = s;
        QNode& q = S.node[s];
        q.x0 = (int16_t)(int)(hX * (float)i);
        q.x1 = (int16_t)(int)(hX * (float)(i + 1));
        q.y0 = 0;
        q.y1 = (int16_t)(L.maxBY - L.minBY);
        q.beg = base;
        q.cnt = cnt;
        q.id = i;  // every initial node takes an id, empty or not
        q.buf = 1;
        q.nomore = cnt == 1;
        q.alive = 1;
        alive++;
      }
      base += cnt;
    }
    int p = QOS - alive;
    for (int i = 0; i < nIni; i++)
      if (slots[i] >= 0) {
        S.order[p] = (int16_t)slots[i];
        S.node[slots[i]].pos = p;
        p++;
      }
    S.ctl[0] = alive;
    S.ctl[1] = nfp;
  }
  __syncthreads();
  int alive = S.ctl[0], nfp = S.ctl[1];
  int next_id = nIni;
  int head = QOS - alive;
  bool overflow = false;
  int nvcur = 0;

  // keys per child of the round's divide d
  auto count = [&](int d) {
    const QNode q = S.node[S.dv[d]];
    const int mx = q.x0 + (int)ceilf((float)(q.x1 - q.x0) / 2), my = q.y0 + (int)ceilf((float)(q.y1 - q.y0) / 2);
    const uint32_t* src = bufs(q.buf) + q.beg;
    int c4[4] = {0, 0, 0, 0};
    for (int c0 = 0; c0 < q.cnt; c0 += 256) {
      int ch[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int idx = c0 + 64 * j + lane;
        ch[j] = idx < q.cnt ? child_of(src[idx], mx, my) : 4;
      }
#pragma unroll
      for (int j = 0; j < 4; j++)
#pragma unroll
        for (int c = 0; c < 4; c++) c4[c] += popc64(ballot(ch[j] == c));
    }
    if (lane < 4) S.dcnt[d][lane] = lane == 0 ? c4[0] : lane == 1 ? c4[1] : lane == 2 ? c4[2] : c4[3];
  };
  // one wave: children / expandable prefixes over the nd divides, the sequential overflow and
  // (final phase) the divide after which alive reaches N; ctl[2..5] = executed, children,
  // expandables, overflow
  auto place = [&](int nd, bool final_phase) {
    if (wv == 0) {
      int chT = 0, exT = 0, ndo = nd, ovf = 0;
      for (int c0 = 0; c0 < nd; c0 += 64) {
        const int d = c0 + lane;
        const bool valid = d < nd;
        int ch = 0, ex = 0;
        if (valid)
#pragma unroll
          for (int c = 0; c < 4; c++) {
            const int k = S.dcnt[d][c];
            ch += k > 0;
            ex += k > 1;
          }
        int pch = ch, pex = ex;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int u = __shfl_up(pch, o, 64), v = __shfl_up(pex, o, 64);
          if (lane >= o) {
            pch += u;
            pex += v;
          }
        }
        if (valid) {
          S.dch[d] = chT + pch - ch;
          S.dex[d] = exT + pex - ex;
        }
        const int ab = alive + chT + pch - ch - d;  // alive before divide d
        const uint64_t mo = ballot(valid && ch > QCAP - ab);
        const uint64_t ms = ballot(final_phase && valid && ab + ch - 1 >= N);
        const int fo = mo ? __builtin_ctzll(mo) : 64, fs = ms ? __builtin_ctzll(ms) : 64;
        if (fo < 64 && fo <= fs) {
          ovf = 1;
          break;
        }
        if (fs < 64) {
          ndo = c0 + fs + 1;
          chT += __shfl(pch, fs, 64);
          exT += __shfl(pex, fs, 64);
          break;
        }
        chT += __shfl(pch, 63, 64);
        exT += __shfl(pex, 63, 64);
      }
      if (lane == 0) {
        S.ctl[2] = ndo;
        S.ctl[3] = chT;
        S.ctl[4] = exT;
        S.ctl[5] = ovf;
      }
    }
  };
  // partition divide d's keys into the other buffer, write its children, erase it
  auto scatter = [&](int d) {
    const int s = S.dv[d];
    const QNode q = S.node[s];
    const int hx = (int)ceilf((float)(q.x1 - q.x0) / 2), hy = (int)ceilf((float)(q.y1 - q.y0) / 2);
    const int mx = q.x0 + hx, my = q.y0 + hy;
    const uint32_t* src = bufs(q.buf) + q.beg;
    uint32_t* dst = bufs(q.buf ^ 1) + q.beg;
    int c4[4], off4[4], run4[4] = {0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < 4; c++) c4[c] = S.dcnt[d][c];
    off4[0] = 0;
    off4[1] = c4[0];
    off4[2] = c4[0] + c4[1];
    off4[3] = off4[2] + c4[2];
    for (int c0 = 0; c0 < q.cnt; c0 += 256) {
      uint32_t kr[4];
      int ch[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int idx = c0 + 64 * j + lane;
        kr[j] = idx < q.cnt ? src[idx] : 0u;
        ch[j] = idx < q.cnt ? child_of(kr[j], mx, my) : 4;
      }
#pragma unroll
      for (int j = 0; j < 4; j++)
#pragma unroll
        for (int c = 0; c < 4; c++) {
          const uint64_t m = ballot(ch[j] == c);
          if (ch[j] == c) dst[off4[c] + run4[c] + popc64(m & lanes_below())] = kr[j];
          run4[c] += popc64(m);
        }
    }
    const int16_t rx0[4] = {q.x0, (int16_t)mx, q.x0, (int16_t)mx};
    const int16_t ry0[4] = {q.y0, q.y0, (int16_t)my, (int16_t)my};
    const int16_t rx1[4] = {(int16_t)mx, q.x1, (int16_t)mx, q.x1};
    const int16_t ry1[4] = {(int16_t)my, (int16_t)my, q.y1, q.y1};
    if (lane == 0) {
      int g = S.dch[d], e = S.dex[d];
      for (int c = 0; c < 4; c++) {
        if (c4[c] == 0) continue;
        const int ns = S.freel[nfp - 1 - g];
        QNode& dn = S.node[ns];
        dn.x0 = rx0[c];
        dn.y0 = ry0[c];
        dn.x1 = rx1[c];
        dn.y1 = ry1[c];
        dn.beg = q.beg + off4[c];
        dn.cnt = c4[c];
        dn.id = next_id + g;
        dn.buf = q.buf ^ 1;
        dn.nomore = c4[c] == 1;
        dn.alive = 1;
        dn.pos = head - 1 - g;
        S.order[head - 1 - g] = (int16_t)ns;
        if (c4[c] > 1) S.vcur[e++] = (int16_t)ns;
        g++;
      }
      S.order[q.pos] = -1;
      S.node[s].alive = 0;
    }
  };
  // one round: count, place, partition; false on the sequential pool overflow
  auto round = [&](int nd, bool final_phase) -> bool {
    for (int d = wv; d < nd; d += NW) count(d);
    __syncthreads();
    place(nd, final_phase);
    __syncthreads();
    const int ndo = S.ctl[2], T = S.ctl[3], E = S.ctl[4];
    if (S.ctl[5]) return false;
    for (int d = wv; d < ndo; d += NW) scatter(d);
    __syncthreads();
    // the parents' slots back to the pool (after every child took its slot)
    for (int d = tid; d < ndo; d += NT) S.freel[nfp - T + d] = S.dv[d];
    alive += T - ndo;
    next_id += T;
    head -= T;
    nfp += ndo - T;
    nvcur = E;
    return true;
  };
  // move live entries of order[head..QOS) to the tail, preserving order
  auto compact = [&]() {
    __syncthreads();
    if (wv == 0) {
      int w = 0;
      for (int c0 = head; c0 < QOS; c0 += 64) {
        const int idx = c0 + lane;
        const int v = idx < QOS ? S.order[idx] : -1;
        const uint64_t m = ballot(v >= 0);
        if (v >= 0) S.skey[w + popc64(m & lanes_below())] = (unsigned long long)v;
        w += popc64(m);
      }
      if (lane == 0) S.ctl[6] = w;
    }
    __syncthreads();
    const int w = S.ctl[6];
    head = QOS - w;
    for (int i = tid; i < w; i += NT) {
      const int s = (int)S.skey[i];
      S.order[head + i] = (int16_t)s;
      S.node[s].pos = head + i;
    }
    __syncthreads();
  };

  bool finish = false;
  while (!finish && !overflow) {
    const int prevSize = alive;
    // the pass divides every expandable node, in list order
    if (wv == 0) {
      int nd = 0;
      for (int c0 = head; c0 < QOS; c0 += 64) {
        const int i = c0 + lane;
        const int s = i < QOS ? (int)S.order[i] : -1;
        const uint64_t m = ballot(s >= 0 && !S.node[s >= 0 ? s : 0].nomore);
        if (s >= 0 && !S.node[s].nomore) S.dv[nd + popc64(m & lanes_below())] = (int16_t)s;
        nd += popc64(m);
      }
      if (lane == 0) S.ctl[7] = nd;
    }
    __syncthreads();
    if (!round(S.ctl[7], false)) {
      overflow = true;
      break;
    }
    compact();
    if (alive >= N || alive == prevSize) {
      finish = true;
    } else if (alive + nvcur * 3 > N) {
      while (!finish && !overflow) {
        const int prev2 = alive;
        const int nv = nvcur;
        // the expandable children by (size, id), largest first
        int P = 1;
        while (P < nv) P <<= 1;
        for (int i = tid; i < P; i += NT) {
          if (i < nv) {
            const int sl = S.vcur[i];
            const QNode& q = S.node[sl];
            S.skey[i] = ((unsigned long long)(uint32_t)q.cnt << 32) | ((unsigned long long)(uint32_t)q.id << 12) |
                        (unsigned long long)sl;
          } else
            S.skey[i] = ~0ull;
        }
        __syncthreads();
        for (int k = 2; k <= P; k <<= 1)
          for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < P; i += NT) {
              const int ixj = i ^ j;
              if (ixj > i) {
                const unsigned long long a = S.skey[i], b = S.skey[ixj];
                if ((a > b) == ((i & k) == 0)) {
                  S.skey[i] = b;
                  S.skey[ixj] = a;
                }
              }
            }
            __syncthreads();
          }
        for (int d = tid; d < nv; d += NT) S.dv[d] = (int16_t)(S.skey[nv - 1 - d] & 0xfffu);
        __syncthreads();
        if (!round(nv, true)) {
          overflow = true;
          break;
        }
        compact();
        if (alive >= N || alive == prev2) finish = true;
      }
    }
  }
  // ---- retain the best keypoint per node (largest score, first in the node's key order on
  // ties), in list order (the list is compact: position i - head)
  if (!overflow)
    for (int i = head + tid; i < QOS; i += NT) {
      const int s = S.order[i];
      const int cnt = S.node[s].cnt;
      const uint32_t* src = bufs(S.node[s].buf) + S.node[s].beg;
      int best_s = -1;
      uint32_t bk = 0;
      for (int idx = 0; idx < cnt; idx++) {
        const uint32_t k = src[idx];
        if (kp_s(k) > best_s) {
          best_s = kp_s(k);
          bk = k;
        }
      }
      if (i - head < L.sel_cap) S_out[i - head] = bk;
    }
  if (tid == 0) *sel_cnt_out = overflow ? -1 : min(QOS - head, L.sel_cap);
}

template <int QCAP, int NW>
__global__ __launch_bounds__(64 * NW) void k_distribute_mw(const uint32_t* __restrict__ cand, long long cand_stride,
                                                           const int* __restrict__ cell_cnt, int ncells,
                                                           const LevelDev* __restrict__ levels,
                                                           const CellDev* __restrict__ cells,
                                                           uint32_t* __restrict__ qbuf, long long qstride,
                                                           uint32_t* __restrict__ sel, long long sel_stride,
                                                           int* __restrict__ sel_cnt, int nlevels, int lds_keys) {
  __shared__ QSharedMW<QCAP> S;
  extern __shared__ uint32_t qk_lds[];
  const int l = blockIdx.y, f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const LevelDev& L = levels[l];
  const uint32_t* C = cand + f * cand_stride;
  uint32_t* S_out = sel + f * sel_stride + L.sel_off;
  int* sc = sel_cnt + f * nlevels + l;
  auto cell_count = [&](int k) -> int {
    return k < L.cell_count ? min(cell_cnt[f * ncells + L.cell_begin + k], cells[L.cell_begin + k].cap) : 0;
  };
  int n = 0;
  for (int k0 = 0; k0 < L.cell_count; k0 += 64) n += wave_sum(cell_count(k0 + lane));
  if (n == 0) {
    if (tid == 0) *sc = 0;
    return;
  }
  // ---- gather in vToDistributeKeys order: wave w takes the groups of 64 cells g = w, w + NW, ..,
  // placed after the earlier groups' totals
  const int ng = (L.cell_count + 63) >> 6;
  auto gather = [&](uint32_t* B0) {
    int* gtot = S.dch;  // [ng], free until the first round
    for (int g = wv; g < ng; g += NW) {
      const int t = wave_sum(cell_count(64 * g + lane));
      if (lane == 0) gtot[g] = t;
    }
    __syncthreads();
    int* gpre = &S.dcnt[0][0] + 128 * wv;  // per-wave scan table
    int* gslot = gpre + 64;
    for (int g = wv; g < ng; g += NW) {
      int o = 0;
      for (int h = 0; h < g; h++) o += gtot[h];
      const int k = 64 * g + lane;
      const int cnt = cell_count(k);
      int pre = cnt;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int u = __shfl_up(pre, d, 64);
        if (lane >= d) pre += u;
      }
      wave_lds_sync();
      gpre[lane] = pre - cnt;
      gslot[lane] = k < L.cell_count ? cells[L.cell_begin + k].slot : 0;
      wave_lds_sync();
      const int tot = __shfl(pre, 63, 64);
      for (int t = lane; t < tot; t += 64) {
        int lo = 0;
#pragma unroll
        for (int step = 32; step > 0; step >>= 1)
          if (gpre[lo + step] <= t) lo += step;
        B0[o + t] = C[gslot[lo] + (t - gpre[lo])];
      }
    }
    __syncthreads();
  };
  if (n <= lds_keys) {
    gather(qk_lds);
    dist_tree_mw<QCAP, NW>(S, qk_lds, qk_lds + lds_keys, n, L, S_out, sc);
  } else {
    uint32_t* B0 = qbuf + f * qstride + 2 * (long long)L.cand_off;
    gather(B0);
    dist_tree_mw<QCAP, NW>(S, B0, B0 + L.cand_cap, n, L, S_out, sc);
  }
}

// ---------------------------------------------------------------- orientation

// fastAtan2 (OpenCV 3.2), fp32, no contraction
__device__ float fast_atan2(float y, float x) {
  const float p1 = 0.9997878412794807f * (float)(180 / M_PI);
  const float p3 = -0.3258083974640975f * (float)(180 / M_PI);
  const float p5 = 0.1555786518463281f * (float)(180 / M_PI);
  const float p7 = -0.04432655554792128f * (float)(180 / M_PI);
  const float ax = fabsf(x), ay = fabsf(y);
  float a, c, c2;
  if (ax >= ay) {
    c = fdiv(ay, fadd(ax, (float)2.220446049250313e-16));
    c2 = fmul(c, c);
    a = fmul(fadd(fmul(fadd(fmul(fadd(fmul(p7, c2), p5), c2), p3), c2), p1), c);
  } else {
    c = fdiv(ax, fadd(ay, (float)2.220446049250313e-16));
    c2 = fmul(c, c);
    a = fsub(90.f, fmul(fadd(fmul(fadd(fmul(fadd(fmul(p7, c2), p5), c2), p3), c2), p1), c));
  }
  if (x < 0) a = fsub(180.f, a);
  if (y < 0) a = fsub(360.f, a);
  return a;
}

// ---------------------------------------------------------------- describe
// GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) of the level, fused: the reference
// blurs a clone of every level (ORBextractor.cc:1085-1086) and computeDescriptors reads
// 512 pattern taps of it around each keypoint. Here one wave per keypoint stages the
// raw 43 x 43 patch (pattern reach 18 + blur 3) in LDS, takes IC_Angle from it, forms
// the horizontal 7-tap sums of the 43 x 37 rows it needs and finishes the vertical sum
// only at the 512 rotated taps -- no blurred plane in HBM. Blur arithmetic is the 8U
// fixed point of cv::GaussianBlur, exact in integers: horizontal sums of 8-bit pixels
// x 8-bit taps stay below 2^16, then (sum_v + 2^15) >> 16, saturated.
constexpr int PR = 21;          // staged patch radius
constexpr int PW = 2 * PR + 1;  // staged rows
constexpr int PD = 13;          // staged dwords per row (12 + one pad for the last column group)
constexpr int HC = 40;          // horizontal sums per row: dx = -18 .. 21 (37 used)

// one workgroup = 4 waves = 4 keypoints; control flow stays uniform over the barriers
__global__ __launch_bounds__(256) void k_describe(
    const uint8_t* __restrict__ frames, int fpitch, long long fstride,
    const uint8_t* __restrict__ pyr, long long pstride, const LevelDev* __restrict__ levels,
    const uint32_t* __restrict__ sel, long long sel_stride, const int* __restrict__ sel_cnt,
    const int2* __restrict__ slot_map, int nslots, int nlevels, const int* __restrict__ umax,
    const int* __restrict__ gk, eao_keypoint_dev* __restrict__ out_kps, uint8_t* __restrict__ out_desc,
    int* __restrict__ out_cnt, int cap, int gx) {
  __shared__ uint32_t raw[4][PW][PD];
  __shared__ uint16_t hs[4][PW][HC];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // XCD-aware order (bijective swizzle): blocks b and b + 8 share an XCD, so each group
  // of blocks takes a contiguous run of (frame, slot group) ids -- a frame's keypoints
  // then read its level planes through one L2 instead of all eight
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int f = wg / gx, sg = wg - f * gx;
  const int slot = sg * 4 + w;
  const int* cnts = sel_cnt + f * nlevels;
  if (sg == 0 && threadIdx.x == 0) {
    int tot = 0;
    for (int i = 0; i < nlevels; i++) tot += max(cnts[i], 0);
    out_cnt[f] = tot;
  }
  int2 sm = make_int2(0, 0);
  bool active = slot < nslots;
  if (active) {
    sm = slot_map[slot];  // (level, index within level)
    active = sm.y < cnts[sm.x];
  }
  const int l = sm.x, k = sm.y;
  const LevelDev& L = levels[l];
  int x = 0, y = 0, off = 0;
  uint32_t pk = 0;
  uint8_t* rb = (uint8_t*)&raw[w][0][0];
  if (active) {
    pk = sel[f * sel_stride + L.sel_off + k];
    x = kp_x(pk) + L.minBX;
    y = kp_y(pk) + L.minBY;
    const uint8_t* img;
    int pitch;
    if (l == 0) {
      img = frames + f * fstride;
      pitch = fpitch;
    } else {
      img = pyr + f * pstride + L.plane_off;
      pitch = L.pitch;
    }
    const int xa = (x - PR) & ~3;
    if (x - PR >= 0 && x + PR < L.w && y - PR >= 0 && y + PR < L.h && (pitch & 3) == 0 && xa + 48 <= pitch) {
      // interior: 12 aligned dwords per row from x - PR rounded down; `off` bytes of lead
      off = x - PR - xa;
      const uint32_t* src = (const uint32_t*)(img + (long long)(y - PR) * pitch + xa);
      for (int i = lane; i < PW * 12; i += 64) {
        const int r = i / 12, c = i - r * 12;
        raw[w][r][c] = src[r * (pitch >> 2) + c];
      }
    } else {
      // near the level edge: bytes with REFLECT_101 on the isolated level (gfedcb|abcdefgh|gfedcba)
      for (int i = lane; i < PW * PW; i += 64) {
        const int r = i / PW, c = i - r * PW;
        int yy = y - PR + r, xx = x - PR + c;
        if (L.h == 1) yy = 0;
        while (yy < 0 || yy >= L.h) yy = yy < 0 ? -yy : 2 * L.h - 2 - yy;
        if (L.w == 1) xx = 0;
        while (xx < 0 || xx >= L.w) xx = xx < 0 ? -xx : 2 * L.w - 2 - xx;
        rb[r * 4 * PD + c] = img[(long long)yy * pitch + xx];
      }
    }
    if (lane < PW) raw[w][lane][12] = 0;
  }
  __syncthreads();
  // ---- IC_Angle (ORBextractor.cc:77-104) on the raw patch: integer moments, wave reduction
  int m10 = 0, m01 = 0;
  const uint8_t* center = rb + PR * 4 * PD + off + PR;
  if (active) {
    if (lane < 31) m10 += (lane - 15) * center[lane - 15];
    for (int v = 1 + (lane >> 5); v <= 15; v += 2) {
      const int d = umax[v];
      const int u = (lane & 31) - d;
      if (u <= d) {
        const int vp = center[u + v * 4 * PD], vm = center[u - v * 4 * PD];
        m10 += u * (vp + vm);
        m01 += v * (vp - vm);
      }
    }
    // ---- horizontal 7-tap sums: item (row, group of 4 output columns); output column c
    // (dx = c - 18) sums staged bytes off + c .. off + c + 6 -- v_dot4 on realigned words
    const uint32_t K0 = (uint32_t)gk[0] | ((uint32_t)gk[1] << 8) | ((uint32_t)gk[2] << 16) | ((uint32_t)gk[3] << 24);
    const uint32_t K1 = (uint32_t)gk[4] | ((uint32_t)gk[5] << 8) | ((uint32_t)gk[6] << 16);
    for (int i = lane; i < PW * (HC / 4); i += 64) {
      const int r = i / (HC / 4), g = i - r * (HC / 4);
      const uint32_t* rw = &raw[w][r][g];
      const uint32_t W0 = rw[0], W1 = rw[1], W2 = rw[2], W3 = rw[3];
      const uint32_t A0 = __builtin_amdgcn_alignbyte(W1, W0, off);
      const uint32_t A1 = __builtin_amdgcn_alignbyte(W2, W1, off);
      const uint32_t A2 = __builtin_amdgcn_alignbyte(W3, W2, off);
      uint32_t h[4];
      h[0] = __builtin_amdgcn_udot4(A0, K0, __builtin_amdgcn_udot4(A1, K1, 0u, false), false);
#pragma unroll
      for (int o = 1; o < 4; o++) {
        const uint32_t lo = __builtin_amdgcn_alignbyte(A1, A0, o), hi = __builtin_amdgcn_alignbyte(A2, A1, o);
        h[o] = __builtin_amdgcn_udot4(lo, K0, __builtin_amdgcn_udot4(hi, K1, 0u, false), false);
      }
      uint32_t* hw = (uint32_t*)&hs[w][r][4 * g];
      hw[0] = h[0] | (h[1] << 16);
      hw[1] = h[2] | (h[3] << 16);
    }
  }
  m10 = wave_sum(m10);
  m01 = wave_sum(m01);
  __syncthreads();
  if (!active) return;  // no barrier follows
  const float angle = fast_atan2((float)m01, (float)m10);
  // ---- rBRIEF (ORBextractor.cc:108-147): the vertical 7-tap sum at each rotated tap
  const float factorPI = (float)(M_PI / 180.f);
  const float ang = fmul(angle, factorPI);
  const float a = (float)cos((double)ang), b = (float)sin((double)ang);
  int kv[7];
#pragma unroll
  for (int j = 0; j < 7; j++) kv[j] = gk[j];
  const int byte = lane >> 1, half = lane & 1;
  int px[8];
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const int pi = 16 * byte + 8 * half + e;
    const float fx = (float)c_pattern[2 * pi], fy = (float)c_pattern[2 * pi + 1];
    const int dy = dev_round(fadd(fmul(fx, b), fmul(fy, a)));
    const int dx = dev_round(fsub(fmul(fx, a), fmul(fy, b)));
    const uint16_t* col = &hs[w][PR + dy - 3][dx + 18];
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < 7; j++) acc += (uint32_t)kv[j] * col[j * HC];
    px[e] = (int)min((acc + (1u << 15)) >> 16, 255u);
  }
  int nib = 0;
#pragma unroll
  for (int t = 0; t < 4; t++) nib |= (px[2 * t] < px[2 * t + 1]) << t;
  const int other = __shfl_xor(nib, 1, 64);
  int off_l = 0;
  for (int i = 0; i < l; i++) off_l += max(cnts[i], 0);
  const long long oi = (long long)f * cap + off_l + k;
  if (half == 0) out_desc[oi * 32 + byte] = (uint8_t)(nib | (other << 4));
  if (lane == 0) {
    eao_keypoint_dev kp;
    if (l == 0) {
      kp.x = (float)x;
      kp.y = (float)y;
    } else {
      kp.x = fmul((float)x, L.scale);
      kp.y = fmul((float)y, L.scale);
    }
    kp.size = L.size;
    kp.angle = angle;
    kp.response = (float)kp_s(pk);
    kp.octave = l;
    kp.class_id = -1;
    out_kps[oi] = kp;
  }
}

// ================================================================ host plan
static inline int cv_round(float v) { return (int)lrintf(v); }
static inline short sat_s16(float v) {
  int iv = cv_round(v);
  return (short)(iv < -32768 ? -32768 : (iv > 32767 ? 32767 : iv));
}

int OrbEngine::plan(const eao_orb_params& prm, int device) {
  p = prm;
  dev = device;
  const int nl = p.nlevels;
  if (nl < 1 || nl > 16 || p.width < 64 || p.height < 64 || p.width > 4096 || p.height > 4096 ||
      p.max_batch < 1 || p.nfeatures < 1) {
    set_error("eao_orb_create: bad parameters");
    return EAO_E_ARG;
  }
  // ORBextractor::ORBextractor, ORBextractor.cc:410-470
  const double sf = (double)p.scale_factor;
  scale.assign(nl, 1.f);
  sigma2.assign(nl, 1.f);
  for (int i = 1; i < nl; i++) {
    scale[i] = (float)((double)scale[i - 1] * sf);
    sigma2[i] = scale[i] * scale[i];
  }
  inv_scale.resize(nl);
  inv_sigma2.resize(nl);
  for (int i = 0; i < nl; i++) {
    inv_scale[i] = 1.0f / scale[i];
    inv_sigma2[i] = 1.0f / sigma2[i];
  }
  quotas.resize(nl);
  {
    float factor = (float)(1.0f / sf);
    float nd = (float)p.nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nl));
    int sum = 0;
    for (int l = 0; l < nl - 1; l++) {
      quotas[l] = cv_round(nd);
      sum += quotas[l];
      nd *= factor;
    }
    quotas[nl - 1] = std::max(p.nfeatures - sum, 0);
  }
  {
    int v, v0;
    const int HP = 15;
    int vmax = (int)std::floor((float)HP * std::sqrt(2.f) / 2 + 1);
    int vmin = (int)std::ceil((float)HP * std::sqrt(2.f) / 2);
    const double hp2 = HP * HP;
    umax.assign(HP + 1, 0);
    for (v = 0; v <= vmax; ++v) umax[v] = (int)lrint(std::sqrt(hp2 - v * v));
    for (v = HP, v0 = 0; v >= vmin; --v) {
      while (umax[v0] == umax[v0 + 1]) ++v0;
      umax[v] = v0;
      ++v0;
    }
  }
  {
    // getGaussianKernel(7, 2, CV_32F) -> x256 integer taps
    float cf[7];
    double s = 0;
    const double scale2X = -0.5 / (2.0 * 2.0);
    for (int i = 0; i < 7; i++) {
      double x = i - 3.0;
      cf[i] = (float)std::exp(scale2X * x * x);
      s += cf[i];
    }
    s = 1. / s;
    gk.resize(7);
    for (int i = 0; i < 7; i++) {
      cf[i] = (float)(cf[i] * s);
      gk[i] = (int)lrint((double)cf[i] * 256.0);
    }
  }
  levels.assign(nl, LevelDev{});
  cells.clear();
  resize_xofs.clear();
  resize_ia.clear();
  resize_yrows.clear();
  resize_ib.clear();
  long long poff = 0;
  int cand_total = 0, sel_total = 0, rsmax = 0, rhmax = 0;
  for (int l = 0; l < nl; l++) {
    LevelDev& L = levels[l];
    L.w = cv_round((float)p.width * inv_scale[l]);
    L.h = cv_round((float)p.height * inv_scale[l]);
    L.pitch = (L.w + 63) & ~63;
    if (l > 0) {
      L.plane_off = poff;
      poff += (long long)L.pitch * L.h;
    }
    L.minBX = 16;
    L.minBY = 16;
    L.maxBX = L.w - 16;
    L.maxBY = L.h - 16;
    L.nfeat = quotas[l];
    L.scale = scale[l];
    L.size = (float)(int)(31 * scale[l]);
    // cells, ORBextractor.cc:769-829
    const float W = 30;
    const float width = (float)(L.maxBX - L.minBX), height = (float)(L.maxBY - L.minBY);
    const int nCols = (int)(width / W), nRows = (int)(height / W);
    if (nCols < 1 || nRows < 1) {
      set_error("eao_orb_create: image too small for the pyramid");
      return EAO_E_ARG;
    }
    L.wCell = (int)std::ceil(width / nCols);
    L.hCell = (int)std::ceil(height / nRows);
    L.cell_begin = (int)cells.size();
    L.cand_off = cand_total;
    for (int i = 0; i < nRows; i++) {
      const float iniY = (float)(L.minBY + i * L.hCell);
      float maxY = iniY + L.hCell + 6;
      if (iniY >= L.maxBY - 3) continue;
      if (maxY > L.maxBY) maxY = (float)L.maxBY;
      for (int j = 0; j < nCols; j++) {
        const float iniX = (float)(L.minBX + j * L.wCell);
        float maxX = iniX + L.wCell + 6;
        if (iniX >= L.maxBX - 6) continue;
        if (maxX > L.maxBX) maxX = (float)L.maxBX;
        CellDev c{};
        c.level = (int16_t)l;
        c.i = (int16_t)i;
        c.j = (int16_t)j;
        c.x0 = (int16_t)(int)iniX;
        c.y0 = (int16_t)(int)iniY;
        c.x1 = (int16_t)(int)maxX;
        c.y1 = (int16_t)(int)maxY;
        const int iw = std::max(c.x1 - c.x0 - 6, 0), ih = std::max(c.y1 - c.y0 - 6, 0);
        c.cap = ((iw + 1) / 2) * ((ih + 1) / 2);
        c.slot = cand_total;
        cand_total += c.cap;
        rsmax = std::max(rsmax, c.x1 - c.x0);
        rhmax = std::max(rhmax, c.y1 - c.y0);
        cells.push_back(c);
      }
    }
    L.cell_count = (int)cells.size() - L.cell_begin;
    L.cand_cap = cand_total - L.cand_off;
    L.nIni = (int)std::round((float)(L.maxBX - L.minBX) / (L.maxBY - L.minBY));
    L.hX = (float)(L.maxBX - L.minBX) / L.nIni;
    if (L.nIni < 1 || L.nIni > 16 || L.nfeat + 4 * L.nIni + 16 > QCAP_MAX) {
      set_error("eao_orb_create: level geometry outside the quadtree kernel limits");
      return EAO_E_ARG;
    }
    L.sel_off = sel_total;
    L.sel_cap = std::max(L.nfeat + 2, 4 * L.nIni) + 8;
    sel_total += L.sel_cap;
    // resize tables (levels >= 1), OpenCV resize INTER_LINEAR
    if (l > 0) {
      const LevelDev& S = levels[l - 1];
      const int sw = S.w, sh = S.h, dw = L.w, dh = L.h;
      const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
      L.tab_x = (int)resize_xofs.size();
      L.tab_y = (int)resize_yrows.size() / 2;
      int xmax = dw;
      for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)std::floor(fx);
        fx -= sx;
        if (sx < 0) {
          fx = 0;
          sx = 0;
        }
        if (sx + 1 >= sw) {
          xmax = std::min(xmax, dx);
          if (sx >= sw - 1) {
            fx = 0;
            sx = sw - 1;
          }
        }
        resize_xofs.push_back(sx);
        resize_ia.push_back(sat_s16((1.f - fx) * 2048));
        resize_ia.push_back(sat_s16(fx * 2048));
      }
      L.xmax = xmax;
      for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = (int)std::floor(fy);
        fy -= sy;
        resize_ib.push_back(sat_s16((1.f - fy) * 2048));
        resize_ib.push_back(sat_s16(fy * 2048));
        resize_yrows.push_back(std::min(std::max(sy, 0), sh - 1));
        resize_yrows.push_back(std::min(std::max(sy + 1, 0), sh - 1));
      }
    }
  }
  pyr_bytes = (long long)((poff + 255) & ~255LL);
  // k_resize_lds tiles: RESIZE_RS-row segments of 4-column groups, up to 4 segments per tile while
  // a tile's items fit RESIZE_IPT per thread of a 1024-thread workgroup; a workgroup of a quarter of
  // the tile's items (4 per thread: 3-wave workgroups at 640x480's level 1) -- more workgroups per CU,
  // so more tiles' loads in flight: 0.257 -> 0.238 ms per 405 frames at 640x480, 1.19 -> 0.94 ms per
  // 256 at 1920x1080 (2 / 3 / 6 / 8 items per thread and 2 / 3 / 8 segments measured slower,
  // profiles/r05_ab_resize_items_per_thread.txt); LDS = the tile's source rows (+16 B: a tap past
  // the last row's end is read with coefficient 0)
  resize_plan.assign(nl, ResizePlan{});
  for (int l = 1; l < nl; l++) {
    const LevelDev& L = levels[l];
    const int G = (L.w + 3) / 4;
    ResizePlan& R = resize_plan[l];
    for (int segs = std::max(1, std::min(4, 1024 * RESIZE_IPT / G)); segs >= 1; segs--) {  // fewer if too wide
      R.tr = RESIZE_RS * segs;
      R.tiles = (L.h + R.tr - 1) / R.tr;
      R.block = std::min(1024, ((G * segs + RESIZE_IPT - 1) / RESIZE_IPT + 63) / 64 * 64);
      int rows = 0;
      for (int t = 0; t < R.tiles; t++) {
        const int d0 = t * R.tr, d1 = std::min(d0 + R.tr, L.h);
        rows = std::max(rows, resize_yrows[2 * (L.tab_y + d1 - 1) + 1] - resize_yrows[2 * (L.tab_y + d0)] + 1);
      }
      R.lds = (size_t)rows * ((levels[l - 1].w + 15) & ~15) + 16;
      if (R.lds <= 64 * 1024) break;
    }
    if (R.lds > 64 * 1024) {
      set_error("eao_orb_create: image too wide for the pyramid kernel's LDS tile");
      return EAO_E_ARG;
    }
  }
  // k_pyr_tail: from the first level a >= 2 whose source level and itself fit LDS together (the
  // later levels are smaller: they ping-pong in the same two images); EAO_PYR_TAIL=0: per-level
  // launches throughout (A/B switch)
  {
    static const bool tail_ok = [] {
      const char* v = getenv("EAO_PYR_TAIL");
      return !(v && v[0] == '0');
    }();
    auto img = [&](int l) { return (size_t)((levels[l].w + 15) & ~15) * levels[l].h + 16; };
    tail_a = nl;
    for (int a = 2; tail_ok && a < nl; a++)
      if (img(a - 1) + img(a) <= 160 * 1024 - 64) {
        tail_a = a;
        tail_img_b = (int)((img(a - 1) + 15) & ~(size_t)15);
        tail_tab_b = (int)((tail_img_b + img(a) + 15) & ~(size_t)15);
        tail_nx = tail_ny = 0;
        for (int l = a; l < nl; l++) {
          tail_nx += levels[l].w;
          tail_ny += levels[l].h;
        }
        tail_lds = tail_tab_b + 8 * (size_t)tail_nx + 12 * (size_t)tail_ny;
        if (tail_lds > 160 * 1024 - 64) {
          tail_a = nl;
          continue;
        }
        break;
      }
  }
  {
    // FAST bands: the cells of a level row share their ROI rows
    bands.clear();
    band_w = band_h = 0;
    for (size_t c = 0; c < cells.size();) {
      // the row of cells starting at c, split into the fewest bands of <= FAST_BAND_W px,
      // with the cells shared out evenly (balanced blocks, narrow LDS rows)
      size_t row_end = c;
      while (row_end < cells.size() && cells[row_end].level == cells[c].level && cells[row_end].i == cells[c].i)
        row_end++;
      const int row_w = cells[row_end - 1].x1 - cells[c].x0;
      const size_t nrow = row_end - c;
      const size_t nb = std::min(nrow, (size_t)((row_w + FAST_BAND_W - 1) / FAST_BAND_W));
      size_t e = c + (nrow + nb - 1) / nb;
      // a band of that many cells may still exceed the limit when cell widths differ
      while (e > c + 1 && cells[e - 1].x1 - cells[c].x0 > FAST_BAND_W) e--;
      BandDev b{};
      b.level = cells[c].level;
      b.ncells = (int16_t)(e - c);
      b.x0 = cells[c].x0;
      b.x1 = cells[e - 1].x1;
      b.y0 = cells[c].y0;
      b.y1 = cells[c].y1;
      b.cell_begin = (int)c;
      band_w = std::max(band_w, b.x1 - b.x0);
      band_h = std::max(band_h, b.y1 - b.y0);
      bands.push_back(b);
      c = e;
    }
  }
  cand_stride = ((long long)cand_total + 63) & ~63LL;
  sel_stride = ((long long)sel_total + 63) & ~63LL;
  cap = sel_total;
  roi_stride = (rsmax + 3) & ~3;
  roi_rows = rhmax;
  slot_map.clear();
  for (int l = 0; l < nl; l++)
    for (int k = 0; k < levels[l].sel_cap; k++) slot_map.push_back({l, k});
  return EAO_OK;
}

int OrbEngine::init(const eao_orb_params& prm, int device) {
  int rc = plan(prm, device);
  if (rc) return rc;
  EAO_HIP_CHECK(hipSetDevice(dev));
  EAO_HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  const int B = p.max_batch;
  auto up = [&](void** d, const void* h, size_t n) -> int {
    EAO_HIP_CHECK(hipMalloc(d, std::max<size_t>(n, 16)));
    if (n) EAO_HIP_CHECK(hipMemcpy(*d, h, n, hipMemcpyHostToDevice));
    return 0;
  };
  if ((rc = up((void**)&d_levels, levels.data(), levels.size() * sizeof(LevelDev)))) return rc;
  if ((rc = up((void**)&d_cells, cells.data(), cells.size() * sizeof(CellDev)))) return rc;
  if ((rc = up((void**)&d_xofs, resize_xofs.data(), resize_xofs.size() * sizeof(int)))) return rc;
  if ((rc = up((void**)&d_ia, resize_ia.data(), resize_ia.size() * sizeof(short)))) return rc;
  if ((rc = up((void**)&d_yrows, resize_yrows.data(), resize_yrows.size() * sizeof(int)))) return rc;
  if ((rc = up((void**)&d_ib, resize_ib.data(), resize_ib.size() * sizeof(short)))) return rc;
  if ((rc = up((void**)&d_umax, umax.data(), umax.size() * sizeof(int)))) return rc;
  if ((rc = up((void**)&d_gk, gk.data(), gk.size() * sizeof(int)))) return rc;
  if ((rc = up((void**)&d_slot_map, slot_map.data(), slot_map.size() * sizeof(int2)))) return rc;
  if ((rc = up((void**)&d_bands, bands.data(), bands.size() * sizeof(BandDev)))) return rc;
  EAO_HIP_CHECK(hipMalloc(&d_pyr, std::max<long long>(pyr_bytes, 256) * B));
  EAO_HIP_CHECK(hipMalloc(&d_cand, cand_stride * sizeof(uint32_t) * B));
  EAO_HIP_CHECK(hipMalloc(&d_qbuf, 2 * cand_stride * sizeof(uint32_t) * B));
  EAO_HIP_CHECK(hipMalloc(&d_cell_cnt, cells.size() * sizeof(int) * B));
  EAO_HIP_CHECK(hipMalloc(&d_sel, sel_stride * sizeof(uint32_t) * B));
  EAO_HIP_CHECK(hipMalloc(&d_sel_cnt, p.nlevels * sizeof(int) * B));
  // single-image staging
  EAO_HIP_CHECK(hipMalloc(&d_img, ((size_t)p.width * p.height + 15) & ~(size_t)15));  // image_in copies 16 B units
  // single-image outputs in one block [count | keypoints | descriptors]: one copy back
  out_kps_off = 16;
  out_desc_off = (out_kps_off + (size_t)cap * sizeof(eao_keypoint_dev) + 15) & ~(size_t)15;
  out_bytes = out_desc_off + (size_t)cap * 32;
  EAO_HIP_CHECK(hipMalloc(&d_out_blk, out_bytes));
  d_out_cnt = (int*)d_out_blk;
  d_out_kps = (eao_keypoint_dev*)(d_out_blk + out_kps_off);
  d_out_desc = d_out_blk + out_desc_off;
  return EAO_OK;
}

OrbEngine::~OrbEngine() {
  void* ptrs[] = {d_levels, d_cells, d_xofs, d_ia, d_yrows, d_ib, d_umax, d_gk, d_slot_map,
                  d_bands, d_pyr, d_cand, d_qbuf, d_cell_cnt, d_sel, d_sel_cnt, d_img, d_out_blk};
  for (void* q : ptrs)
    if (q) (void)hipFree(q);
  if (stream) (void)hipStreamDestroy(stream);
  for (auto& e : ev)
    if (e) (void)hipEventDestroy(e);
}

// Single-image calls move their image and outputs by kernel between pinned host memory and HBM: a
// copy-engine transfer queues behind every other engine's transfers on the device (the drop-in's line
// calls and matching run beside the extraction), a kernel copy does not.
__global__ __launch_bounds__(256) void k_stage_in(const uint4* __restrict__ src, uint4* __restrict__ dst, int n16) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256) dst[i] = src[i];
}

__global__ __launch_bounds__(256) void k_orb_out(const uint8_t* __restrict__ blk, uint8_t* __restrict__ host,
                                                 int kps_off, int desc_off, int cap) {
  const int n = max(0, min(*(const int*)blk, cap));
  if (blockIdx.x == 0 && threadIdx.x == 0) *(int*)host = *(const int*)blk;
  const int nk = (n * (int)sizeof(eao_keypoint_dev) + 15) >> 4, nd = n * 2;
  const uint4* ks = (const uint4*)(blk + kps_off);
  const uint4* ds = (const uint4*)(blk + desc_off);
  uint4* kd = (uint4*)(host + kps_off);
  uint4* dd = (uint4*)(host + desc_off);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < nk + nd; i += gridDim.x * 256) {
    if (i < nk)
      kd[i] = ks[i];
    else
      dd[i - nk] = ds[i - nk];
  }
}

int OrbEngine::image_in(size_t bytes) {
  const int n16 = (int)((bytes + 15) >> 4);  // both buffers 16-aligned and rounded up to 16 B
  hipLaunchKernelGGL(k_stage_in, dim3(std::min(120, (n16 + 255) / 256)), dim3(256), 0, stream,
                     (const uint4*)stage_in.h, (uint4*)d_img, n16);
  EAO_HIP_CHECK(hipGetLastError());
  return EAO_OK;
}

int OrbEngine::outputs_out() {
  hipLaunchKernelGGL(k_orb_out, dim3(16), dim3(256), 0, stream, d_out_blk, (uint8_t*)stage_out.h, (int)out_kps_off,
                     (int)out_desc_off, cap);
  EAO_HIP_CHECK(hipGetLastError());
  return EAO_OK;
}

int OrbEngine::run(const uint8_t* d_frames, int nframes, int pitch, eao_keypoint_dev* d_kps,
                   uint8_t* d_desc, int* d_counts, int out_cap, hipStream_t s) {
  if (nframes < 1 || nframes > p.max_batch || pitch < p.width || out_cap < cap) {
    set_error("eao_orb_extract_batch_device: bad batch arguments");
    return EAO_E_ARG;
  }
  if (!s) s = stream;
  const long long fstride = (long long)pitch * p.height;
  const int nl = p.nlevels;
  if (timing) EAO_HIP_CHECK(hipEventRecord(ev[0], s));
  // pyramid: k_resize_lds (EAO_RESIZE=0: the round-4 k_resize_tile, A/B switch)
  static const int resize_lds = [] {
    const char* v = getenv("EAO_RESIZE");
    return v && v[0] == '0' ? 0 : 1;
  }();
  for (int l = 1; l < nl; l++) {
    // the small levels in one launch -- for batches: one workgroup per frame makes a single frame's
    // levels in series (22 us at 640x480, against ~13 us for its per-level launches)
    if (resize_lds && l == tail_a && nframes >= tail_min_frames) {
      hipLaunchKernelGGL(k_pyr_tail, dim3(nframes), dim3(1024), tail_lds, s, d_pyr, pyr_bytes,
                         (const LevelDev*)d_levels, tail_a, nl, tail_img_b, tail_tab_b, tail_nx, tail_ny, 1,
                         (const int*)d_xofs, (const short*)d_ia,
                         (const int*)d_yrows, (const short*)d_ib);
      break;
    }
    const LevelDev& L = levels[l];
    const LevelDev& S = levels[l - 1];
    const uint8_t* src = l == 1 ? d_frames : d_pyr + S.plane_off;
    const int spitch = l == 1 ? pitch : S.pitch;
    const long long sstride = l == 1 ? fstride : pyr_bytes;
    if (resize_lds) {
      const ResizePlan& R = resize_plan[l];
      const bool vec = l > 1 || ((uintptr_t)d_frames % 16 == 0 && pitch % 16 == 0);
      auto kr = vec ? k_resize_lds<true> : k_resize_lds<false>;
      hipLaunchKernelGGL(kr, dim3(R.tiles, nframes), dim3(R.block), R.lds, s, src, spitch, sstride,
                         d_pyr + L.plane_off, L.pitch, pyr_bytes, S.w, S.h, L.w, L.h, R.tr,
                         1. / ((double)L.h / S.h), d_xofs + L.tab_x, d_ia + 2 * L.tab_x, L.xmax,
                         d_yrows + 2 * L.tab_y, d_ib + 2 * L.tab_y);
      continue;
    }
    dim3 g(1, (L.h + RESIZE_TR - 1) / RESIZE_TR, nframes);
    hipLaunchKernelGGL(k_resize_tile, g, dim3(256), 0, s, src, spitch, sstride, d_pyr + L.plane_off,
                       L.pitch, pyr_bytes, L.w, L.h, d_xofs + L.tab_x, d_ia + 2 * L.tab_x, L.xmax,
                       d_yrows + 2 * L.tab_y, d_ib + 2 * L.tab_y);
  }
  if (timing) EAO_HIP_CHECK(hipEventRecord(ev[1], s));
  // FAST per band of cells
  {
    // 16-byte staged rows: level planes are 64-byte pitched; level 0 is the
    // caller's frame buffer
    const int vec_ok = ((uintptr_t)d_frames % 16 == 0 && pitch % 16 == 0) ? 1 : 0;
    if (band_w + 30 > FAST_RS) {
      set_error("orb: FAST band wider than the LDS row");
      return EAO_E_CAPACITY;
    }
    dim3 g((unsigned)bands.size(), nframes);
    if (band_h - 6 > 64 || band_h < 7) {  // k_fast_band emits one detection row per lane
      set_error("orb: FAST cell rows exceed one wave");
      return EAO_E_CAPACITY;
    }
    const bool narrow = band_w + 30 <= FAST_RS_NARROW;
    const int rs = narrow ? FAST_RS_NARROW : FAST_RS;
    size_t lds = (size_t)rs * (2 * band_h - 6);  // roi, kept strengths of the detection rows
    auto kf = narrow ? k_fast_band<FAST_RS_NARROW> : k_fast_band<FAST_RS>;
    // XCD-aware band order (k_fast_band): FETCH 611 -> 363 MB per 405-frame launch, time unchanged
    // (profiles/r04_ab_fast.txt); EAO_FAST_XCD=0 restores the row-major order (A/B switch)
    static const int xcd = [] {
      const char* v = getenv("EAO_FAST_XCD");
      return v && v[0] == '0' ? 0 : 1;
    }();
    hipLaunchKernelGGL(kf, g, dim3(256), lds, s,
                       d_frames, pitch, fstride, d_pyr, pyr_bytes, d_levels, d_bands, d_cells, p.ini_th_fast,
                       p.min_th_fast, d_cand, cand_stride, d_cell_cnt, (int)cells.size(), vec_ok, xcd);
  }
  if (timing) EAO_HIP_CHECK(hipEventRecord(ev[2], s));
  // quadtree distribution
  {
    dim3 g(nframes, nl);
    int need = 0;
    for (int l = 0; l < nl; l++) need = std::max(need, levels[l].nfeat + 4 * levels[l].nIni + 16);
    auto kd = need <= 256 ? k_distribute<256> : need <= 512 ? k_distribute<512> : k_distribute<1024>;
    const size_t stat = need <= 256 ? sizeof(QShared<256>) : need <= 512 ? sizeof(QShared<512>) : sizeof(QShared<1024>);
    // a few frames (the drop-in's single calls): one (level, frame) per CU at most, so each quadtree
    // takes the CU's LDS for its keys; batches keep the keys in qbuf (LDS per workgroup sets how
    // many of the 405 x 8 quadtrees are resident at once)
    static const int lds_on = [] {
      const char* v = getenv("EAO_DIST_LDS");
      return v && v[0] == '0' ? 0 : 1;
    }();
    static const int mw_on = [] {
      const char* v = getenv("EAO_DIST_MW");
      return v && v[0] == '0' ? 0 : 1;
    }();
    if (mw_on && nframes * nl <= 256) {
      // a few frames: NW waves per tree (k_distribute_mw)
      constexpr int NW = 8;
      auto km = need <= 256 ? k_distribute_mw<256, NW> : need <= 512 ? k_distribute_mw<512, NW> : k_distribute_mw<1024, NW>;
      const size_t mstat = need <= 256 ? sizeof(QSharedMW<256>) : need <= 512 ? sizeof(QSharedMW<512>) : sizeof(QSharedMW<1024>);
      const int lds_keys = lds_on ? (int)std::min<size_t>(16384, ((size_t)152 * 1024 - mstat) / 8) : 0;
      hipLaunchKernelGGL(km, g, dim3(64 * NW), (size_t)8 * lds_keys, s, d_cand, cand_stride, d_cell_cnt,
                         (int)cells.size(), d_levels, d_cells, d_qbuf, 2 * cand_stride, d_sel, sel_stride, d_sel_cnt, nl,
                         lds_keys);
    } else {
      int lds_keys = 0;
      if (lds_on && nframes * nl <= 256) lds_keys = (int)std::min<size_t>(16384, ((size_t)152 * 1024 - stat) / 8);
      hipLaunchKernelGGL(kd, g, dim3(64), (size_t)8 * lds_keys, s, d_cand, cand_stride, d_cell_cnt, (int)cells.size(),
                         d_levels, d_cells, d_qbuf, 2 * cand_stride, d_sel, sel_stride, d_sel_cnt, nl, lds_keys);
    }
  }
  if (timing) EAO_HIP_CHECK(hipEventRecord(ev[3], s));
  // orientation + blur at the pattern taps + descriptors
  {
    const int nslots = (int)slot_map.size();
    const int gx = (nslots + 3) / 4;
    hipLaunchKernelGGL(k_describe, dim3(gx * nframes), dim3(256), 0, s, d_frames, pitch, fstride, d_pyr,
                       pyr_bytes, d_levels, d_sel, sel_stride, d_sel_cnt, d_slot_map, nslots, nl, d_umax, d_gk,
                       d_kps, d_desc, d_counts, out_cap, gx);
  }
  if (timing) EAO_HIP_CHECK(hipEventRecord(ev[4], s));
  EAO_HIP_CHECK(hipGetLastError());
  return EAO_OK;
}

}  // namespace eao
