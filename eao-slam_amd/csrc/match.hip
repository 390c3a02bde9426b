// match.hip -- ORB matching on gfx950: the MI355X replacement of the Frame
// grid (reference src/Frame.cc:351-513) and ORBmatcher searches
// (src/ORBmatcher.cc:45-137, 405-520, 1328-1663).
//
// Sequential first-wins semantics are kept exactly: each
// search runs one wave per frame pair that walks the queries in reference
// order; inside a query the 64 lanes evaluate the grid window in parallel
// and reduce on the key (distance, window order), which reproduces the
// reference's strict-< scan. Assignment state lives in LDS.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <vector>

#include "common.h"
#include "match.h"

namespace eao {

constexpr int MAXK = 8192;  // keypoints per frame handled by one wave (LDS state)
constexpr int TH_HIGH = 100, TH_LOW = 50, HISTO_LENGTH = 30;  // ORBmatcher.cc:37-39

CamDev make_cam(const eao_camera& c) {
  CamDev d;
  d.fx = c.fx;
  d.fy = c.fy;
  d.cx = c.cx;
  d.cy = c.cy;
  d.minX = 0.0f;
  d.maxX = (float)c.img_w;
  d.minY = 0.0f;
  d.maxY = (float)c.img_h;
  d.invW = (float)GRID_COLS / (d.maxX - d.minX);
  d.invH = (float)GRID_ROWS / (d.maxY - d.minY);
  return d;
}

__device__ __forceinline__ int hamming256(const uint8_t* a, const uint8_t* b) {
  const uint4* pa = (const uint4*)a;
  const uint4* pb = (const uint4*)b;
  const uint4 a0 = pa[0], a1 = pa[1], b0 = pb[0], b1 = pb[1];
  return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
         __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// Frame::PosInGrid, Frame.cc:503-513
__device__ __forceinline__ int grid_cell(const CamDev& c, float x, float y) {
  const int px = (int)roundf(fmul(fsub(x, c.minX), c.invW));
  const int py = (int)roundf(fmul(fsub(y, c.minY), c.invH));
  if (px < 0 || px >= GRID_COLS || py < 0 || py >= GRID_ROWS) return -1;
  return px * GRID_ROWS + py;  // ix-major so window order is (ix, iy)
}

// AssignFeaturesToGrid (Frame.cc:351-366) as CSR; cells keep ascending index
__global__ __launch_bounds__(256) void k_grid(const eao_keypoint_dev* __restrict__ kps,
                                              const int* __restrict__ counts, int n_single,
                                              int cap, CamDev cam, int* __restrict__ gstart,
                                              int* __restrict__ gitems) {
  __shared__ int cnt[GRID_CELLS];
  __shared__ int part[256];
  const int f = blockIdx.x, t = threadIdx.x;
  const int n = counts ? min(counts[f], cap) : n_single;
  const eao_keypoint_dev* K = kps + (long long)f * cap;
  int* S = gstart + (long long)f * (GRID_CELLS + 1);
  int* I = gitems + (long long)f * cap;
  for (int i = t; i < GRID_CELLS; i += 256) cnt[i] = 0;
  __syncthreads();
  for (int i = t; i < n; i += 256) {
    const int c = grid_cell(cam, K[i].x, K[i].y);
    if (c >= 0) atomicAdd(&cnt[c], 1);
  }
  __syncthreads();
  // exclusive scan, 12 cells per thread
  const int per = GRID_CELLS / 256;
  int loc = 0;
  for (int k = 0; k < per; k++) loc += cnt[t * per + k];
  part[t] = loc;
  __syncthreads();
  if (t == 0) {
    int run = 0;
    for (int k = 0; k < 256; k++) {
      const int v = part[k];
      part[k] = run;
      run += v;
    }
  }
  __syncthreads();
  int run = part[t];
  for (int k = 0; k < per; k++) {
    const int c = t * per + k;
    const int v = cnt[c];
    S[c] = run;
    cnt[c] = run;  // becomes the fill cursor
    run += v;
  }
  if (t == 255) S[GRID_CELLS] = run;
  __syncthreads();
  for (int i = t; i < n; i += 256) {
    const int c = grid_cell(cam, K[i].x, K[i].y);
    if (c >= 0) I[atomicAdd(&cnt[c], 1)] = i;
  }
  __syncthreads();
  // restore ascending index order inside each cell (insertion sort, tiny cells)
  for (int c = t; c < GRID_CELLS; c += 256) {
    const int b = S[c], e = S[c + 1];
    for (int i = b + 1; i < e; i++) {
      const int v = I[i];
      int j = i - 1;
      while (j >= b && I[j] > v) {
        I[j + 1] = I[j];
        j--;
      }
      I[j + 1] = v;
    }
  }
}

// cv::Mat small gemm: float dot then (float)(t + c) in double (see oracle)
__device__ __forceinline__ void transform_point(const float* T, const float* P, float* out) {
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const float t = fadd(fadd(fmul(T[4 * r], P[0]), fmul(T[4 * r + 1], P[1])), fmul(T[4 * r + 2], P[2]));
    out[r] = (float)((double)t + (double)T[4 * r + 3]);
  }
}

struct Window {
  int x0, x1, y0, y1;  // cell ranges, inclusive
  bool empty;
};

// Frame::GetFeaturesInArea cell range, Frame.cc:448-473
__device__ __forceinline__ Window window_cells(const CamDev& c, float x, float y, float r) {
  Window w;
  w.empty = true;
  w.x0 = max(0, (int)floorf(fmul(fsub(fsub(x, c.minX), r), c.invW)));
  if (w.x0 >= GRID_COLS) return w;
  w.x1 = min(GRID_COLS - 1, (int)ceilf(fmul(fadd(fsub(x, c.minX), r), c.invW)));
  if (w.x1 < 0) return w;
  w.y0 = max(0, (int)floorf(fmul(fsub(fsub(y, c.minY), r), c.invH)));
  if (w.y0 >= GRID_ROWS) return w;
  w.y1 = min(GRID_ROWS - 1, (int)ceilf(fmul(fadd(fsub(y, c.minY), r), c.invH)));
  if (w.y1 < 0) return w;
  w.empty = false;
  return w;
}

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long u = __shfl_xor(v, o, 64);
    v = u < v ? u : v;
  }
  return v;
}

__device__ __forceinline__ int rot_bin(float a_last, float a_cur) {
  const float factor = 1.0f / HISTO_LENGTH;
  float rot = fsub(a_last, a_cur);
  if (rot < 0.0f) rot = fadd(rot, 360.0f);
  int bin = (int)roundf(fmul(rot, factor));
  if (bin == HISTO_LENGTH) bin = 0;
  return bin;
}

// ComputeThreeMaxima, ORBmatcher.cc:1601-1642 (run by one lane)
__device__ void three_maxima(const int* h, int& ind1, int& ind2, int& ind3) {
  int max1 = 0, max2 = 0, max3 = 0;
  ind1 = ind2 = ind3 = -1;
  for (int i = 0; i < HISTO_LENGTH; i++) {
    const int s = h[i];
    if (s > max1) {
      max3 = max2; max2 = max1; max1 = s;
      ind3 = ind2; ind2 = ind1; ind1 = i;
    } else if (s > max2) {
      max3 = max2; max2 = s;
      ind3 = ind2; ind2 = i;
    } else if (s > max3) {
      max3 = s;
      ind3 = i;
    }
  }
  if (max2 < fmul(0.1f, (float)max1)) {
    ind2 = -1;
    ind3 = -1;
  } else if (max3 < fmul(0.1f, (float)max1)) {
    ind3 = -1;
  }
}

constexpr unsigned long long KEY_NONE = ~0ull;
__device__ __forceinline__ unsigned long long make_key(int dist, int cellk, int idx) {
  return ((unsigned long long)dist << 42) | ((unsigned long long)cellk << 21) | (unsigned long long)idx;
}
__device__ __forceinline__ int key_dist(unsigned long long k) { return (int)(k >> 42); }
__device__ __forceinline__ int key_idx(unsigned long long k) { return (int)(k & 0x1fffff); }

// SearchByProjection(CurrentFrame, LastFrame, th, bMono=true), ORBmatcher.cc:1328-1470,
// in two phases. The query loop is sequential only through the first-wins
// assignment (a current keypoint taken by an earlier map point is skipped,
// Q18), and the winner of a query is the smallest key (distance, window
// order) among its untaken candidates (Q17). So:
//   1. k_motion_cand, one thread per (pair, last-frame map point): projection,
//      window and candidate scan exactly as the reference, keeping the MK
//      smallest keys with distance <= TH_HIGH (larger ones can never be
//      assigned) and their rotation bins, plus the candidate count;
//   2. k_motion_resolve, one wave per pair: walks the queries in order; the
//      lanes test the query's stored candidates against the taken flags in
//      LDS at once and the first untaken one wins. Only a query whose MK
//      stored candidates are all taken while it has more falls back to the
//      full window scan (rare).
constexpr int MK = 8;

struct MotionGeom {
  float u, v, r;
  int oct;
  bool ok;
};

// projection + radius of last-frame map point i for pair (ls -> cs)
__device__ __forceinline__ MotionGeom motion_geom(const CamDev& cam, const float* T, float th,
                                                  const eao_keypoint_dev* LK, const uint8_t* HM,
                                                  const float* MP, const float* scales, int i) {
  MotionGeom g;
  g.ok = false;
  if (!HM[i]) return g;
  float x3Dc[3];
  transform_point(T, MP + 3 * i, x3Dc);
  const float invzc = (float)(1.0 / (double)x3Dc[2]);
  if (invzc < 0) return g;
  g.u = fadd(fmul(fmul(cam.fx, x3Dc[0]), invzc), cam.cx);
  g.v = fadd(fmul(fmul(cam.fy, x3Dc[1]), invzc), cam.cy);
  if (g.u < cam.minX || g.u > cam.maxX) return g;
  if (g.v < cam.minY || g.v > cam.maxY) return g;
  g.oct = LK[i].octave;
  g.r = fmul(th, scales[g.oct]);
  g.ok = true;
  return g;
}

__global__ __launch_bounds__(256) void k_motion_cand(
    CamDev cam, const float* __restrict__ Tcw, float th, const eao_keypoint_dev* __restrict__ kps,
    const uint8_t* __restrict__ desc, const int* __restrict__ counts, int cap,
    const uint8_t* __restrict__ has_mp, const float* __restrict__ mp_pos, const uint8_t* __restrict__ mp_desc,
    const float* __restrict__ scales, const int* __restrict__ gstart, const int* __restrict__ gitems,
    unsigned long long* __restrict__ ckeys, signed char* __restrict__ cbins, int* __restrict__ ccnt) {
  const int p = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
  const int ls = p, cs = p + 1;
  if (i >= counts[ls]) return;
  const eao_keypoint_dev* LK = kps + (long long)ls * cap;
  const eao_keypoint_dev* CK = kps + (long long)cs * cap;
  const uint8_t* CD = desc + (long long)cs * cap * 32;
  const int* GS = gstart + (long long)cs * (GRID_CELLS + 1);
  const int* GI = gitems + (long long)cs * cap;
  float T[16];
  for (int k = 0; k < 16; k++) T[k] = Tcw[cs * 16 + k];
  const long long qi = (long long)p * cap + i;
  const MotionGeom g = motion_geom(cam, T, th, LK, has_mp + (long long)ls * cap, mp_pos + (long long)ls * cap * 3,
                                   scales, i);
  int n = 0;
  unsigned long long best[MK];
#pragma unroll
  for (int k = 0; k < MK; k++) best[k] = KEY_NONE;
  if (g.ok) {
    const Window w = window_cells(cam, g.u, g.v, g.r);
    if (!w.empty) {
      const int minL = g.oct - 1, maxL = g.oct + 1;
      const int ncy = w.y1 - w.y0 + 1, ncell = (w.x1 - w.x0 + 1) * ncy;
      const uint8_t* d = mp_desc + ((long long)ls * cap + i) * 32;
      const uint4* pd = (const uint4*)d;
      const uint4 d0 = pd[0], d1 = pd[1];
      for (int ck = 0; ck < ncell; ck++) {
        const int cell = (w.x0 + ck / ncy) * GRID_ROWS + w.y0 + ck % ncy;
        for (int q = GS[cell]; q < GS[cell + 1]; q++) {
          const int i2 = GI[q];
          const eao_keypoint_dev& kp = CK[i2];
          if (kp.octave < minL || kp.octave > maxL) continue;
          if (!(fabsf(fsub(kp.x, g.u)) < g.r && fabsf(fsub(kp.y, g.v)) < g.r)) continue;
          const uint4* pc = (const uint4*)(CD + 32 * (long long)i2);
          const uint4 c0 = pc[0], c1 = pc[1];
          const int dist = __popc(d0.x ^ c0.x) + __popc(d0.y ^ c0.y) + __popc(d0.z ^ c0.z) + __popc(d0.w ^ c0.w) +
                           __popc(d1.x ^ c1.x) + __popc(d1.y ^ c1.y) + __popc(d1.z ^ c1.z) + __popc(d1.w ^ c1.w);
          if (dist > TH_HIGH) continue;
          n++;
          unsigned long long key = make_key(dist, ck, i2);
#pragma unroll
          for (int k = 0; k < MK; k++) {  // sorted insertion, smallest first
            const unsigned long long lo = key < best[k] ? key : best[k];
            key = key < best[k] ? best[k] : key;
            best[k] = lo;
          }
        }
      }
    }
  }
  ccnt[qi] = n;
  const int nk = min(n, MK);
  for (int k = 0; k < nk; k++) {
    ckeys[qi * MK + k] = best[k];
    cbins[qi * MK + k] = (signed char)rot_bin(LK[i].angle, CK[key_idx(best[k])].angle);
  }
}

// k_motion_cand with one wave per query (the latency form, few pairs: a single-call search has
// ~1000 queries, 4 workgroups of the thread-per-query form): the lanes share the query's window
// cells, each keeps its MK smallest keys, and the wave merges them by MK wave minima (keys are
// unique: the index is in them). Same outputs as k_motion_cand.
__global__ __launch_bounds__(256) void k_motion_cand_wave(
    CamDev cam, const float* __restrict__ Tcw, float th, const eao_keypoint_dev* __restrict__ kps,
    const uint8_t* __restrict__ desc, const int* __restrict__ counts, int cap,
    const uint8_t* __restrict__ has_mp, const float* __restrict__ mp_pos, const uint8_t* __restrict__ mp_desc,
    const float* __restrict__ scales, const int* __restrict__ gstart, const int* __restrict__ gitems,
    unsigned long long* __restrict__ ckeys, signed char* __restrict__ cbins, int* __restrict__ ccnt) {
  const int p = blockIdx.y, lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ls = p, cs = p + 1;
  if (i >= counts[ls]) return;  // the whole wave
  const eao_keypoint_dev* LK = kps + (long long)ls * cap;
  const eao_keypoint_dev* CK = kps + (long long)cs * cap;
  const uint8_t* CD = desc + (long long)cs * cap * 32;
  const int* GS = gstart + (long long)cs * (GRID_CELLS + 1);
  const int* GI = gitems + (long long)cs * cap;
  float T[16];
  for (int k = 0; k < 16; k++) T[k] = Tcw[cs * 16 + k];
  const long long qi = (long long)p * cap + i;
  const MotionGeom g = motion_geom(cam, T, th, LK, has_mp + (long long)ls * cap, mp_pos + (long long)ls * cap * 3,
                                   scales, i);
  int n = 0;
  unsigned long long best[MK];
#pragma unroll
  for (int k = 0; k < MK; k++) best[k] = KEY_NONE;
  if (g.ok) {
    const Window w = window_cells(cam, g.u, g.v, g.r);
    if (!w.empty) {
      const int minL = g.oct - 1, maxL = g.oct + 1;
      const int ncy = w.y1 - w.y0 + 1, ncell = (w.x1 - w.x0 + 1) * ncy;
      const uint4* pd = (const uint4*)(mp_desc + ((long long)ls * cap + i) * 32);
      const uint4 d0 = pd[0], d1 = pd[1];
      for (int ck = lane; ck < ncell; ck += 64) {
        const int cell = (w.x0 + ck / ncy) * GRID_ROWS + w.y0 + ck % ncy;
        for (int q = GS[cell]; q < GS[cell + 1]; q++) {
          const int i2 = GI[q];
          const eao_keypoint_dev& kp = CK[i2];
          if (kp.octave < minL || kp.octave > maxL) continue;
          if (!(fabsf(fsub(kp.x, g.u)) < g.r && fabsf(fsub(kp.y, g.v)) < g.r)) continue;
          const uint4* pc = (const uint4*)(CD + 32 * (long long)i2);
          const uint4 c0 = pc[0], c1 = pc[1];
          const int dist = __popc(d0.x ^ c0.x) + __popc(d0.y ^ c0.y) + __popc(d0.z ^ c0.z) + __popc(d0.w ^ c0.w) +
                           __popc(d1.x ^ c1.x) + __popc(d1.y ^ c1.y) + __popc(d1.z ^ c1.z) + __popc(d1.w ^ c1.w);
          if (dist > TH_HIGH) continue;
          n++;
          unsigned long long key = make_key(dist, ck, i2);
#pragma unroll
          for (int k = 0; k < MK; k++) {  // sorted insertion, smallest first
            const unsigned long long lo = key < best[k] ? key : best[k];
            key = key < best[k] ? best[k] : key;
            best[k] = lo;
          }
        }
      }
    }
  }
  n = wave_sum(n);
  const int nk = min(n, MK);
  for (int k = 0; k < nk; k++) {  // the wave's k-th smallest: its holder pops it
    const unsigned long long m = wave_min_u64(best[0]);
    if (best[0] == m) {
#pragma unroll
      for (int j = 0; j < MK - 1; j++) best[j] = best[j + 1];
      best[MK - 1] = KEY_NONE;
    }
    if (lane == 0) {
      ckeys[qi * MK + k] = m;
      cbins[qi * MK + k] = (signed char)rot_bin(LK[i].angle, CK[key_idx(m)].angle);
    }
  }
  if (lane == 0) ccnt[qi] = n;
}

// the full window scan of query i against the untaken current keypoints (its stored candidates are
// all taken and it has more): the whole wave, the smallest (distance, window order, index) key
__device__ __forceinline__ void motion_rescan(const CamDev& cam, const float* __restrict__ Tcw, float th,
                                              const eao_keypoint_dev* LK, const eao_keypoint_dev* CK,
                                              const uint8_t* CD, const int* GS, const int* GI,
                                              const uint8_t* __restrict__ has_mp, const float* __restrict__ mp_pos,
                                              const uint8_t* __restrict__ mp_desc, const float* __restrict__ scales,
                                              const int* match, int ls, int cs, int cap, int i, int& i2, int& bin) {
  const int lane = threadIdx.x & 63;
  float T[16];
  for (int k = 0; k < 16; k++) T[k] = Tcw[cs * 16 + k];
  const MotionGeom g = motion_geom(cam, T, th, LK, has_mp + (long long)ls * cap, mp_pos + (long long)ls * cap * 3,
                                   scales, i);
  const Window w = window_cells(cam, g.u, g.v, g.r);
  const int minL = g.oct - 1, maxL = g.oct + 1;
  const int ncy = w.y1 - w.y0 + 1, ncell = (w.x1 - w.x0 + 1) * ncy;
  const uint8_t* d = mp_desc + ((long long)ls * cap + i) * 32;
  unsigned long long best = KEY_NONE;
  for (int ck = lane; ck < ncell; ck += 64) {
    const int cell = (w.x0 + ck / ncy) * GRID_ROWS + w.y0 + ck % ncy;
    for (int q = GS[cell]; q < GS[cell + 1]; q++) {
      const int c2 = GI[q];
      const eao_keypoint_dev& kp = CK[c2];
      if (kp.octave < minL || kp.octave > maxL) continue;
      if (!(fabsf(fsub(kp.x, g.u)) < g.r && fabsf(fsub(kp.y, g.v)) < g.r)) continue;
      if (match[c2] >= 0) continue;
      const unsigned long long k2 = make_key(hamming256(d, CD + 32 * (long long)c2), ck, c2);
      best = k2 < best ? k2 : best;
    }
  }
  best = wave_min_u64(best);
  if (best != KEY_NONE && key_dist(best) <= TH_HIGH) {
    i2 = key_idx(best);
    bin = rot_bin(LK[i].angle, CK[i2].angle);
  }
}

__global__ __launch_bounds__(64) void k_motion_resolve(
    CamDev cam, const float* __restrict__ Tcw, float th, int check_ori, const eao_keypoint_dev* __restrict__ kps,
    const uint8_t* __restrict__ desc, const int* __restrict__ counts, int cap, const uint8_t* __restrict__ has_mp,
    const float* __restrict__ mp_pos, const uint8_t* __restrict__ mp_desc, const float* __restrict__ scales,
    const int* __restrict__ gstart, const int* __restrict__ gitems, const unsigned long long* __restrict__ ckeys,
    const signed char* __restrict__ cbins, const int* __restrict__ ccnt, int* __restrict__ cur_match,
    int* __restrict__ nmatches_out) {
  __shared__ int match[MAXK];
  __shared__ signed char bins[MAXK];
  __shared__ int hist[HISTO_LENGTH];
  __shared__ unsigned long long kb[64 * MK];
  __shared__ signed char bb[64 * MK];
  __shared__ int nb[64];
  __shared__ int claim[MAXK];  // the lowest lane proposing a current keypoint in a round (64: none)
  const int p = blockIdx.x, lane = threadIdx.x;
  const int ls = p, cs = p + 1;
  const int n_last = counts[ls], n_cur = counts[cs];
  const eao_keypoint_dev* LK = kps + (long long)ls * cap;
  const eao_keypoint_dev* CK = kps + (long long)cs * cap;
  const uint8_t* CD = desc + (long long)cs * cap * 32;
  const int* GS = gstart + (long long)cs * (GRID_CELLS + 1);
  const int* GI = gitems + (long long)cs * cap;
  for (int i = lane; i < n_cur; i += 64) {
    match[i] = -1;
    bins[i] = -1;
    claim[i] = 64;
  }
  int nmatches = 0;
  for (int base = 0; base < n_last; base += 64) {
    const int nq = min(64, n_last - base);
    const long long q0 = (long long)p * cap + base;
    const int myn = lane < nq ? ccnt[q0 + lane] : 0;
    nb[lane] = myn;
    __syncthreads();
    for (int k = lane; k < nq * MK; k += 64) {
      const int qq = k / MK, c = k - qq * MK;
      if (c < min(nb[qq], MK)) {
        kb[k] = ckeys[q0 * MK + k];
        bb[k] = cbins[q0 * MK + k];
      }
    }
    __syncthreads();
    // The block's queries in rounds (the first-wins order kept): every undone lane proposes its
    // first stored candidate not yet taken; the lanes commit up to the first one whose proposal an
    // earlier undone lane of the round also makes (claims by LDS atomicMin: that lane re-proposes
    // next round, after its predecessors are in) or that needs the window rescan (run right after
    // the commit, by the whole wave). A committed lane's proposal is the sequential walk's choice:
    // its skipped candidates were taken before the round, and no earlier lane of the round takes it.
    const int nk = min(myn, MK);
    int pos = 0;
    bool done = lane >= nq || myn == 0;
    while (true) {
      if (!ballot(!done)) break;
      int c = -1;
      bool resc = false;
      if (!done) {
        while (pos < nk && match[key_idx(kb[lane * MK + pos])] >= 0) pos++;
        if (pos < nk)
          c = key_idx(kb[lane * MK + pos]);
        else
          resc = myn > MK;  // every stored candidate taken and more exist: the rescan
      }
      if (c >= 0) atomicMin(&claim[c], lane);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      const bool conflict = c >= 0 && claim[c] != lane;
      const uint64_t stop = ballot(!done && (conflict || resc));
      const int f = stop ? __builtin_ctzll(stop) : 64;
      if (c >= 0 && !conflict) claim[c] = 64;  // the claim's owner resets it (after every lane read it)
      const bool commit = !done && lane < f;
      if (commit && c >= 0) {
        match[c] = base + lane;
        bins[c] = bb[lane * MK + pos];
      }
      nmatches += popc64(ballot(commit && c >= 0));
      done = done || commit;
      if (f < 64 && __builtin_amdgcn_readlane((int)resc, f)) {
        __syncthreads();  // the commits visible to every lane of the rescan
        int i2 = -1, bin = -1;
        motion_rescan(cam, Tcw, th, LK, CK, CD, GS, GI, has_mp, mp_pos, mp_desc, scales, match, ls, cs, cap,
                      base + f, i2, bin);
        if (i2 >= 0) {
          if (lane == 0) {
            match[i2] = base + f;
            bins[i2] = (signed char)bin;
          }
          nmatches++;
        }
        if (lane == f) done = true;
      }
      __syncthreads();
    }
    __syncthreads();
  }
  if (check_ori) {
    for (int b = lane; b < HISTO_LENGTH; b += 64) hist[b] = 0;
    __syncthreads();
    for (int i2 = lane; i2 < n_cur; i2 += 64)
      if (match[i2] >= 0) atomicAdd(&hist[bins[i2]], 1);
    __syncthreads();
    int ind1, ind2, ind3;
    three_maxima(hist, ind1, ind2, ind3);
    int removed = 0;
    for (int i2 = lane; i2 < n_cur; i2 += 64) {
      if (match[i2] >= 0) {
        const int b = bins[i2];
        if (b != ind1 && b != ind2 && b != ind3) {
          match[i2] = -1;
          removed++;
        }
      }
    }
    nmatches -= wave_sum(removed);
    __syncthreads();
  }
  int* out = cur_match + (long long)cs * cap;
  for (int i2 = lane; i2 < n_cur; i2 += 64) out[i2] = match[i2];
  if (lane == 0) nmatches_out[cs] = nmatches;
}

// Frame::isInFrustum + MapPoint::PredictScale (see oracle/match_ref.cpp)
__global__ __launch_bounds__(256) void k_frustum(CamDev cam, const float* __restrict__ T, int n,
                                                 const float* __restrict__ pos,
                                                 const float* __restrict__ nrm,
                                                 const float* __restrict__ mind,
                                                 const float* __restrict__ maxd, float vclim,
                                                 float logsf, uint8_t* __restrict__ in_view,
                                                 float* __restrict__ proj, int* __restrict__ level,
                                                 float* __restrict__ vcos) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float Ow[3];
#pragma unroll
  for (int c = 0; c < 3; c++) {
    double s = (double)T[c] * (double)T[3];
    s = __dadd_rn(s, (double)T[4 + c] * (double)T[7]);
    s = __dadd_rn(s, (double)T[8 + c] * (double)T[11]);
    Ow[c] = (float)(s * -1.0);
  }
  in_view[i] = 0;
  const float* P = pos + 3 * i;
  float Pc[3];
  transform_point(T, P, Pc);
  if (Pc[2] < 0.0f) return;
  const float invz = fdiv(1.0f, Pc[2]);
  const float u = fadd(fmul(fmul(cam.fx, Pc[0]), invz), cam.cx);
  const float v = fadd(fmul(fmul(cam.fy, Pc[1]), invz), cam.cy);
  if (u < cam.minX || u > cam.maxX) return;
  if (v < cam.minY || v > cam.maxY) return;
  const float maxDistance = fmul(1.2f, maxd[i]);
  const float minDistance = fmul(0.8f, mind[i]);
  const float PO[3] = {fsub(P[0], Ow[0]), fsub(P[1], Ow[1]), fsub(P[2], Ow[2])};
  double s = 0;
  for (int k = 0; k < 3; k++) s = __dadd_rn(s, __dmul_rn((double)PO[k], (double)PO[k]));
  const float dist = (float)sqrt(s);
  if (dist < minDistance || dist > maxDistance) return;
  double dot = 0;
  for (int k = 0; k < 3; k++) dot = __dadd_rn(dot, __dmul_rn((double)PO[k], (double)nrm[3 * i + k]));
  const float viewCos = (float)(dot / (double)dist);
  if (viewCos < vclim) return;
  const float ratio = fdiv(maxd[i], dist);
  const int lvl = (int)ceilf(fdiv((float)log((double)ratio), logsf));
  in_view[i] = 1;
  proj[2 * i] = u;
  proj[2 * i + 1] = v;
  level[i] = lvl;
  vcos[i] = viewCos;
}

// ---- candidate phases of the single-frame searches (local map, relocalisation,
// initialisation): one thread per query scans its window exactly as the sequential
// search does and keeps the MK smallest keys (distance, window order, index) among the
// candidates that no later assignment can add back, plus the candidate count. The
// sequential phase then decides a query from its stored keys when they settle it
// (enough of them still pass the assignment-dependent test, or the query has no more
// candidates) and falls back to the full window scan otherwise -- the same answer.
// a batch of independent searches: search f reads its queries at f * qs and its
// frame at f * cs (grid slot f), with per-search counts; a single call passes
// null counts (the scalar ones apply) and zero strides
struct BatchDims {
  const int* nq;
  const int* nc;
  int qs, cs;
};
template <typename T>
__device__ __forceinline__ T* at_slot(T* p, int f, long long stride) {
  return p ? p + f * stride : p;
}

__device__ __forceinline__ void keep_smallest(unsigned long long (&best)[MK], unsigned long long key) {
#pragma unroll
  for (int k = 0; k < MK; k++) {  // sorted insertion, smallest first
    const unsigned long long lo = key < best[k] ? key : best[k];
    key = key < best[k] ? best[k] : key;
    best[k] = lo;
  }
}
__device__ __forceinline__ void store_keys(unsigned long long* __restrict__ ckeys, int* __restrict__ ccnt, int q,
                                           int n, const unsigned long long (&best)[MK]) {
  ccnt[q] = n;
  for (int k = 0; k < min(n, MK); k++) ckeys[(long long)q * MK + k] = best[k];
}

// SearchByProjection(Frame&, vector<MapPoint*>, th) candidates, ORBmatcher.cc:45-114
__global__ __launch_bounds__(256) void k_local_cand(
    CamDev cam, float th, int n_mp, const uint8_t* __restrict__ inview, const float* __restrict__ proj,
    const int* __restrict__ level, const float* __restrict__ vcos, const uint8_t* __restrict__ mdesc,
    const eao_keypoint_dev* __restrict__ CK, const uint8_t* __restrict__ CD, const int* __restrict__ pre, int nlevels,
    const float* __restrict__ scales, const int* __restrict__ GS, const int* __restrict__ GI,
    unsigned long long* __restrict__ ckeys, int* __restrict__ ccnt, BatchDims bd) {
  const int f = blockIdx.y, iMP = blockIdx.x * blockDim.x + threadIdx.x;
  if (bd.nq) n_mp = min(bd.nq[f], bd.qs);
  if (iMP >= n_mp) return;
  inview = at_slot(inview, f, bd.qs);
  proj = at_slot(proj, f, 2LL * bd.qs);
  level = at_slot(level, f, bd.qs);
  vcos = at_slot(vcos, f, bd.qs);
  mdesc = at_slot(mdesc, f, 32LL * bd.qs);
  CK = at_slot(CK, f, bd.cs);
  CD = at_slot(CD, f, 32LL * bd.cs);
  pre = at_slot(pre, f, bd.cs);
  GS = at_slot(GS, f, GRID_CELLS + 1);
  GI = at_slot(GI, f, bd.cs);
  ckeys = at_slot(ckeys, f, (long long)MK * bd.qs);
  ccnt = at_slot(ccnt, f, bd.qs);
  unsigned long long best[MK];
#pragma unroll
  for (int k = 0; k < MK; k++) best[k] = KEY_NONE;
  int n = 0;
  if (inview[iMP]) {
    const int L = min(max(level[iMP], 0), nlevels - 1);  // Q13 clamp
    float r = vcos[iMP] > 0.998f ? 2.5f : 4.0f;
    if (th != 1.0f) r = fmul(r, th);
    const float rr = fmul(r, scales[L]);
    const float x = proj[2 * iMP], y = proj[2 * iMP + 1];
    const Window w = window_cells(cam, x, y, rr);
    if (!w.empty) {
      const int minL = L - 1, maxL = L;
      const bool checkL = (minL > 0) || (maxL >= 0);
      const int ncy = w.y1 - w.y0 + 1, ncell = (w.x1 - w.x0 + 1) * ncy;
      const uint8_t* d = mdesc + 32 * (long long)iMP;
      for (int ck = 0; ck < ncell; ck++) {
        const int cell = (w.x0 + ck / ncy) * GRID_ROWS + w.y0 + ck % ncy;
        for (int q = GS[cell]; q < GS[cell + 1]; q++) {
          const int idx = GI[q];
          const eao_keypoint_dev& kp = CK[idx];
          if (checkL) {
            if (kp.octave < minL) continue;
            if (maxL >= 0 && kp.octave > maxL) continue;
          }
          if (!(fabsf(fsub(kp.x, x)) < rr && fabsf(fsub(kp.y, y)) < rr)) continue;
          if (pre && pre[idx] >= 0) continue;  // taken before the search starts
          n++;
          keep_smallest(best, make_key(hamming256(d, CD + 32 * (long long)idx), ck, idx));
        }
      }
    }
  }
  store_keys(ckeys, ccnt, iMP, n, best);
}

// SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist) candidates,
// ORBmatcher.cc:1472-1560: the query geometry (projection without a depth test,
// distance gate, PredictScale clamped -- Q13) into geo[], then the window scan
__global__ __launch_bounds__(256) void k_keyframe_cand(
    CamDev cam, const float* __restrict__ Tg, float th, int n_kf, const uint8_t* __restrict__ valid,
    const float* __restrict__ pos, const uint8_t* __restrict__ mdesc, const float* __restrict__ mind,
    const float* __restrict__ maxd, float logsf, const eao_keypoint_dev* __restrict__ CK,
    const uint8_t* __restrict__ CD, const int* __restrict__ pre, int nlevels, const float* __restrict__ scales,
    const int* __restrict__ GS, const int* __restrict__ GI, float4* __restrict__ geo,
    unsigned long long* __restrict__ ckeys, int* __restrict__ ccnt, BatchDims bd) {
  const int f = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
  if (bd.nq) n_kf = min(bd.nq[f], bd.qs);
  if (i >= n_kf) return;
  Tg = at_slot(Tg, f, bd.qs ? 16 : 0);
  valid = at_slot(valid, f, bd.qs);
  pos = at_slot(pos, f, 3LL * bd.qs);
  mdesc = at_slot(mdesc, f, 32LL * bd.qs);
  mind = at_slot(mind, f, bd.qs);
  maxd = at_slot(maxd, f, bd.qs);
  CK = at_slot(CK, f, bd.cs);
  CD = at_slot(CD, f, 32LL * bd.cs);
  pre = at_slot(pre, f, bd.cs);
  GS = at_slot(GS, f, GRID_CELLS + 1);
  GI = at_slot(GI, f, bd.cs);
  geo = at_slot(geo, f, bd.qs);
  ckeys = at_slot(ckeys, f, (long long)MK * bd.qs);
  ccnt = at_slot(ccnt, f, bd.qs);
  float T[16];
  for (int k = 0; k < 16; k++) T[k] = Tg[k];
  float Ow[3];  // -Rcw^T tcw: transposed gemm operand, double accumulation (see k_frustum)
#pragma unroll
  for (int c = 0; c < 3; c++) {
    double s = (double)T[c] * (double)T[3];
    s = __dadd_rn(s, (double)T[4 + c] * (double)T[7]);
    s = __dadd_rn(s, (double)T[8 + c] * (double)T[11]);
    Ow[c] = (float)(s * -1.0);
  }
  float4 g = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
  if (valid[i]) {
    const float* P = pos + 3 * i;
    float Pc[3];
    transform_point(T, P, Pc);
    const float invzc = (float)(1.0 / (double)Pc[2]);
    const float u = fadd(fmul(fmul(cam.fx, Pc[0]), invzc), cam.cx);
    const float v = fadd(fmul(fmul(cam.fy, Pc[1]), invzc), cam.cy);
    const float PO[3] = {fsub(P[0], Ow[0]), fsub(P[1], Ow[1]), fsub(P[2], Ow[2])};
    double s = 0;
    for (int k = 0; k < 3; k++) s = __dadd_rn(s, __dmul_rn((double)PO[k], (double)PO[k]));
    const float dist3D = (float)sqrt(s);
    const float maxDistance = fmul(1.2f, maxd[i]);
    const float minDistance = fmul(0.8f, mind[i]);
    if (!(u < cam.minX || u > cam.maxX || v < cam.minY || v > cam.maxY || dist3D < minDistance ||
          dist3D > maxDistance)) {
      const float ratio = fdiv(maxd[i], dist3D);
      int lvl = (int)ceilf(fdiv((float)log((double)ratio), logsf));
      lvl = min(max(lvl, 0), nlevels - 1);
      g = make_float4(u, v, fmul(th, scales[lvl]), __int_as_float(lvl));
    }
  }
  geo[i] = g;
  unsigned long long best[MK];
#pragma unroll
  for (int k = 0; k < MK; k++) best[k] = KEY_NONE;
  int n = 0;
  const int lvl = __float_as_int(g.w);
  if (lvl >= 0) {
    const float u = g.x, v = g.y, r = g.z;
    const Window w = window_cells(cam, u, v, r);
    if (!w.empty) {
      const int minL = lvl - 1, maxL = lvl + 1;
      const int ncy = w.y1 - w.y0 + 1, ncell = (w.x1 - w.x0 + 1) * ncy;
      const uint8_t* d = mdesc + 32 * (long long)i;
      for (int ck = 0; ck < ncell; ck++) {
        const int cell = (w.x0 + ck / ncy) * GRID_ROWS + w.y0 + ck % ncy;
        for (int q = GS[cell]; q < GS[cell + 1]; q++) {
          const int i2 = GI[q];
          const eao_keypoint_dev& kp = CK[i2];
          if (minL > 0 && kp.octave < minL) continue;  // bCheckLevels: minL > 0 || maxL >= 0
          if (kp.octave > maxL) continue;
          if (!(fabsf(fsub(kp.x, u)) < r && fabsf(fsub(kp.y, v)) < r)) continue;
          if (pre && pre[i2] >= 0) continue;
          n++;
          keep_smallest(best, make_key(hamming256(d, CD + 32 * (long long)i2), ck, i2));
        }
      }
    }
  }
  store_keys(ckeys, ccnt, i, n, best);
}

// SearchForInitialization candidates, ORBmatcher.cc:405-450: level-0 keypoints of frame 1
// in a square window around their previous matches (the vMatchedDistance test is the
// assignment-dependent part, applied in k_match_init)
__global__ __launch_bounds__(256) void k_init_cand(
    CamDev cam, int n1, const eao_keypoint_dev* __restrict__ K1, const uint8_t* __restrict__ D1,
    const eao_keypoint_dev* __restrict__ K2, const uint8_t* __restrict__ D2, const float* __restrict__ prev, int window,
    const int* __restrict__ GS, const int* __restrict__ GI, unsigned long long* __restrict__ ckeys,
    int* __restrict__ ccnt, BatchDims bd) {
  const int f = blockIdx.y, i1 = blockIdx.x * blockDim.x + threadIdx.x;
  if (bd.nq) n1 = min(bd.nq[f], bd.qs);
  if (i1 >= n1) return;
  K1 = at_slot(K1, f, bd.qs);
  D1 = at_slot(D1, f, 32LL * bd.qs);
  prev = at_slot(prev, f, 2LL * bd.qs);
  K2 = at_slot(K2, f, bd.cs);
  D2 = at_slot(D2, f, 32LL * bd.cs);
  GS = at_slot(GS, f, GRID_CELLS + 1);
  GI = at_slot(GI, f, bd.cs);
  ckeys = at_slot(ckeys, f, (long long)MK * bd.qs);
  ccnt = at_slot(ccnt, f, bd.qs);
  unsigned long long best[MK];
#pragma unroll
  for (int k = 0; k < MK; k++) best[k] = KEY_NONE;
  int n = 0;
  if (K1[i1].octave <= 0) {
    const float r = (float)window;
    const float x = prev[2 * i1], y = prev[2 * i1 + 1];
    const Window w = window_cells(cam, x, y, r);
    if (!w.empty) {
      const int ncy = w.y1 - w.y0 + 1, ncell = (w.x1 - w.x0 + 1) * ncy;
      const uint8_t* d1 = D1 + 32 * (long long)i1;
      for (int ck = 0; ck < ncell; ck++) {
        const int cell = (w.x0 + ck / ncy) * GRID_ROWS + w.y0 + ck % ncy;
        for (int q = GS[cell]; q < GS[cell + 1]; q++) {
          const int i2 = GI[q];
          const eao_keypoint_dev& kp = K2[i2];
          if (kp.octave < 0 || kp.octave > 0) continue;
          if (!(fabsf(fsub(kp.x, x)) < r && fabsf(fsub(kp.y, y)) < r)) continue;
          n++;
          keep_smallest(best, make_key(hamming256(d1, D2 + 32 * (long long)i2), ck, i2));
        }
      }
    }
  }
  store_keys(ckeys, ccnt, i1, n, best);
}

// stored keys of queries [base, base + nq) into LDS (kb: MK per query, nb: counts)
__device__ __forceinline__ void stage_keys(const unsigned long long* __restrict__ ckeys, const int* __restrict__ ccnt,
                                           int base, int nq, unsigned long long* kb, int* nb) {
  const int lane = threadIdx.x;
  __syncthreads();
  nb[lane] = lane < nq ? ccnt[base + lane] : 0;
  __syncthreads();
  for (int k = lane; k < nq * MK; k += 64) {
    const int qq = k / MK, c = k - qq * MK;
    if (c < min(nb[qq], MK)) kb[k] = ckeys[(long long)base * MK + k];
  }
  __syncthreads();
}

// SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist), ORBmatcher.cc:1472-1599
// (relocalisation, Tracking.cc:2295,2309). One wave. Phase 1 is lane-parallel: each lane
// projects its map points (no depth test, as :1501-1506), applies the distance gate and
// PredictScale (clamped, Q13) and leaves (u, v, radius, level) in geo[]. Phase 2 walks the
// map points in order with the first-wins assignment (Q17/Q18) like k_motion_resolve.
__global__ __launch_bounds__(64) void k_match_keyframe(
    CamDev cam, const float* __restrict__ Tg, float th, int orb_dist, int check_ori, int n_kf,
    const eao_keypoint_dev* __restrict__ KK, const uint8_t* __restrict__ valid,
    const float* __restrict__ pos, const uint8_t* __restrict__ mdesc,
    const float* __restrict__ mind, const float* __restrict__ maxd, float logsf, int n_cur,
    const eao_keypoint_dev* __restrict__ CK, const uint8_t* __restrict__ CD,
    const int* __restrict__ pre, int nlevels, const float* __restrict__ scales,
    const int* __restrict__ GS, const int* __restrict__ GI, const float4* __restrict__ geo,
    const unsigned long long* __restrict__ ckeys, const int* __restrict__ ccnt,
    int* __restrict__ out, int* __restrict__ nmatch_out, BatchDims bd) {
  __shared__ int match[MAXK];
  __shared__ signed char bins[MAXK];
  __shared__ int hist[HISTO_LENGTH];
  __shared__ unsigned long long kb[64 * MK];
  __shared__ int nb[64];
  const int lane = threadIdx.x, f = blockIdx.x;
  if (bd.nq) {
    n_kf = min(bd.nq[f], bd.qs);
    n_cur = min(bd.nc[f], bd.cs);
  }
  KK = at_slot(KK, f, bd.qs);
  mdesc = at_slot(mdesc, f, 32LL * bd.qs);
  geo = at_slot(geo, f, bd.qs);
  CK = at_slot(CK, f, bd.cs);
  CD = at_slot(CD, f, 32LL * bd.cs);
  pre = at_slot(pre, f, bd.cs);
  GS = at_slot(GS, f, GRID_CELLS + 1);
  GI = at_slot(GI, f, bd.cs);
  ckeys = at_slot(ckeys, f, (long long)MK * bd.qs);
  ccnt = at_slot(ccnt, f, bd.qs);
  out = at_slot(out, f, bd.cs);
  nmatch_out += f;
  for (int i = lane; i < n_cur; i += 64) {
    match[i] = pre ? pre[i] : -1;
    bins[i] = -1;
  }
  int nmatches = 0;
  for (int i = 0; i < n_kf; i++) {
    if ((i & 63) == 0) stage_keys(ckeys, ccnt, i, min(64, n_kf - i), kb, nb);
    const int n = nb[i & 63];
    if (n == 0) continue;  // not projected into the frame, or no candidate
    // the smallest stored key whose keypoint is still free is the search's answer;
    // only when every stored one is taken and the query has more candidates does the
    // window have to be scanned again
    const int nk = min(n, MK);
    const unsigned long long sk = lane < nk ? kb[(i & 63) * MK + lane] : KEY_NONE;
    const uint64_t fm = ballot(lane < nk && match[key_idx(sk)] < 0);
    unsigned long long best = KEY_NONE;
    if (fm) {
      const int l = __builtin_ctzll(fm);
      best = (unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)sk, l) |
             ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(sk >> 32), l) << 32);
    } else if (n > MK) {
    const float4 g = geo[i];
    const int lvl = __float_as_int(g.w);
    const float u = g.x, v = g.y, r = g.z;
    const Window w = window_cells(cam, u, v, r);
    const int minL = lvl - 1, maxL = lvl + 1;
    const int ncy = w.y1 - w.y0 + 1, ncell = (w.x1 - w.x0 + 1) * ncy;
    const uint8_t* d = mdesc + 32 * (long long)i;
    for (int ck = lane; ck < ncell; ck += 64) {
      const int ix = w.x0 + ck / ncy, iy = w.y0 + ck % ncy;
      const int cell = ix * GRID_ROWS + iy;
      for (int q = GS[cell]; q < GS[cell + 1]; q++) {
        const int i2 = GI[q];
        const eao_keypoint_dev& kp = CK[i2];
        if (minL > 0 && kp.octave < minL) continue;  // bCheckLevels: minL > 0 || maxL >= 0
        if (kp.octave > maxL) continue;
        if (!(fabsf(fsub(kp.x, u)) < r && fabsf(fsub(kp.y, v)) < r)) continue;
        if (match[i2] >= 0) continue;  // CurrentFrame.mvpMapPoints[i2]
        const int dist = hamming256(d, CD + 32 * (long long)i2);
        const unsigned long long key = make_key(dist, ck, i2);
        best = key < best ? key : best;
      }
    }
    best = wave_min_u64(best);
    }
    if (best != KEY_NONE && key_dist(best) <= orb_dist) {
      const int i2 = key_idx(best);
      if (lane == 0) {
        match[i2] = i;
        if (check_ori) bins[i2] = (signed char)rot_bin(KK[i].angle, CK[i2].angle);
      }
      nmatches++;
    }
    __syncthreads();
  }
  if (check_ori) {
    for (int b = lane; b < HISTO_LENGTH; b += 64) hist[b] = 0;
    __syncthreads();
    for (int i2 = lane; i2 < n_cur; i2 += 64)
      if (bins[i2] >= 0) atomicAdd(&hist[bins[i2]], 1);
    __syncthreads();
    int ind1, ind2, ind3;
    three_maxima(hist, ind1, ind2, ind3);
    int removed = 0;
    for (int i2 = lane; i2 < n_cur; i2 += 64) {
      const int b = bins[i2];
      if (b >= 0 && b != ind1 && b != ind2 && b != ind3) {
        match[i2] = -1;
        removed++;
      }
    }
    nmatches -= wave_sum(removed);
    __syncthreads();
  }
  for (int i2 = lane; i2 < n_cur; i2 += 64) out[i2] = match[i2];
  if (lane == 0) *nmatch_out = nmatches;
}

// SearchByProjection(Frame&, vector<MapPoint*>, th), ORBmatcher.cc:45-129
__global__ __launch_bounds__(64) void k_match_local(
    CamDev cam, float th, float nnratio, int n_mp, const uint8_t* __restrict__ inview,
    const float* __restrict__ proj,
    const int* __restrict__ level, const float* __restrict__ vcos,
    const uint8_t* __restrict__ mdesc, int n_cur, const eao_keypoint_dev* __restrict__ CK,
    const uint8_t* __restrict__ CD, const int* __restrict__ pre, int nlevels,
    const float* __restrict__ scales, const int* __restrict__ GS, const int* __restrict__ GI,
    const unsigned long long* __restrict__ ckeys, const int* __restrict__ ccnt, int* __restrict__ out,
    int* __restrict__ nmatch_out, BatchDims bd) {
  __shared__ int match[MAXK];
  __shared__ unsigned long long kb[64 * MK];
  __shared__ int nb[64];
  const int lane = threadIdx.x, f = blockIdx.x;
  if (bd.nq) {
    n_mp = min(bd.nq[f], bd.qs);
    n_cur = min(bd.nc[f], bd.cs);
  }
  proj = at_slot(proj, f, 2LL * bd.qs);
  level = at_slot(level, f, bd.qs);
  vcos = at_slot(vcos, f, bd.qs);
  mdesc = at_slot(mdesc, f, 32LL * bd.qs);
  CK = at_slot(CK, f, bd.cs);
  CD = at_slot(CD, f, 32LL * bd.cs);
  pre = at_slot(pre, f, bd.cs);
  GS = at_slot(GS, f, GRID_CELLS + 1);
  GI = at_slot(GI, f, bd.cs);
  ckeys = at_slot(ckeys, f, (long long)MK * bd.qs);
  ccnt = at_slot(ccnt, f, bd.qs);
  out = at_slot(out, f, bd.cs);
  nmatch_out += f;
  for (int i = lane; i < n_cur; i += 64) match[i] = pre ? pre[i] : -1;
  __syncthreads();
  const bool bFactor = th != 1.0f;
  int nmatches = 0;
  for (int iMP = 0; iMP < n_mp; iMP++) {
    if ((iMP & 63) == 0) stage_keys(ckeys, ccnt, iMP, min(64, n_mp - iMP), kb, nb);
    const int n = nb[iMP & 63];
    if (n == 0) continue;  // not in view, or no candidate
    // best and second best among the free candidates: the two smallest free stored
    // keys when two of them are free or the query has no more candidates
    const int nk = min(n, MK);
    const unsigned long long sk = lane < nk ? kb[(iMP & 63) * MK + lane] : KEY_NONE;
    const uint64_t fm = ballot(lane < nk && match[key_idx(sk)] < 0);
    unsigned long long m1 = KEY_NONE, m2 = KEY_NONE;
    auto lane_key = [&](int l) {
      return (unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)sk, l) |
             ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(sk >> 32), l) << 32);
    };
    if (__builtin_popcountll(fm) >= 2 || n <= MK) {
      if (fm) m1 = lane_key(__builtin_ctzll(fm));
      const uint64_t f2 = fm & (fm - 1);
      if (f2) m2 = lane_key(__builtin_ctzll(f2));
    } else {
    const int L = min(max(level[iMP], 0), nlevels - 1);  // Q13 clamp
    float r = vcos[iMP] > 0.998f ? 2.5f : 4.0f;
    if (bFactor) r = fmul(r, th);
    const float rr = fmul(r, scales[L]);
    const float x = proj[2 * iMP], y = proj[2 * iMP + 1];
    const Window w = window_cells(cam, x, y, rr);
    const int minL = L - 1, maxL = L;
    const bool checkL = (minL > 0) || (maxL >= 0);
    const int ncy = w.y1 - w.y0 + 1, ncell = (w.x1 - w.x0 + 1) * ncy;
    const uint8_t* d = mdesc + 32 * (long long)iMP;
    unsigned long long b1 = KEY_NONE, b2 = KEY_NONE;
    for (int ck = lane; ck < ncell; ck += 64) {
      const int ix = w.x0 + ck / ncy, iy = w.y0 + ck % ncy;
      const int cell = ix * GRID_ROWS + iy;
      for (int q = GS[cell]; q < GS[cell + 1]; q++) {
        const int idx = GI[q];
        const eao_keypoint_dev& kp = CK[idx];
        if (checkL) {
          if (kp.octave < minL) continue;
          if (maxL >= 0 && kp.octave > maxL) continue;
        }
        if (!(fabsf(fsub(kp.x, x)) < rr && fabsf(fsub(kp.y, y)) < rr)) continue;
        if (match[idx] >= 0) continue;
        const int dist = hamming256(d, CD + 32 * (long long)idx);
        const unsigned long long key = make_key(dist, ck, idx);
        if (key < b1) {
          b2 = b1;
          b1 = key;
        } else if (key < b2) {
          b2 = key;
        }
      }
    }
    m1 = wave_min_u64(b1);
    m2 = wave_min_u64(b1 == m1 ? b2 : b1);
    }
    if (m1 == KEY_NONE) continue;
    const int bestDist = key_dist(m1);
    if (bestDist <= TH_HIGH) {
      const int bestIdx = key_idx(m1);
      const int bestLevel = CK[bestIdx].octave;
      const int bestDist2 = m2 == KEY_NONE ? 256 : key_dist(m2);
      const int bestLevel2 = m2 == KEY_NONE ? -1 : CK[key_idx(m2)].octave;
      if (bestLevel == bestLevel2 && (float)bestDist > fmul(nnratio, (float)bestDist2)) continue;
      if (lane == 0) match[bestIdx] = iMP;
      nmatches++;
      __syncthreads();
    }
  }
  __syncthreads();
  for (int i = lane; i < n_cur; i += 64) out[i] = match[i];
  if (lane == 0) *nmatch_out = nmatches;
}

// SearchForInitialization, ORBmatcher.cc:405-520
__global__ __launch_bounds__(64) void k_match_init(
    CamDev cam, float nnratio, int check_ori, int n1, const eao_keypoint_dev* __restrict__ K1,
    const uint8_t* __restrict__ D1, int n2, const eao_keypoint_dev* __restrict__ K2,
    const uint8_t* __restrict__ D2, float* __restrict__ prev, int window,
    const int* __restrict__ GS, const int* __restrict__ GI, const unsigned long long* __restrict__ ckeys,
    const int* __restrict__ ccnt, int* __restrict__ m12, int* __restrict__ nmatch_out, BatchDims bd) {
  __shared__ unsigned long long kb[64 * MK];
  __shared__ int nb[64];
  __shared__ int mdist[MAXK];
  __shared__ int m21[MAXK];
  __shared__ signed char bins1[MAXK];
  __shared__ int hist[HISTO_LENGTH];
  const int lane = threadIdx.x, f = blockIdx.x;
  if (bd.nq) {
    n1 = min(bd.nq[f], bd.qs);
    n2 = min(bd.nc[f], bd.cs);
  }
  K1 = at_slot(K1, f, bd.qs);
  D1 = at_slot(D1, f, 32LL * bd.qs);
  prev = at_slot(prev, f, 2LL * bd.qs);
  K2 = at_slot(K2, f, bd.cs);
  D2 = at_slot(D2, f, 32LL * bd.cs);
  GS = at_slot(GS, f, GRID_CELLS + 1);
  GI = at_slot(GI, f, bd.cs);
  ckeys = at_slot(ckeys, f, (long long)MK * bd.qs);
  ccnt = at_slot(ccnt, f, bd.qs);
  m12 = at_slot(m12, f, bd.qs);
  nmatch_out += f;
  for (int i = lane; i < n2; i += 64) {
    mdist[i] = INT_MAX;
    m21[i] = -1;
  }
  for (int i = lane; i < n1; i += 64) {
    m12[i] = -1;
    bins1[i] = -1;
  }
  __syncthreads();
  int nmatches = 0;
  const float r = (float)window;
  for (int i1 = 0; i1 < n1; i1++) {
    if ((i1 & 63) == 0) stage_keys(ckeys, ccnt, i1, min(64, n1 - i1), kb, nb);
    const int n = nb[i1 & 63];
    if (n == 0) continue;  // a level > 0 keypoint, or no candidate
    // the vMatchedDistance test (a keypoint of frame 2 is open to strictly closer
    // matches only) decides among the stored keys when two pass or no more exist
    const int nk = min(n, MK);
    const unsigned long long sk = lane < nk ? kb[(i1 & 63) * MK + lane] : KEY_NONE;
    const uint64_t fm = ballot(lane < nk && !(mdist[key_idx(sk)] <= key_dist(sk)));
    unsigned long long m1 = KEY_NONE, m2 = KEY_NONE;
    auto lane_key = [&](int l) {
      return (unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)sk, l) |
             ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(sk >> 32), l) << 32);
    };
    if (__builtin_popcountll(fm) >= 2 || n <= MK) {
      if (fm) m1 = lane_key(__builtin_ctzll(fm));
      const uint64_t f2 = fm & (fm - 1);
      if (f2) m2 = lane_key(__builtin_ctzll(f2));
    } else {
    const float x = prev[2 * i1], y = prev[2 * i1 + 1];
    const Window w = window_cells(cam, x, y, r);
    const int ncy = w.y1 - w.y0 + 1, ncell = (w.x1 - w.x0 + 1) * ncy;
    const uint8_t* d1 = D1 + 32 * (long long)i1;
    unsigned long long b1 = KEY_NONE, b2 = KEY_NONE;
    for (int ck = lane; ck < ncell; ck += 64) {
      const int ix = w.x0 + ck / ncy, iy = w.y0 + ck % ncy;
      const int cell = ix * GRID_ROWS + iy;
      for (int q = GS[cell]; q < GS[cell + 1]; q++) {
        const int i2 = GI[q];
        const eao_keypoint_dev& kp = K2[i2];
        if (kp.octave < 0 || kp.octave > 0) continue;
        if (!(fabsf(fsub(kp.x, x)) < r && fabsf(fsub(kp.y, y)) < r)) continue;
        const int dist = hamming256(d1, D2 + 32 * (long long)i2);
        if (mdist[i2] <= dist) continue;
        const unsigned long long key = make_key(dist, ck, i2);
        if (key < b1) {
          b2 = b1;
          b1 = key;
        } else if (key < b2) {
          b2 = key;
        }
      }
    }
    m1 = wave_min_u64(b1);
    m2 = wave_min_u64(b1 == m1 ? b2 : b1);
    }
    if (m1 == KEY_NONE) continue;
    const int bestDist = key_dist(m1);
    const int bestDist2 = m2 == KEY_NONE ? INT_MAX : key_dist(m2);
    if (bestDist <= TH_LOW && (float)bestDist < fmul((float)bestDist2, nnratio)) {
      const int bestIdx2 = key_idx(m1);
      const int prev21 = m21[bestIdx2];
      if (prev21 >= 0) nmatches--;
      if (lane == 0) {
        if (prev21 >= 0) m12[prev21] = -1;
        m12[i1] = bestIdx2;
        m21[bestIdx2] = i1;
        mdist[bestIdx2] = bestDist;
        if (check_ori) bins1[i1] = (signed char)rot_bin(K1[i1].angle, K2[bestIdx2].angle);
      }
      nmatches++;
      __syncthreads();
    }
  }
  __syncthreads();
  if (check_ori) {
    for (int b = lane; b < HISTO_LENGTH; b += 64) hist[b] = 0;
    __syncthreads();
    for (int i = lane; i < n1; i += 64)
      if (bins1[i] >= 0) atomicAdd(&hist[bins1[i]], 1);
    __syncthreads();
    int ind1, ind2, ind3;
    three_maxima(hist, ind1, ind2, ind3);
    int removed = 0;
    for (int i = lane; i < n1; i += 64) {
      const int b = bins1[i];
      if (b < 0 || b == ind1 || b == ind2 || b == ind3) continue;
      if (m12[i] >= 0) {
        m12[i] = -1;
        removed++;
      }
    }
    nmatches -= wave_sum(removed);
  }
  __syncthreads();
  for (int i = lane; i < n1; i += 64)
    if (m12[i] >= 0) {
      prev[2 * i] = K2[m12[i]].x;
      prev[2 * i + 1] = K2[m12[i]].y;
    }
  if (lane == 0) *nmatch_out = nmatches;
}

__global__ void k_hamming_pairs(const uint8_t* __restrict__ q, const uint8_t* __restrict__ t,
                                const int* __restrict__ qi, const int* __restrict__ ti, int n,
                                int* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = hamming256(q + 32 * (long long)qi[i], t + 32 * (long long)ti[i]);
}

// ================================================================ host
int MatchEngine::init(int device, int mk, int mb) {
  dev = device;
  max_kps = mk;
  max_batch = std::max(mb, 2);
  if (mk < 1 || mk > MAXK) {
    set_error("eao_matcher_create: max_kps outside [1, 8192]");
    return EAO_E_ARG;
  }
  EAO_HIP_CHECK(hipSetDevice(dev));
  EAO_HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  EAO_HIP_CHECK(hipMalloc(&d_gstart, sizeof(int) * (GRID_CELLS + 1) * max_batch));
  EAO_HIP_CHECK(hipMalloc(&d_gitems, sizeof(int) * (size_t)mk * max_batch));
  EAO_HIP_CHECK(hipMalloc(&d_kps, sizeof(eao_keypoint_dev) * mk * 2));
  EAO_HIP_CHECK(hipMalloc(&d_desc, (size_t)32 * mk * 2));
  EAO_HIP_CHECK(hipMalloc(&d_u8, (size_t)mk * 2));
  EAO_HIP_CHECK(hipMalloc(&d_f, sizeof(float) * 3 * mk * 2));
  EAO_HIP_CHECK(hipMalloc(&d_f2, sizeof(float) * 3 * mk));
  EAO_HIP_CHECK(hipMalloc(&d_f3, sizeof(float) * 3 * mk));
  EAO_HIP_CHECK(hipMalloc(&d_f4, sizeof(float) * 3 * mk));
  EAO_HIP_CHECK(hipMalloc(&d_mdesc, (size_t)32 * mk * 2));
  EAO_HIP_CHECK(hipMalloc(&d_i32, sizeof(int) * mk * 2));
  EAO_HIP_CHECK(hipMalloc(&d_i32b, sizeof(int) * mk * 2));
  EAO_HIP_CHECK(hipMalloc(&d_out, sizeof(int) * (mk * 2 + 16)));
  EAO_HIP_CHECK(hipMalloc(&d_T, sizeof(float) * 16 * 2));
  EAO_HIP_CHECK(hipMalloc(&d_scales, sizeof(float) * 32));
  EAO_HIP_CHECK(hipMalloc(&d_geo, sizeof(float) * 4 * (size_t)mk * max_batch));
  EAO_HIP_CHECK(hipMalloc(&d_ckeys, sizeof(unsigned long long) * MK * (size_t)mk * max_batch));
  EAO_HIP_CHECK(hipMalloc(&d_cbins, (size_t)MK * mk * max_batch));
  EAO_HIP_CHECK(hipMalloc(&d_ccnt, sizeof(int) * (size_t)mk * max_batch));
  return EAO_OK;
}

MatchEngine::~MatchEngine() {
  void* ptrs[] = {d_gstart, d_gitems, d_kps, d_desc, d_u8, d_f, d_f2, d_f3, d_f4,
                  d_mdesc, d_i32, d_i32b, d_out, d_T, d_scales, d_geo, d_ckeys, d_cbins, d_ccnt};
  for (void* q : ptrs)
    if (q) (void)hipFree(q);
  if (stream) (void)hipStreamDestroy(stream);
}

// the two phases of the motion-model search for pairs (p, p+1), p < nframes-1
int MatchEngine::motion(const CamDev& cd, const float* d_T, float th, int check_ori, const eao_keypoint_dev* d_kps,
                        const uint8_t* d_desc, const int* d_counts, int cap, const uint8_t* d_has,
                        const float* d_pos, const uint8_t* d_mdesc_, const float* d_sc, int nframes, int* d_match,
                        int* d_nm, hipStream_t s) {
  const int np = nframes - 1;
  if (np < 1) return EAO_OK;
  if ((long long)np * cap > (long long)max_batch * max_kps) {
    set_error("motion search: scratch too small");
    return EAO_E_CAPACITY;
  }
  if (np <= 4)  // latency form: a wave per query (a single call's ~1000 queries fill the chip)
    hipLaunchKernelGGL(k_motion_cand_wave, dim3((cap + 3) / 4, np), dim3(256), 0, s, cd, d_T, th, d_kps, d_desc,
                       d_counts, cap, d_has, d_pos, d_mdesc_, d_sc, d_gstart, d_gitems, d_ckeys, d_cbins, d_ccnt);
  else
    hipLaunchKernelGGL(k_motion_cand, dim3((cap + 255) / 256, np), dim3(256), 0, s, cd, d_T, th, d_kps, d_desc,
                       d_counts, cap, d_has, d_pos, d_mdesc_, d_sc, d_gstart, d_gitems, d_ckeys, d_cbins, d_ccnt);
  EAO_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_motion_resolve, dim3(np), dim3(64), 0, s, cd, d_T, th, check_ori, d_kps, d_desc, d_counts,
                     cap, d_has, d_pos, d_mdesc_, d_sc, d_gstart, d_gitems, d_ckeys, d_cbins, d_ccnt, d_match, d_nm);
  EAO_HIP_CHECK(hipGetLastError());
  return EAO_OK;
}

int MatchEngine::build_grid(const CamDev& cam, const eao_keypoint_dev* kps, const int* counts,
                            int n_single, int cap, int nframes, hipStream_t s) {
  hipLaunchKernelGGL(k_grid, dim3(nframes), dim3(256), 0, s, kps, counts, n_single, cap, cam,
                     d_gstart, d_gitems);
  EAO_HIP_CHECK(hipGetLastError());
  return EAO_OK;
}

}  // namespace eao

// ---------------------------------------------------------------- C ABI
using namespace eao;

struct eao_matcher {
  MatchEngine e;
};


extern "C" {

int eao_matcher_create(int device, int max_kps, int max_batch, eao_matcher** out) {
  if (!out) return EAO_E_ARG;
  *out = nullptr;
  if (!eao_device_ok(device)) {
    set_error("no usable gfx950 device (the engine has no CPU fallback)");
    return EAO_E_NODEVICE;
  }
  eao_matcher* m = new eao_matcher();
  int rc = m->e.init(device, max_kps, max_batch);
  if (rc) {
    delete m;
    return rc;
  }
  *out = m;
  return EAO_OK;
}

int eao_matcher_destroy(eao_matcher* m) {
  delete m;
  return EAO_OK;
}

int eao_hamming_pairs(eao_matcher* m, const uint8_t* q, int nq, const uint8_t* t, int nt,
                      const int32_t* qidx, const int32_t* tidx, int npairs, int32_t* dist) {
  if (!m || npairs < 0 || nq > m->e.max_kps || nt > m->e.max_kps || npairs > 2 * m->e.max_kps)
    return EAO_E_ARG;
  if (npairs == 0) return EAO_OK;
  MatchEngine& e = m->e;
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_desc, q, (size_t)nq * 32, hipMemcpyHostToDevice, e.stream));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_mdesc, t, (size_t)nt * 32, hipMemcpyHostToDevice, e.stream));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_i32, qidx, sizeof(int) * npairs, hipMemcpyHostToDevice, e.stream));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_i32b, tidx, sizeof(int) * npairs, hipMemcpyHostToDevice, e.stream));
  hipLaunchKernelGGL(k_hamming_pairs, dim3((npairs + 255) / 256), dim3(256), 0, e.stream, e.d_desc,
                     e.d_mdesc, e.d_i32, e.d_i32b, npairs, e.d_out);
  EAO_HIP_CHECK(hipMemcpyAsync(dist, e.d_out, sizeof(int) * npairs, hipMemcpyDeviceToHost, e.stream));
  EAO_HIP_CHECK(hipStreamSynchronize(e.stream));
  return EAO_OK;
}

int eao_match_motion(eao_matcher* m, const eao_camera* cam, const float* Tcw, float th,
                     int check_ori, int n_last, const eao_keypoint* last_kps,
                     const uint8_t* last_has_mp, const float* last_mp_pos,
                     const uint8_t* last_mp_desc, int n_cur, const eao_keypoint* cur_kps,
                     const uint8_t* cur_desc, int nlevels, const float* scale_factors,
                     int32_t* cur_match) {
  if (!m || !cam || !Tcw || n_last < 0 || n_cur < 0 || nlevels < 1 || nlevels > 32) return EAO_E_ARG;
  MatchEngine& e = m->e;
  const int K = e.max_kps;
  if (n_last > K || n_cur > K) {
    set_error("eao_match_motion: more keypoints than max_kps");
    return EAO_E_CAPACITY;
  }
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  hipStream_t s = e.stream;
  // slot stride C (the kernels take it as cap): the two frames' inputs packed into the pinned
  // staging image, one copy over; the current frame's matches and the counts come back in one
  // (C <= max_kps: the grid items, candidate keys and results are sized [2][max_kps])
  const int C = std::min((std::max(std::max(n_last, n_cur), 1) + 63) & ~63, K);
  const int counts[4] = {n_last, n_cur, 0, 0};
  float T2[32];
  for (int k = 0; k < 16; k++) T2[k] = T2[16 + k] = Tcw[k];
  HostStage& st = e.stage;
  const size_t kb = sizeof(eao_keypoint);
  EAO_HIP_CHECK(st.reserve(HostStage::al(2 * C * kb) + 2 * (size_t)C * 32 + C + 12 * (size_t)C + 32 * (size_t)C + 512));
  const size_t o_kps = st.put(nullptr, 2 * C * kb);
  std::memcpy(st.h + o_kps, last_kps, kb * n_last);
  std::memcpy(st.h + o_kps + kb * C, cur_kps, kb * n_cur);
  const size_t o_desc = st.put(nullptr, 2 * (size_t)C * 32);  // slot 0 unused by the motion search
  std::memcpy(st.h + o_desc + (size_t)C * 32, cur_desc, (size_t)n_cur * 32);
  const size_t o_has = st.put(last_has_mp, n_last);
  const size_t o_pos = st.put(last_mp_pos, sizeof(float) * 3 * n_last);
  const size_t o_md = st.put(last_mp_desc, (size_t)n_last * 32);
  const size_t o_cnt = st.put(counts, sizeof(counts));
  const size_t o_T = st.put(T2, sizeof(T2));
  const size_t o_sc = st.put(scale_factors, sizeof(float) * nlevels);
  EAO_HIP_CHECK(st.upload(s));
  const CamDev cd = make_cam(*cam);
  const eao_keypoint_dev* dk = st.dev<const eao_keypoint_dev>(o_kps);
  const int* dc = st.dev<const int>(o_cnt);
  int rc = e.build_grid(cd, dk, dc, 0, C, 2, s);
  if (rc) return rc;
  rc = e.motion(cd, st.dev<const float>(o_T), th, check_ori, dk, st.dev<const uint8_t>(o_desc), dc, C,
                st.dev<const uint8_t>(o_has), st.dev<const float>(o_pos), st.dev<const uint8_t>(o_md),
                st.dev<const float>(o_sc), 2, e.d_out, e.d_out + 2 * C, s);
  if (rc) return rc;
  EAO_HIP_CHECK(hipGetLastError());
  // [C matches of slot 1][nm[0], nm[1]]
  EAO_HIP_CHECK(e.res.reserve(sizeof(int) * (C + 2)));
  EAO_HIP_CHECK(hipMemcpyAsync(e.res.h, e.d_out + C, sizeof(int) * (C + 2), hipMemcpyDeviceToHost, s));
  EAO_HIP_CHECK(hipStreamSynchronize(s));
  const int* r = (const int*)e.res.h;
  std::memcpy(cur_match, r, sizeof(int) * n_cur);
  return r[C + 1];
}

int eao_match_motion_batch_device(eao_matcher* m, const eao_camera* cam, int nframes, int cap,
                                  const float* d_Tcw, float th, int check_ori,
                                  const eao_keypoint* d_kps, const uint8_t* d_desc,
                                  const int32_t* d_counts, const uint8_t* d_has_mp,
                                  const float* d_mp_pos, const uint8_t* d_mp_desc, int nlevels,
                                  const float* scale_factors, int32_t* d_cur_match,
                                  int32_t* d_nmatches, void* stream) {
  if (!m || !cam || nframes < 2 || nframes > m->e.max_batch || cap > m->e.max_kps || nlevels < 1 ||
      nlevels > 32)
    return EAO_E_ARG;
  MatchEngine& e = m->e;
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  hipStream_t s = stream ? (hipStream_t)stream : e.stream;
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_scales, scale_factors, sizeof(float) * nlevels, hipMemcpyHostToDevice, s));
  const CamDev cd = make_cam(*cam);
  int rc = e.build_grid(cd, (const eao_keypoint_dev*)d_kps, d_counts, 0, cap, nframes, s);
  if (rc) return rc;
  rc = e.motion(cd, d_Tcw, th, check_ori, (const eao_keypoint_dev*)d_kps, d_desc, d_counts, cap, d_has_mp, d_mp_pos,
                d_mp_desc, e.d_scales, nframes, d_cur_match, d_nmatches, s);
  if (rc) return rc;
  EAO_HIP_CHECK(hipGetLastError());
  return EAO_OK;
}

// ---- batched, HBM-resident single-frame searches: search f reads query slot f and
// frame slot f; one candidate launch over all searches, one resolving wave per search
static int batch_args(eao_matcher* m, const eao_camera* cam, int nsearch, int qcap, int cap, int nlevels,
                      const void* q_counts, const void* c_counts, const char* what) {
  if (!m || !cam || nsearch < 1 || qcap < 1 || cap < 1 || nlevels < 1 || nlevels > 32 || !q_counts || !c_counts)
    return EAO_E_ARG;
  if (nsearch > m->e.max_batch || qcap > m->e.max_kps || cap > m->e.max_kps) {
    set_error(std::string(what) + ": more searches than max_batch or slots larger than max_kps");
    return EAO_E_CAPACITY;
  }
  return EAO_OK;
}

int eao_match_local_batch_device(eao_matcher* m, const eao_camera* cam, int nsearch, float th, float nnratio,
                                 int mp_cap, const int32_t* d_n_mp, const uint8_t* d_in_view, const float* d_proj_xy,
                                 const int32_t* d_pred_level, const float* d_view_cos, const uint8_t* d_mp_desc,
                                 int cap, const int32_t* d_n_cur, const eao_keypoint* d_cur_kps,
                                 const uint8_t* d_cur_desc, const int32_t* d_cur_preassigned, int nlevels,
                                 const float* scale_factors, int32_t* d_cur_match, int32_t* d_nmatches,
                                 void* stream) {
  int rc = batch_args(m, cam, nsearch, mp_cap, cap, nlevels, d_n_mp, d_n_cur, "eao_match_local_batch_device");
  if (rc) return rc;
  MatchEngine& e = m->e;
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  hipStream_t s = stream ? (hipStream_t)stream : e.stream;
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_scales, scale_factors, sizeof(float) * nlevels, hipMemcpyHostToDevice, s));
  const CamDev cd = make_cam(*cam);
  const auto* CK = (const eao_keypoint_dev*)d_cur_kps;
  rc = e.build_grid(cd, CK, d_n_cur, 0, cap, nsearch, s);
  if (rc) return rc;
  const BatchDims bd{d_n_mp, d_n_cur, mp_cap, cap};
  hipLaunchKernelGGL(k_local_cand, dim3((mp_cap + 255) / 256, nsearch), dim3(256), 0, s, cd, th, 0, d_in_view,
                     d_proj_xy, d_pred_level, d_view_cos, d_mp_desc, CK, d_cur_desc, d_cur_preassigned, nlevels,
                     e.d_scales, e.d_gstart, e.d_gitems, e.d_ckeys, e.d_ccnt, bd);
  hipLaunchKernelGGL(k_match_local, dim3(nsearch), dim3(64), 0, s, cd, th, nnratio, 0, d_in_view, d_proj_xy,
                     d_pred_level, d_view_cos, d_mp_desc, 0, CK, d_cur_desc, d_cur_preassigned, nlevels, e.d_scales,
                     e.d_gstart, e.d_gitems, e.d_ckeys, e.d_ccnt, d_cur_match, d_nmatches, bd);
  EAO_HIP_CHECK(hipGetLastError());
  return EAO_OK;
}

int eao_match_keyframe_batch_device(eao_matcher* m, const eao_camera* cam, int nsearch, const float* d_Tcw,
                                    float th, int orb_dist, int check_ori, int kf_cap, const int32_t* d_n_kf,
                                    const eao_keypoint* d_kf_kps, const uint8_t* d_kf_mp_valid,
                                    const float* d_kf_mp_pos, const uint8_t* d_kf_mp_desc,
                                    const float* d_kf_mp_min_dist, const float* d_kf_mp_max_dist,
                                    float log_scale_factor, int cap, const int32_t* d_n_cur,
                                    const eao_keypoint* d_cur_kps, const uint8_t* d_cur_desc,
                                    const int32_t* d_cur_preassigned, int nlevels, const float* scale_factors,
                                    int32_t* d_cur_match, int32_t* d_nmatches, void* stream) {
  int rc = batch_args(m, cam, nsearch, kf_cap, cap, nlevels, d_n_kf, d_n_cur, "eao_match_keyframe_batch_device");
  if (rc) return rc;
  if (!d_Tcw) return EAO_E_ARG;
  MatchEngine& e = m->e;
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  hipStream_t s = stream ? (hipStream_t)stream : e.stream;
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_scales, scale_factors, sizeof(float) * nlevels, hipMemcpyHostToDevice, s));
  const CamDev cd = make_cam(*cam);
  const auto* CK = (const eao_keypoint_dev*)d_cur_kps;
  const auto* KK = (const eao_keypoint_dev*)d_kf_kps;
  rc = e.build_grid(cd, CK, d_n_cur, 0, cap, nsearch, s);
  if (rc) return rc;
  const BatchDims bd{d_n_kf, d_n_cur, kf_cap, cap};
  hipLaunchKernelGGL(k_keyframe_cand, dim3((kf_cap + 255) / 256, nsearch), dim3(256), 0, s, cd, d_Tcw, th, 0,
                     d_kf_mp_valid, d_kf_mp_pos, d_kf_mp_desc, d_kf_mp_min_dist, d_kf_mp_max_dist, log_scale_factor,
                     CK, d_cur_desc, d_cur_preassigned, nlevels, e.d_scales, e.d_gstart, e.d_gitems,
                     reinterpret_cast<float4*>(e.d_geo), e.d_ckeys, e.d_ccnt, bd);
  hipLaunchKernelGGL(k_match_keyframe, dim3(nsearch), dim3(64), 0, s, cd, d_Tcw, th, orb_dist, check_ori, 0, KK,
                     d_kf_mp_valid, d_kf_mp_pos, d_kf_mp_desc, d_kf_mp_min_dist, d_kf_mp_max_dist, log_scale_factor, 0,
                     CK, d_cur_desc, d_cur_preassigned, nlevels, e.d_scales, e.d_gstart, e.d_gitems,
                     reinterpret_cast<const float4*>(e.d_geo), e.d_ckeys, e.d_ccnt, d_cur_match, d_nmatches, bd);
  EAO_HIP_CHECK(hipGetLastError());
  return EAO_OK;
}

int eao_match_init_batch_device(eao_matcher* m, const eao_camera* cam, int nsearch, float nnratio, int check_ori,
                                int cap1, const int32_t* d_n1, const eao_keypoint* d_kps1, const uint8_t* d_desc1,
                                int cap2, const int32_t* d_n2, const eao_keypoint* d_kps2, const uint8_t* d_desc2,
                                float* d_prev_matched_xy, int window, int32_t* d_matches12, int32_t* d_nmatches,
                                void* stream) {
  int rc = batch_args(m, cam, nsearch, cap1, cap2, 1, d_n1, d_n2, "eao_match_init_batch_device");
  if (rc) return rc;
  MatchEngine& e = m->e;
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  hipStream_t s = stream ? (hipStream_t)stream : e.stream;
  const CamDev cd = make_cam(*cam);
  const auto* K1 = (const eao_keypoint_dev*)d_kps1;
  const auto* K2 = (const eao_keypoint_dev*)d_kps2;
  rc = e.build_grid(cd, K2, d_n2, 0, cap2, nsearch, s);
  if (rc) return rc;
  const BatchDims bd{d_n1, d_n2, cap1, cap2};
  hipLaunchKernelGGL(k_init_cand, dim3((cap1 + 255) / 256, nsearch), dim3(256), 0, s, cd, 0, K1, d_desc1, K2,
                     d_desc2, d_prev_matched_xy, window, e.d_gstart, e.d_gitems, e.d_ckeys, e.d_ccnt, bd);
  hipLaunchKernelGGL(k_match_init, dim3(nsearch), dim3(64), 0, s, cd, nnratio, check_ori, 0, K1, d_desc1, 0, K2,
                     d_desc2, d_prev_matched_xy, window, e.d_gstart, e.d_gitems, e.d_ckeys, e.d_ccnt, d_matches12,
                     d_nmatches, bd);
  EAO_HIP_CHECK(hipGetLastError());
  return EAO_OK;
}

int eao_is_in_frustum(eao_matcher* m, const eao_camera* cam, const float* Tcw, int n_mp,
                      const float* mp_pos, const float* mp_normal, const float* mp_min_dist,
                      const float* mp_max_dist, float view_cos_limit, float log_scale_factor,
                      uint8_t* in_view, float* proj_xy, int32_t* pred_level, float* view_cos) {
  if (!m || !cam || n_mp < 0 || n_mp > m->e.max_kps) return EAO_E_ARG;
  if (n_mp == 0) return 0;
  MatchEngine& e = m->e;
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  hipStream_t s = e.stream;
  const int K = e.max_kps;
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_T, Tcw, sizeof(float) * 16, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_f, mp_pos, sizeof(float) * 3 * n_mp, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_f2, mp_normal, sizeof(float) * 3 * n_mp, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_f3, mp_min_dist, sizeof(float) * n_mp, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_f3 + K, mp_max_dist, sizeof(float) * n_mp, hipMemcpyHostToDevice, s));
  const CamDev cd = make_cam(*cam);
  hipLaunchKernelGGL(k_frustum, dim3((n_mp + 255) / 256), dim3(256), 0, s, cd, e.d_T, n_mp, e.d_f,
                     e.d_f2, e.d_f3, e.d_f3 + K, view_cos_limit, log_scale_factor, e.d_u8, e.d_f4,
                     e.d_i32, e.d_f4 + 2 * K);
  EAO_HIP_CHECK(hipGetLastError());
  EAO_HIP_CHECK(hipMemcpyAsync(in_view, e.d_u8, n_mp, hipMemcpyDeviceToHost, s));
  EAO_HIP_CHECK(hipMemcpyAsync(proj_xy, e.d_f4, sizeof(float) * 2 * n_mp, hipMemcpyDeviceToHost, s));
  EAO_HIP_CHECK(hipMemcpyAsync(pred_level, e.d_i32, sizeof(int) * n_mp, hipMemcpyDeviceToHost, s));
  EAO_HIP_CHECK(hipMemcpyAsync(view_cos, e.d_f4 + 2 * K, sizeof(float) * n_mp, hipMemcpyDeviceToHost, s));
  EAO_HIP_CHECK(hipStreamSynchronize(s));
  int c = 0;
  for (int i = 0; i < n_mp; i++) c += in_view[i] ? 1 : 0;
  return c;
}

int eao_match_local(eao_matcher* m, const eao_camera* cam, float th, float nnratio, int n_mp,
                    const uint8_t* in_view, const float* proj_xy, const int32_t* pred_level,
                    const float* view_cos,
                    const uint8_t* mp_desc, int n_cur, const eao_keypoint* cur_kps,
                    const uint8_t* cur_desc, const int32_t* cur_preassigned, int nlevels,
                    const float* scale_factors, int32_t* cur_match) {
  if (!m || !cam || n_mp < 0 || n_cur < 0 || nlevels < 1 || nlevels > 32) return EAO_E_ARG;
  MatchEngine& e = m->e;
  const int K = e.max_kps;
  if (n_mp > K || n_cur > K) return EAO_E_CAPACITY;
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  hipStream_t s = e.stream;
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_kps, cur_kps, sizeof(eao_keypoint) * n_cur, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_desc, cur_desc, (size_t)n_cur * 32, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_f, proj_xy, sizeof(float) * 2 * n_mp, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_i32, pred_level, sizeof(int) * n_mp, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_f2, view_cos, sizeof(float) * n_mp, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_mdesc, mp_desc, (size_t)n_mp * 32, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_u8, in_view, n_mp, hipMemcpyHostToDevice, s));
  if (cur_preassigned)
    EAO_HIP_CHECK(hipMemcpyAsync(e.d_i32b, cur_preassigned, sizeof(int) * n_cur, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_scales, scale_factors, sizeof(float) * nlevels, hipMemcpyHostToDevice, s));
  const CamDev cd = make_cam(*cam);
  int rc = e.build_grid(cd, e.d_kps, nullptr, n_cur, K, 1, s);
  if (rc) return rc;
  if (n_mp > 0)
    hipLaunchKernelGGL(k_local_cand, dim3((n_mp + 255) / 256), dim3(256), 0, s, cd, th, n_mp, e.d_u8, e.d_f,
                       e.d_i32, e.d_f2, e.d_mdesc, e.d_kps, e.d_desc, cur_preassigned ? e.d_i32b : nullptr, nlevels,
                       e.d_scales, e.d_gstart, e.d_gitems, e.d_ckeys, e.d_ccnt, BatchDims{});
  hipLaunchKernelGGL(k_match_local, dim3(1), dim3(64), 0, s, cd, th, nnratio, n_mp, e.d_u8, e.d_f, e.d_i32,
                     e.d_f2, e.d_mdesc, n_cur, e.d_kps, e.d_desc,
                     cur_preassigned ? e.d_i32b : nullptr, nlevels, e.d_scales, e.d_gstart,
                     e.d_gitems, e.d_ckeys, e.d_ccnt, e.d_out, e.d_out + 2 * K, BatchDims{});
  EAO_HIP_CHECK(hipGetLastError());
  int nm = 0;
  EAO_HIP_CHECK(hipMemcpyAsync(cur_match, e.d_out, sizeof(int) * n_cur, hipMemcpyDeviceToHost, s));
  // the stream's work is complete before the count is read (no async copy into a stack variable)
  EAO_HIP_CHECK(hipStreamSynchronize(s));
  EAO_HIP_CHECK(hipMemcpy(&nm, e.d_out + 2 * K, sizeof(int), hipMemcpyDeviceToHost));
  return nm;
}

int eao_match_keyframe(eao_matcher* m, const eao_camera* cam, const float* Tcw, float th,
                       int orb_dist, int check_ori, int n_kf, const eao_keypoint* kf_kps,
                       const uint8_t* kf_mp_valid, const float* kf_mp_pos,
                       const uint8_t* kf_mp_desc, const float* kf_mp_min_dist,
                       const float* kf_mp_max_dist, float log_scale_factor, int n_cur,
                       const eao_keypoint* cur_kps, const uint8_t* cur_desc,
                       const int32_t* cur_preassigned, int nlevels, const float* scale_factors,
                       int32_t* cur_match) {
  if (!m || !cam || !Tcw || n_kf < 0 || n_cur < 0 || nlevels < 1 || nlevels > 32) return EAO_E_ARG;
  MatchEngine& e = m->e;
  const int K = e.max_kps;
  if (n_kf > K || n_cur > K) {
    set_error("eao_match_keyframe: more keypoints than max_kps");
    return EAO_E_CAPACITY;
  }
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  hipStream_t s = e.stream;
  // slot 0 = current frame (grid), slot 1 = keyframe keypoints (angles)
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_kps, cur_kps, sizeof(eao_keypoint) * n_cur, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_kps + K, kf_kps, sizeof(eao_keypoint) * n_kf, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_desc, cur_desc, (size_t)n_cur * 32, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_u8, kf_mp_valid, n_kf, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_f, kf_mp_pos, sizeof(float) * 3 * n_kf, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_mdesc, kf_mp_desc, (size_t)n_kf * 32, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_f3, kf_mp_min_dist, sizeof(float) * n_kf, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_f3 + K, kf_mp_max_dist, sizeof(float) * n_kf, hipMemcpyHostToDevice, s));
  if (cur_preassigned)
    EAO_HIP_CHECK(hipMemcpyAsync(e.d_i32b, cur_preassigned, sizeof(int) * n_cur, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_T, Tcw, sizeof(float) * 16, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_scales, scale_factors, sizeof(float) * nlevels, hipMemcpyHostToDevice, s));
  const CamDev cd = make_cam(*cam);
  int rc = e.build_grid(cd, e.d_kps, nullptr, n_cur, K, 1, s);
  if (rc) return rc;
  if (n_kf > 0)
    hipLaunchKernelGGL(k_keyframe_cand, dim3((n_kf + 255) / 256), dim3(256), 0, s, cd, e.d_T, th, n_kf, e.d_u8,
                       e.d_f, e.d_mdesc, e.d_f3, e.d_f3 + K, log_scale_factor, e.d_kps, e.d_desc,
                       cur_preassigned ? e.d_i32b : nullptr, nlevels, e.d_scales, e.d_gstart, e.d_gitems,
                       reinterpret_cast<float4*>(e.d_geo), e.d_ckeys, e.d_ccnt, BatchDims{});
  hipLaunchKernelGGL(k_match_keyframe, dim3(1), dim3(64), 0, s, cd, e.d_T, th, orb_dist, check_ori,
                     n_kf, e.d_kps + K, e.d_u8, e.d_f, e.d_mdesc, e.d_f3, e.d_f3 + K,
                     log_scale_factor, n_cur, e.d_kps, e.d_desc,
                     cur_preassigned ? e.d_i32b : nullptr, nlevels, e.d_scales, e.d_gstart,
                     e.d_gitems, reinterpret_cast<const float4*>(e.d_geo), e.d_ckeys, e.d_ccnt, e.d_out,
                     e.d_out + 2 * K, BatchDims{});
  EAO_HIP_CHECK(hipGetLastError());
  int nm = 0;
  EAO_HIP_CHECK(hipMemcpyAsync(cur_match, e.d_out, sizeof(int) * n_cur, hipMemcpyDeviceToHost, s));
  // the stream's work is complete before the count is read (no async copy into a stack variable)
  EAO_HIP_CHECK(hipStreamSynchronize(s));
  EAO_HIP_CHECK(hipMemcpy(&nm, e.d_out + 2 * K, sizeof(int), hipMemcpyDeviceToHost));
  return nm;
}

int eao_match_init(eao_matcher* m, const eao_camera* cam, float nnratio, int check_ori, int n1,
                   const eao_keypoint* kps1, const uint8_t* desc1, int n2,
                   const eao_keypoint* kps2, const uint8_t* desc2, float* prev_matched_xy,
                   int window, int32_t* matches12) {
  if (!m || !cam || n1 < 0 || n2 < 0) return EAO_E_ARG;
  MatchEngine& e = m->e;
  const int K = e.max_kps;
  if (n1 > K || n2 > K) return EAO_E_CAPACITY;
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  hipStream_t s = e.stream;
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_kps, kps2, sizeof(eao_keypoint) * n2, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_desc, desc2, (size_t)n2 * 32, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_kps + K, kps1, sizeof(eao_keypoint) * n1, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_desc + (size_t)K * 32, desc1, (size_t)n1 * 32, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_f, prev_matched_xy, sizeof(float) * 2 * n1, hipMemcpyHostToDevice, s));
  const CamDev cd = make_cam(*cam);
  int rc = e.build_grid(cd, e.d_kps, nullptr, n2, K, 1, s);
  if (rc) return rc;
  if (n1 > 0)
    hipLaunchKernelGGL(k_init_cand, dim3((n1 + 255) / 256), dim3(256), 0, s, cd, n1, e.d_kps + K,
                       e.d_desc + (size_t)K * 32, e.d_kps, e.d_desc, e.d_f, window, e.d_gstart, e.d_gitems,
                       e.d_ckeys, e.d_ccnt, BatchDims{});
  hipLaunchKernelGGL(k_match_init, dim3(1), dim3(64), 0, s, cd, nnratio, check_ori, n1,
                     e.d_kps + K, e.d_desc + (size_t)K * 32, n2, e.d_kps, e.d_desc, e.d_f, window,
                     e.d_gstart, e.d_gitems, e.d_ckeys, e.d_ccnt, e.d_out, e.d_out + 2 * K, BatchDims{});
  EAO_HIP_CHECK(hipGetLastError());
  int nm = 0;
  EAO_HIP_CHECK(hipMemcpyAsync(matches12, e.d_out, sizeof(int) * n1, hipMemcpyDeviceToHost, s));
  EAO_HIP_CHECK(hipMemcpyAsync(prev_matched_xy, e.d_f, sizeof(float) * 2 * n1, hipMemcpyDeviceToHost, s));
  // the stream's work is complete before the count is read (no async copy into a stack variable)
  EAO_HIP_CHECK(hipStreamSynchronize(s));
  EAO_HIP_CHECK(hipMemcpy(&nm, e.d_out + 2 * K, sizeof(int), hipMemcpyDeviceToHost));
  return nm;
}

}  // extern "C"
