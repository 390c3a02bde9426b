// assoc.hip -- EAO object-association kernels on gfx950 (reference src/Object.cc,
// include/isolation_forest.h).
//
//   k_np_pairs     one workgroup per (detection, object) pair: the Wilcoxon
//                  rank-sum of NoParaDataAssociation (Object.cc:714-930) as
//                  sort + rank counting (counts identical to the O(m*n) loop)
//   k_rects        one workgroup per cloud: ComputeProjectRectFrame (:1558-1603)
//   k_iforest_tree one workgroup per (tree, cloud): IsolationTree::Build with
//                  the libstdc++-11 mt19937 / Lemire / shuffle / canonical-float
//                  stream replicated exactly (isolation_forest.h:165-224,300-345),
//                  tree and sample resident in LDS, then every point's path
//                  length through it
//   k_iforest_sum  one thread per point: path lengths summed in tree order,
//                  score 2^(-E[h]/c(psi)) (isolation_forest.h:499-530)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "assoc.h"
#include "common.h"

namespace eao {

// ---------------------------------------------------------------- NP test
__device__ void block_bitonic_sort(float* a, int P) {
  for (int k = 2; k <= P; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += blockDim.x) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const float x = a[i], y = a[ixj];
          const bool up = (i & k) == 0;
          if ((x > y) == up) {
            a[i] = y;
            a[ixj] = x;
          }
        }
      }
      __syncthreads();
    }
}

__device__ int block_sum_int(int v, int* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  int t = 0;
  for (int i = 0; i < (int)(blockDim.x >> 6); i++) t += red[i];
  __syncthreads();
  return t;
}

__global__ __launch_bounds__(256) void k_np_pairs(const float* __restrict__ fp,
                                                  const uint8_t* __restrict__ fv,
                                                  const int* __restrict__ foff,
                                                  const int* __restrict__ flen,
                                                  const float* __restrict__ op,
                                                  const uint8_t* __restrict__ ov,
                                                  const int* __restrict__ ooff,
                                                  const int* __restrict__ olen,
                                                  eao_np_stats* __restrict__ out) {
  __shared__ float S[NP_MAXN];
  __shared__ int red[8];
  __shared__ int wpos[4];
  const int p = blockIdx.x, t = threadIdx.x;
  const float* F = fp + 3 * (long long)foff[p];
  const uint8_t* FV = fv + foff[p];
  const int mt = flen[p];
  const float* O = op + 3 * (long long)ooff[p];
  const uint8_t* OV = ov + ooff[p];
  const int nt = olen[p];
  int mloc = 0, nloc = 0;
  for (int i = t; i < mt; i += 256) mloc += FV[i] ? 1 : 0;
  for (int i = t; i < nt; i += 256) nloc += OV[i] ? 1 : 0;
  const int m = block_sum_int(mloc, red);
  const int nvalid = block_sum_int(nloc, red);
  eao_np_stats r;
  r.m = m;
  r.n = nvalid;
  for (int a = 0; a < 3; a++) r.w[a] = r.cnt_gt[a] = r.cnt_lt[a] = r.cnt_eq[a] = 0.f;
  r.r1 = r.r2 = 0.f;
  if (m < 20 || nvalid < 20 || nvalid > NP_MAXN) {
    if (t == 0) {
      r.verdict = m < 20 ? 0 : (nvalid > NP_MAXN ? -1 : 2);
      out[p] = r;
    }
    return;
  }
  const bool sub = nvalid > 3 * m;
  const int step = sub ? nt / (3 * m) : 1;  // step counts invalid points too (Q3)
  const int nsamp = sub ? (nvalid + step - 1) / step : nvalid;
  int P = 1;
  while (P < nvalid) P <<= 1;
  for (int a = 0; a < 3; a++) {
    // compact valid coordinates of axis a (order irrelevant: sorted next)
    if (t == 0) wpos[0] = 0;
    __syncthreads();
    for (int i = t; i < nt; i += 256)
      if (OV[i]) S[atomicAdd(&wpos[0], 1)] = O[3 * i + a];
    for (int i = nvalid + t; i < P; i += 256) S[i] = INFINITY;
    __syncthreads();
    block_bitonic_sort(S, P);
    if (sub) {
      // x_pt_map_sample = sorted[0], sorted[step], ... (Object.cc:780-794)
      float v[NP_MAXN / 256 + 1];
      int c = 0;
      for (int k = t; k < nsamp; k += 256) v[c++] = S[k * step];
      __syncthreads();
      c = 0;
      for (int k = t; k < nsamp; k += 256) S[k] = v[c++];
      __syncthreads();
    }
    int gt = 0, lt = 0, eq = 0;
    for (int i = t; i < mt; i += 256) {
      if (!FV[i]) continue;
      const float x = F[3 * i + a];
      int lo = 0, hi = nsamp;  // lower_bound
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (S[mid] < x) lo = mid + 1;
        else hi = mid;
      }
      int lo2 = lo, hi2 = nsamp;  // upper_bound
      while (lo2 < hi2) {
        const int mid = (lo2 + hi2) >> 1;
        if (S[mid] <= x) lo2 = mid + 1;
        else hi2 = mid;
      }
      gt += lo;
      eq += lo2 - lo;
      lt += nsamp - lo2;
    }
    gt = block_sum_int(gt, red);
    lt = block_sum_int(lt, red);
    eq = block_sum_int(eq, red);
    r.cnt_gt[a] = (float)gt;
    r.cnt_lt[a] = (float)lt;
    r.cnt_eq[a] = (float)eq;
    __syncthreads();
  }
  if (t == 0) {
    const int n = nsamp;
    r.n = n;
    const int mm = (int)((uint32_t)m * (uint32_t)(m + 1) / 2u);
    const int nn = (int)((uint32_t)n * (uint32_t)(n + 1) / 2u);
    int add = 0;
    const int prod = (int)((uint32_t)m * (uint32_t)n * (uint32_t)(m + n + 1));  // Q4
    const int q = prod / 12;
    const double base = __dmul_rn(__dmul_rn(0.5, (double)m), (double)(m + n + 1));
    const double spread = __dmul_rn(1.282, sqrt((double)q));
    r.r1 = (float)__dsub_rn(base, spread);
    r.r2 = (float)__dadd_rn(base, spread);
    for (int a = 0; a < 3; a++) {
      const float x = fadd(r.cnt_gt[a], (float)mm), y = fadd(r.cnt_lt[a], (float)nn);
      r.w[a] = fadd(fminf(x, y), fdiv(r.cnt_eq[a], 2.0f));
      if (r.w[a] > r.r1 && r.w[a] < r.r2) add++;
    }
    r.verdict = add == 3 ? 1 : 2;
    out[p] = r;
  }
}

// ---------------------------------------------------------------- rects
__device__ __forceinline__ void project_pt(const CamDev& c, const float* T, const float* P, float& u,
                                           float& v) {
  float pc[3];
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const float t = fadd(fadd(fmul(T[4 * r], P[0]), fmul(T[4 * r + 1], P[1])), fmul(T[4 * r + 2], P[2]));
    pc[r] = (float)((double)t + (double)T[4 * r + 3]);
  }
  const float invzc = (float)(1.0 / (double)pc[2]);
  u = fadd(fmul(fmul(c.fx, pc[0]), invzc), c.cx);
  v = fadd(fmul(fmul(c.fy, pc[1]), invzc), c.cy);
}

__global__ __launch_bounds__(256) void k_rects(CamDev cam, const float* __restrict__ Tg,
                                               const float* __restrict__ pts,
                                               const int* __restrict__ off,
                                               const int* __restrict__ len, int* __restrict__ rect,
                                               uint8_t* __restrict__ ok) {
  __shared__ float red[4][4];
  const int c = blockIdx.x, t = threadIdx.x;
  const int n = len[c];
  const float* P = pts + 3 * (long long)off[c];
  float T[16];
  for (int k = 0; k < 16; k++) T[k] = Tg[k];
  float xmn = INFINITY, xmx = -INFINITY, ymn = INFINITY, ymx = -INFINITY;
  for (int i = t; i < n; i += 256) {
    float u, v;
    project_pt(cam, T, P + 3 * i, u, v);
    xmn = fminf(xmn, u);
    xmx = fmaxf(xmx, u);
    ymn = fminf(ymn, v);
    ymx = fmaxf(ymx, v);
  }
  for (int o = 32; o > 0; o >>= 1) {
    xmn = fminf(xmn, __shfl_xor(xmn, o, 64));
    xmx = fmaxf(xmx, __shfl_xor(xmx, o, 64));
    ymn = fminf(ymn, __shfl_xor(ymn, o, 64));
    ymx = fmaxf(ymx, __shfl_xor(ymx, o, 64));
  }
  const int w = t >> 6;
  if ((t & 63) == 0) {
    red[w][0] = xmn;
    red[w][1] = xmx;
    red[w][2] = ymn;
    red[w][3] = ymx;
  }
  __syncthreads();
  if (t == 0) {
    for (int k = 1; k < 4; k++) {
      xmn = fminf(xmn, red[k][0]);
      xmx = fmaxf(xmx, red[k][1]);
      ymn = fminf(ymn, red[k][2]);
      ymx = fmaxf(ymx, red[k][3]);
    }
    if (n <= 0) {
      ok[c] = 0;
      return;
    }
    if (xmn < 0) xmn = 0;
    if (ymn < 0) ymn = 0;
    if (xmx > cam.maxX) xmx = cam.maxX;
    if (ymx > cam.maxY) ymx = cam.maxY;
    rect[4 * c] = (int)xmn;
    rect[4 * c + 1] = (int)ymn;
    rect[4 * c + 2] = (int)fsub(xmx, xmn);
    rect[4 * c + 3] = (int)fsub(ymx, ymn);
    ok[c] = 1;
  }
}

// ---------------------------------------------------------------- iForest
// Compiler barrier between the phases of a one-wave algorithm: a wave's LDS
// operations execute in program order, so only compiler reordering across
// lanes' data dependencies has to be prevented.
#define WAVE_FENCE() __asm__ volatile("" ::: "memory")

// std::mt19937 for one wave: state in LDS, tempered outputs buffered one per
// lane in a VGPR and handed out in stream order with v_readlane.
struct WaveRng {
  uint32_t* mt;  // LDS [624]
  int idx;       // next untempered state word (uniform)
  uint32_t buf;  // lane j: draw number (base + j) of the current chunk
  int bp, blen;  // uniform read position / valid length of buf

  __device__ void seed(uint32_t s) {
    if (lane_id() == 0) {
      uint32_t x = s;
      mt[0] = x;
      for (int i = 1; i < 624; i++) {
        x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)i;
        mt[i] = x;
      }
    }
    idx = 624;
    bp = blen = 0;
    WAVE_FENCE();
  }
  // libstdc++ _M_gen_rand in chunks of 64 words in increasing order: word k
  // reads k+1 (old) and (k+397)%624 (new for k >= 227, written by an earlier
  // chunk), exactly the in-place order of the sequential recurrence.
  __device__ void twist() {
    const int l = lane_id();
    for (int c0 = 0; c0 < 623; c0 += 64) {
      const int k = c0 + l;
      uint32_t nv = 0;
      if (k < 623) {
        const uint32_t y = (mt[k] & 0x80000000u) | (mt[k + 1] & 0x7fffffffu);
        nv = mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      }
      WAVE_FENCE();
      if (k < 623) mt[k] = nv;
      WAVE_FENCE();
    }
    if (l == 0) {
      const uint32_t y = (mt[623] & 0x80000000u) | (mt[0] & 0x7fffffffu);
      mt[623] = mt[396] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    WAVE_FENCE();
    idx = 0;
  }
  __device__ void refill() {
    if (idx >= 624) twist();
    blen = min(64, 624 - idx);
    const int l = lane_id();
    uint32_t y = l < blen ? mt[idx + l] : 0u;
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    buf = y;
    idx += blen;
    bp = 0;
  }
  __device__ uint32_t next() {
    if (bp >= blen) refill();
    return (uint32_t)__builtin_amdgcn_readlane((int)buf, bp++);
  }
  // uniform_int_distribution<uint32_t>(0, range-1) with a 32-bit URNG (Lemire)
  __device__ uint32_t lemire(uint32_t range) {
    uint64_t product = (uint64_t)next() * (uint64_t)range;
    uint32_t low = (uint32_t)product;
    if (low < range) {
      const uint32_t threshold = (uint32_t)(0u - range) % range;
      while (low < threshold) {
        product = (uint64_t)next() * (uint64_t)range;
        low = (uint32_t)product;
      }
    }
    return (uint32_t)(product >> 32);
  }
  // uniform_real_distribution<float>(a, b): generate_canonical<float, 24>
  __device__ float uniform_real(float a, float b) {
    float ret = fdiv(fmul((float)next(), 1.0f), 4294967296.0f);
    if (ret >= 1.0f) ret = __uint_as_float(0x3f7fffffu);  // nextafter(1, 0)
    return fadd(fmul(ret, fsub(b, a)), a);
  }
};

__device__ __forceinline__ double iforest_c(uint32_t n) {  // CalculateC, isolation_forest.h:97-118
  if (n > 2) {
    const double h = log((double)(n - 1)) + 0.5772156649;
    return __dsub_rn(2.0 * h, (2.0 * (double)(n - 1)) / (double)n);
  } else if (n == 2)
    return 1.0;
  return 0.0;
}

__host__ __device__ __forceinline__ size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }

// dynamic LDS carve of k_iforest_tree for clouds of <= N points, samples <= S
struct IfLds {
  size_t mt, b0, b1, nodes, right, shuf, total;
  __host__ __device__ IfLds(int N, int S) {
    mt = 0;
    b0 = al16(624 * 4);
    b1 = b0 + al16(12 * (size_t)S);
    nodes = b1 + al16(12 * (size_t)S);
    right = nodes + al16(8 * 2 * (size_t)S);
    const size_t build_end = right + al16(2 * 2 * (size_t)S);
    shuf = b1;  // shuffle scratch aliases B1 / nodes (dead until the build)
    const size_t shuf_end = shuf + al16(2 * (size_t)N) + 2 * al16(4 * ((size_t)N + 1)) + al16(2 * (size_t)N);
    total = build_end > shuf_end ? build_end : shuf_end;
  }
};

// One workgroup (4 waves) per (tree, cloud): IsolationTree::Build of
// isolation_forest.h:165-224,300-345 by wave 0 -- the libstdc++-11 draw stream
// replicated exactly -- then every wave walks the cloud's points through the
// tree (GetAnomalyScores' PathLength, :499-530); the per-(tree, point) path
// length is summed in tree order by k_iforest_sum.
//
// Sampling: std::shuffle of ids [0, n) (paired Lemire draws, stl_algo.h) is a
// Fisher-Yates sequence of positions p_j <= j.  The draws are taken 64 at a
// time in parallel; the swaps are not replayed: with v_j = j before step j
// the final content of position k is the last step that wrote k,
//   final(k)   = max{ j > k : p_j = k }   or else  f(p_k, k)  (k if p_k = k)
//   f(q, t)    = max{ j in (q, t) : p_j = q } or else f(p_q, q) (q if p_q = q, 0 at q = 0)
// resolved per lane from per-position writer lists.  Only the sample's set
// matters to the build (min/max, counts and membership are order-free), so
// the sampled coordinates are gathered straight into LDS and partitioned
// between two ping-pong buffers by depth parity.
__global__ __launch_bounds__(256) void k_iforest_tree(const float* __restrict__ pts,
                                                      const int* __restrict__ off,
                                                      const int* __restrict__ len,
                                                      const uint32_t* __restrict__ seeds,
                                                      const uint32_t* __restrict__ sample,
                                                      int maxN, int maxS, int npts_total,
                                                      double* __restrict__ contrib) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const IfLds L(maxN, maxS);
  uint32_t* mts = (uint32_t*)(smem + L.mt);
  float* B0 = (float*)(smem + L.b0);
  float* B1 = (float*)(smem + L.b1);
  uint2* nodes = (uint2*)(smem + L.nodes);
  uint16_t* right = (uint16_t*)(smem + L.right);
  __shared__ int s_nodes_bad;

  const int tr = blockIdx.x, c = blockIdx.y, ntrees = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = len[c];
  const int psi = (int)sample[c];
  const float* P = pts + 3 * (long long)off[c];
  double* out = contrib + (long long)tr * npts_total + off[c];
  if (n <= 0 || psi <= 0 || psi > n || n > maxN || psi > maxS) {
    for (int i = tid; i < n; i += blockDim.x) out[i] = __longlong_as_double(0x7ff8000000000000ll);
    return;
  }

  if (wave == 0) {
    WaveRng g;
    g.mt = mts;
    g.seed(seeds[tr]);
    // ---- shuffle draws: positions p[j], j = 1..n-1
    uint16_t* p = (uint16_t*)(smem + L.shuf);
    uint32_t* start = (uint32_t*)(smem + L.shuf + al16(2 * (size_t)n));
    uint32_t* fill = (uint32_t*)((unsigned char*)start + al16(4 * ((size_t)n + 1)));
    uint16_t* items = (uint16_t*)((unsigned char*)fill + al16(4 * ((size_t)n + 1)));
    const bool even = (n % 2) == 0;
    const int nsteps = even ? n / 2 : (n - 1) / 2;
    int s = 0;
    while (s < nsteps) {
      if (g.bp >= g.blen) g.refill();
      const int avail = min(g.blen - g.bp, nsteps - s);
      const uint32_t raw = (uint32_t)__shfl((int)g.buf, g.bp + lane, 64);
      const int step = s + lane;
      const bool single = even && step == 0;
      const uint32_t i = even ? 2u * step : 2u * step + 1u;
      const uint32_t sr = i + 1u;
      const uint32_t range = single ? 2u : sr * (sr + 1u);
      const uint64_t prod = (uint64_t)raw * range;
      const uint32_t low = (uint32_t)prod;
      bool rej = false;
      if (lane < avail && low < range) rej = low < (uint32_t)(0u - range) % range;
      const uint64_t rm = ballot(rej);
      const int r = rm ? (int)__ffsll((unsigned long long)rm) - 1 : avail;
      if (lane < r) {
        const uint32_t x = (uint32_t)(prod >> 32);
        if (single) {
          p[1] = (uint16_t)x;
        } else {
          p[i] = (uint16_t)(x / (sr + 1u));
          p[i + 1] = (uint16_t)(x % (sr + 1u));
        }
      }
      s += r;
      g.bp += r + (rm ? 1 : 0);  // a rejected draw is consumed; its step retries
    }
    WAVE_FENCE();
    // ---- writer lists: for position q the steps j > q with p_j = q
    for (int q = lane; q <= n; q += 64) start[q] = 0;
    WAVE_FENCE();
    for (int j = 1 + lane; j < n; j += 64) {
      const int q = p[j];
      if (q != j) atomicAdd(&start[q], 1u);
    }
    WAVE_FENCE();
    uint32_t carry = 0;
    for (int b = 0; b <= n; b += 64) {
      const int q = b + lane;
      const uint32_t v = q <= n ? start[q] : 0u;
      uint32_t inc = v;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)inc, o, 64);
        if (lane >= o) inc += t;
      }
      if (q <= n) {
        start[q] = carry + inc - v;
        fill[q] = carry + inc - v;
      }
      carry += (uint32_t)__shfl((int)inc, 63, 64);
    }
    WAVE_FENCE();
    for (int j = 1 + lane; j < n; j += 64) {
      const int q = p[j];
      if (q != j) items[atomicAdd(&fill[q], 1u)] = (uint16_t)j;
    }
    WAVE_FENCE();
    // ---- sample = final content of positions [0, psi): gather into B0
    for (int k = lane; k < psi; k += 64) {
      int q = k, t = n, id;
      while (true) {
        int m = -1;
        for (uint32_t e = start[q]; e < start[q + 1]; e++) {
          const int j = items[e];
          if (j < t && j > m) m = j;
        }
        if (m >= 0) {
          id = m;
          break;
        }
        if (q == 0) {
          id = 0;
          break;
        }
        const int pq = p[q];
        if (pq == q) {
          id = q;
          break;
        }
        t = q;
        q = pq;
      }
      B0[k] = P[3 * id];
      B0[psi + k] = P[3 * id + 1];
      B0[2 * psi + k] = P[3 * id + 2];
    }
    WAVE_FENCE();
    // ---- Node::Build in DFS pre-order; stack entry e lives in lane e
    const int maxDepth = (int)ceil(log2((double)psi));
    int sf = 0, sl = psi - 1, sd = 0, spar = -1;  // lane 0 = root
    int sp = 1, nn = 0, bad = 0;
    while (sp > 0) {
      sp--;
      const int first = __builtin_amdgcn_readlane(sf, sp);
      const int last = __builtin_amdgcn_readlane(sl, sp);
      const int depth = __builtin_amdgcn_readlane(sd, sp);
      const int parent = __builtin_amdgcn_readlane(spar, sp);
      const int me = nn++;
      if (parent >= 0 && lane == 0) right[parent] = (uint16_t)me;
      const int cnt = last - first + 1;
      if (cnt < 2 || depth >= maxDepth) {
        if (lane == 0) nodes[me] = make_uint2((uint32_t)cnt << 2, 0u);
        continue;
      }
      const uint32_t dim = g.lemire(3);
      const float* src = (depth & 1) ? B1 : B0;
      float* dst = (depth & 1) ? B0 : B1;
      float mn = INFINITY, mx = -INFINITY;
      for (int i = first + lane; i <= last; i += 64) {
        const float v = src[dim * psi + i];
        mn = fminf(mn, v);
        mx = fmaxf(mx, v);
      }
      for (int o = 32; o > 0; o >>= 1) {
        mn = fminf(mn, __shfl_xor(mn, o, 64));
        mx = fmaxf(mx, __shfl_xor(mx, o, 64));
      }
      if (mn == mx) {
        if (lane == 0) nodes[me] = make_uint2((uint32_t)cnt << 2, 0u);
        continue;
      }
      const float split = g.uniform_real(mn, mx);
      int nl = 0, nr = 0;
      for (int c0 = first; c0 <= last; c0 += 64) {
        const int i = c0 + lane;
        const bool in = i <= last;
        float x = 0.f, y = 0.f, z = 0.f;
        if (in) {
          x = src[i];
          y = src[psi + i];
          z = src[2 * psi + i];
        }
        const float v = dim == 0 ? x : (dim == 1 ? y : z);
        const bool lft = in && v < split;
        const uint64_t ml = ballot(lft), mr = ballot(in && !lft);
        if (in) {
          const int d = lft ? first + nl + popc64(ml & lanes_below())
                            : last - (nr + popc64(mr & lanes_below()));
          dst[d] = x;
          dst[psi + d] = y;
          dst[2 * psi + d] = z;
        }
        nl += popc64(ml);
        nr += popc64(mr);
      }
      WAVE_FENCE();
      if (nl == 0) {  // middle == first
        if (lane == 0) nodes[me] = make_uint2((uint32_t)cnt << 2, 0u);
        continue;
      }
      if (nr == 0) bad = 1;  // right range empty: Node::Build returns false
      if (lane == 0) nodes[me] = make_uint2(dim + 1u, __float_as_uint(split));
      const int middle = first + nl;
      // push right, then left: the left subtree is built (and draws) first
      if (lane == sp) {
        sf = middle;
        sl = last;
        sd = depth + 1;
        spar = me;
      }
      if (lane == sp + 1) {
        sf = first;
        sl = middle - 1;
        sd = depth + 1;
        spar = -1;
      }
      sp += 2;
      if (bad) break;
    }
    if (lane == 0) s_nodes_bad = bad;
  }
  __syncthreads();
  // ---- path length of every point of the cloud through this tree
  if (s_nodes_bad) {
    for (int i = tid; i < n; i += blockDim.x) out[i] = __longlong_as_double(0x7ff8000000000000ll);
    return;
  }
  for (int i = tid; i < n; i += blockDim.x) {
    const float x0 = P[3 * i], x1 = P[3 * i + 1], x2 = P[3 * i + 2];
    int k = 0, depth = 0;
    uint2 nd = nodes[0];
    while ((nd.x & 3u) != 0u) {
      const uint32_t d = nd.x & 3u;
      const float v = d == 1u ? x0 : (d == 2u ? x1 : x2);
      k = v < __uint_as_float(nd.y) ? k + 1 : (int)right[k];
      nd = nodes[k];
      depth++;
    }
    out[i] = (double)depth + iforest_c(nd.x >> 2);
  }
}

// score = 2^(-E[h(x)] / c(psi)), E[h] summed over the trees in order
__global__ __launch_bounds__(256) void k_iforest_sum(const int* __restrict__ off,
                                                     const int* __restrict__ len,
                                                     const uint32_t* __restrict__ sample,
                                                     int ntrees, int npts_total,
                                                     const double* __restrict__ contrib,
                                                     double* __restrict__ scores) {
  const int c = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= len[c]) return;
  const long long g = (long long)off[c] + i;
  double total = 0;
  for (int t = 0; t < ntrees; t++) total += contrib[(long long)t * npts_total + g];
  const double avg = total / (double)ntrees;
  scores[g] = pow(2.0, -avg / iforest_c(sample[c]));
}

// ================================================================ host
int AssocEngine::init(int device, int mp) {
  dev = device;
  max_points = mp;
  if (mp < 1 || mp > (1 << 22)) {
    set_error("eao_assoc_create: max_points out of range");
    return EAO_E_ARG;
  }
  EAO_HIP_CHECK(hipSetDevice(dev));
  EAO_HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  EAO_HIP_CHECK(hipMalloc(&d_pts, sizeof(float) * 3 * (size_t)mp * 2));
  EAO_HIP_CHECK(hipMalloc(&d_valid, (size_t)mp * 2));
  EAO_HIP_CHECK(hipMalloc(&d_meta, sizeof(int) * 8 * max_pairs));
  EAO_HIP_CHECK(hipMalloc(&d_np, sizeof(eao_np_stats) * max_pairs));
  EAO_HIP_CHECK(hipMalloc(&d_rect, sizeof(int) * 4 * max_pairs));
  EAO_HIP_CHECK(hipMalloc(&d_ok, max_pairs));
  EAO_HIP_CHECK(hipMalloc(&d_T, sizeof(float) * 16));
  EAO_HIP_CHECK(hipMalloc(&d_seeds, sizeof(uint32_t) * max_trees));
  EAO_HIP_CHECK(hipMalloc(&d_scores, sizeof(double) * (size_t)mp));
  EAO_HIP_CHECK(hipMalloc(&d_contrib, sizeof(double) * (size_t)mp * max_trees));
  hipDeviceProp_t prop;
  EAO_HIP_CHECK(hipGetDeviceProperties(&prop, dev));
  lds_limit = std::min((size_t)IF_LDS, (size_t)prop.sharedMemPerBlock) - 64;  // static LDS of the kernel
  return EAO_OK;
}

AssocEngine::~AssocEngine() {
  void* ptrs[] = {d_pts, d_valid, d_meta, d_np, d_rect, d_ok, d_T, d_seeds, d_scores, d_contrib};
  for (void* q : ptrs)
    if (q) (void)hipFree(q);
  if (stream) (void)hipStreamDestroy(stream);
}

int AssocEngine::np_batch(int npairs, const float* d_fp, const uint8_t* d_fv, const int* d_foff,
                          const int* d_flen, const float* d_op, const uint8_t* d_ov,
                          const int* d_ooff, const int* d_olen, eao_np_stats* d_out,
                          hipStream_t s) {
  if (npairs <= 0) return EAO_OK;
  hipLaunchKernelGGL(k_np_pairs, dim3(npairs), dim3(256), 0, s, d_fp, d_fv, d_foff, d_flen, d_op,
                     d_ov, d_ooff, d_olen, d_out);
  EAO_HIP_CHECK(hipGetLastError());
  return EAO_OK;
}

// IsolationForest::Build: per-tree seeds are the raw draws of mt19937(seed)
// (uniform_int<uint32>(0, UINT32_MAX), isolation_forest.h:463-474)
static void forest_seeds(uint32_t seed, uint32_t trees, std::vector<uint32_t>& out) {
  uint32_t mt[624];
  mt[0] = seed;
  for (int i = 1; i < 624; i++) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
  int idx = 624;
  out.resize(trees);
  for (uint32_t t = 0; t < trees; t++) {
    if (idx >= 624) {
      for (int k = 0; k < 624; k++) {
        uint32_t y = (mt[k] & 0x80000000u) | (mt[(k + 1) % 624] & 0x7fffffffu);
        mt[k] = mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      }
      idx = 0;
    }
    uint32_t y = mt[idx++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    out[t] = y;
  }
}

int AssocEngine::iforest_batch(int nclouds, const float* pts, const int* off, const int* len,
                               uint32_t trees, uint32_t seed, const uint32_t* d_sample,
                               double* scores, hipStream_t s, int maxN, int maxS, int npts_total) {
  if (nclouds <= 0) return EAO_OK;
  if ((int)trees > max_trees || nclouds > max_clouds || npts_total > max_points) {
    set_error("iforest: too many trees, clouds or points per call");
    return EAO_E_CAPACITY;
  }
  const IfLds L(maxN, maxS);
  if (maxN > IF_MAXN || L.total > lds_limit) {
    set_error("iforest: cloud exceeds the LDS-resident tree capacity");
    return EAO_E_CAPACITY;
  }
  if (seed != cached_seed || trees != cached_trees) {
    std::vector<uint32_t> sd;
    forest_seeds(seed, trees, sd);
    EAO_HIP_CHECK(hipMemcpyAsync(d_seeds, sd.data(), sizeof(uint32_t) * trees, hipMemcpyHostToDevice, s));
    cached_seed = seed;
    cached_trees = trees;
  }
  hipLaunchKernelGGL(k_iforest_tree, dim3(trees, nclouds), dim3(256), L.total, s, pts, off, len,
                     d_seeds, d_sample, maxN, maxS, npts_total, d_contrib);
  EAO_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_iforest_sum, dim3((maxN + 255) / 256, nclouds), dim3(256), 0, s, off, len,
                     d_sample, (int)trees, npts_total, (const double*)d_contrib, scores);
  EAO_HIP_CHECK(hipGetLastError());
  return EAO_OK;
}

int AssocEngine::rects(const CamDev& cam, const float* Tg, int nclouds, const float* pts,
                       const int* off, const int* len, int* rect, uint8_t* ok, hipStream_t s) {
  if (nclouds <= 0) return EAO_OK;
  hipLaunchKernelGGL(k_rects, dim3(nclouds), dim3(256), 0, s, cam, Tg, pts, off, len, rect, ok);
  EAO_HIP_CHECK(hipGetLastError());
  return EAO_OK;
}

}  // namespace eao

// ---------------------------------------------------------------- C ABI
using namespace eao;

struct eao_assoc {
  AssocEngine e;
};

namespace eao {
AssocEngine* assoc_engine(eao_assoc* a) { return &a->e; }
}  // namespace eao

extern "C" {

int eao_assoc_create(int device, int max_points, eao_assoc** out) {
  if (!out) return EAO_E_ARG;
  *out = nullptr;
  if (!eao_device_ok(device)) {
    set_error("no usable gfx950 device (the engine has no CPU fallback)");
    return EAO_E_NODEVICE;
  }
  eao_assoc* a = new eao_assoc();
  int rc = a->e.init(device, max_points);
  if (rc) {
    delete a;
    return rc;
  }
  *out = a;
  return EAO_OK;
}

int eao_assoc_destroy(eao_assoc* a) {
  delete a;
  return EAO_OK;
}

int eao_np_test_batch(eao_assoc* a, int npairs, const float* frame_pts, const uint8_t* frame_valid,
                      const int32_t* frame_off, const int32_t* frame_len, const float* obj_pts,
                      const uint8_t* obj_valid, const int32_t* obj_off, const int32_t* obj_len,
                      eao_np_stats* out) {
  if (!a || npairs < 0 || npairs > a->e.max_pairs) return EAO_E_ARG;
  if (npairs == 0) return EAO_OK;
  AssocEngine& e = a->e;
  int nf = 0, no = 0;
  for (int p = 0; p < npairs; p++) {
    nf = std::max(nf, frame_off[p] + frame_len[p]);
    no = std::max(no, obj_off[p] + obj_len[p]);
  }
  if (nf > e.max_points || no > e.max_points) return EAO_E_CAPACITY;
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  hipStream_t s = e.stream;
  float* dF = e.d_pts;
  float* dO = e.d_pts + 3 * (size_t)e.max_points;
  uint8_t* vF = e.d_valid;
  uint8_t* vO = e.d_valid + e.max_points;
  EAO_HIP_CHECK(hipMemcpyAsync(dF, frame_pts, sizeof(float) * 3 * nf, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(dO, obj_pts, sizeof(float) * 3 * no, hipMemcpyHostToDevice, s));
  if (frame_valid) EAO_HIP_CHECK(hipMemcpyAsync(vF, frame_valid, nf, hipMemcpyHostToDevice, s));
  else EAO_HIP_CHECK(hipMemsetAsync(vF, 1, nf, s));
  if (obj_valid) EAO_HIP_CHECK(hipMemcpyAsync(vO, obj_valid, no, hipMemcpyHostToDevice, s));
  else EAO_HIP_CHECK(hipMemsetAsync(vO, 1, no, s));
  int* m = e.d_meta;
  EAO_HIP_CHECK(hipMemcpyAsync(m, frame_off, sizeof(int) * npairs, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(m + e.max_pairs, frame_len, sizeof(int) * npairs, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(m + 2 * e.max_pairs, obj_off, sizeof(int) * npairs, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(m + 3 * e.max_pairs, obj_len, sizeof(int) * npairs, hipMemcpyHostToDevice, s));
  int rc = e.np_batch(npairs, dF, vF, m, m + e.max_pairs, dO, vO, m + 2 * e.max_pairs,
                      m + 3 * e.max_pairs, e.d_np, s);
  if (rc) return rc;
  EAO_HIP_CHECK(hipMemcpyAsync(out, e.d_np, sizeof(eao_np_stats) * npairs, hipMemcpyDeviceToHost, s));
  EAO_HIP_CHECK(hipStreamSynchronize(s));
  return EAO_OK;
}

int eao_iforest_scores_batch(eao_assoc* a, int nclouds, const float* pts, const int32_t* off,
                             const int32_t* len, uint32_t trees, uint32_t seed,
                             const uint32_t* sample_size, double* scores) {
  if (!a || nclouds < 0 || nclouds > a->e.max_clouds) return EAO_E_ARG;
  if (nclouds == 0) return EAO_OK;
  AssocEngine& e = a->e;
  int np = 0, maxN = 0, maxS = 0;
  for (int c = 0; c < nclouds; c++) {
    np = std::max(np, off[c] + len[c]);
    maxN = std::max(maxN, len[c]);
    maxS = std::max(maxS, (int)sample_size[c]);
    if (len[c] > IF_MAXN || len[c] > e.max_points) return EAO_E_CAPACITY;
    if (sample_size[c] == 0 || (int)sample_size[c] > len[c]) return EAO_E_ARG;  // Build() fails
  }
  if (np > e.max_points) return EAO_E_CAPACITY;
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  hipStream_t s = e.stream;
  int* m = e.d_meta;
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_pts, pts, sizeof(float) * 3 * np, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(m, off, sizeof(int) * nclouds, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(m + e.max_pairs, len, sizeof(int) * nclouds, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(m + 2 * e.max_pairs, sample_size, sizeof(int) * nclouds, hipMemcpyHostToDevice, s));
  int rc = e.iforest_batch(nclouds, e.d_pts, m, m + e.max_pairs, trees, seed,
                           (const uint32_t*)(m + 2 * e.max_pairs), e.d_scores, s, maxN, maxS, np);
  if (rc) return rc;
  EAO_HIP_CHECK(hipMemcpyAsync(scores, e.d_scores, sizeof(double) * np, hipMemcpyDeviceToHost, s));
  EAO_HIP_CHECK(hipStreamSynchronize(s));
  return EAO_OK;
}

int eao_project_rects(eao_assoc* a, const eao_camera* cam, const float* Tcw, int nclouds,
                      const float* pts, const int32_t* off, const int32_t* len, int32_t* rect,
                      uint8_t* ok) {
  if (!a || !cam || !Tcw || nclouds < 0 || nclouds > a->e.max_pairs) return EAO_E_ARG;
  if (nclouds == 0) return EAO_OK;
  AssocEngine& e = a->e;
  int np = 0;
  for (int c = 0; c < nclouds; c++) np = std::max(np, off[c] + len[c]);
  if (np > e.max_points) return EAO_E_CAPACITY;
  EAO_HIP_CHECK(hipSetDevice(e.dev));
  hipStream_t s = e.stream;
  int* m = e.d_meta;
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_pts, pts, sizeof(float) * 3 * np, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(m, off, sizeof(int) * nclouds, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(m + e.max_pairs, len, sizeof(int) * nclouds, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_T, Tcw, sizeof(float) * 16, hipMemcpyHostToDevice, s));
  EAO_HIP_CHECK(hipMemcpyAsync(e.d_rect, rect, sizeof(int) * 4 * nclouds, hipMemcpyHostToDevice, s));
  int rc = e.rects(make_cam(*cam), e.d_T, nclouds, e.d_pts, m, m + e.max_pairs, e.d_rect, e.d_ok, s);
  if (rc) return rc;
  EAO_HIP_CHECK(hipMemcpyAsync(rect, e.d_rect, sizeof(int) * 4 * nclouds, hipMemcpyDeviceToHost, s));
  EAO_HIP_CHECK(hipMemcpyAsync(ok, e.d_ok, nclouds, hipMemcpyDeviceToHost, s));
  EAO_HIP_CHECK(hipStreamSynchronize(s));
  return EAO_OK;
}

}  // extern "C"
