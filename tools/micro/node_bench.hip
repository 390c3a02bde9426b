// Micro-benchmark of the isolation-forest register-path node step (one wave,
// rank-space subtree build of assoc.hip) with ablations, to find where the
// cycles of a node go. Development aid only.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I../../eao-slam_amd/csrc node_bench.hip -o node_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "iforest_wave.h"

using namespace eao;

enum { NO_LDS = 1, CHEAP_RNG = 2, INT_SPLIT = 4, NO_CONVERT = 8, NO_STACK = 16 };

template <int MODE>
__global__ void k_bench(const int* keys, int cnt, int reps, unsigned long long* out) {
  __shared__ uint32_t mts[624];
  __shared__ uint2 nodes[256];
  __shared__ uint16_t right[256];
  const int lane = threadIdx.x;
  for (int i = lane; i < 624; i += 64) mts[i] = 0x9e3779b9u * (i + 1);
  __syncthreads();
  WaveRng g;
  g.mt = mts;
  g.idx = 0;
  g.bp = g.blen = 0;
  uint32_t cheap = 12345u;
  auto draw = [&]() -> uint32_t {
    if (MODE & CHEAP_RNG) {
      cheap = cheap * 1664525u + 1013904223u;
      return cheap;
    }
    return g.next();
  };
  const bool has = lane < cnt;
  const int kx = has ? keys[lane] : INT_MAX, ky = has ? keys[64 + lane] : INT_MAX,
            kz = has ? keys[128 + lane] : INT_MAX;
  auto sk64 = [&](int k) { return ((uint64_t)((uint32_t)k ^ 0x80000000u) << 32) | (uint32_t)lane; };
  uint64_t vx = sk64(kx), vy = sk64(ky), vz = sk64(kz);
  const unsigned long long t0 = clock64();
  wave_sort3(vx, vy, vz);
  const int sx = (int)((uint32_t)(vx >> 32) ^ 0x80000000u), px = (int)(uint32_t)vx;
  const int sy = (int)((uint32_t)(vy >> 32) ^ 0x80000000u), py = (int)(uint32_t)vy;
  const int sz = (int)((uint32_t)(vz >> 32) ^ 0x80000000u), pz = (int)(uint32_t)vz;
  const int rx = __builtin_amdgcn_ds_permute(px << 2, lane);
  const int ry = __builtin_amdgcn_ds_permute(py << 2, lane);
  const int rz = __builtin_amdgcn_ds_permute(pz << 2, lane);
  const unsigned long long t1 = clock64();
  const uint64_t all = cnt == 64 ? ~0ull : ((1ull << cnt) - 1ull);
  const int maxDepth = 7;
  long long nn_total = 0;
  int sink = 0;
  for (int r = 0; r < reps; r++) {
    uint64_t mX = all, mY = all, mZ = all;
    int d = 0, node = 0, ssp = 0, nn = 1;
    int q0 = 0, q1 = 0, q2 = 0, q3 = 0, q4 = 0, q5 = 0, q6 = 0, q7 = 0;
    while (true) {
      const int cn = __builtin_popcountll(mX);
      bool leaf = cn < 2 || d >= maxDepth;
      if (!leaf) {
        uint32_t dim;
        {
          uint64_t product = (uint64_t)draw() * 3ull;
          uint32_t low = (uint32_t)product;
          if (low < 3u)
            while (low < 1u) {
              product = (uint64_t)draw() * 3ull;
              low = (uint32_t)product;
            }
          dim = (uint32_t)(product >> 32);
        }
        const uint64_t md = dim == 0 ? mX : (dim == 1 ? mY : mZ);
        const int sk = dim == 0 ? sx : (dim == 1 ? sy : sz);
        const int lo = __builtin_ctzll(md), hi = 63 - __builtin_clzll(md);
        const int mn = __builtin_amdgcn_readlane(sk, lo), mx = __builtin_amdgcn_readlane(sk, hi);
        if (mn == mx) {
          leaf = true;
        } else {
          int ks;
          float split = 0.f;
          if (MODE & INT_SPLIT) {
            ks = mn + (int)((uint32_t)(mx - mn) / 2u) + (int)(draw() & 1u);
          } else {
            float ret = fmul((float)draw(), 0x1p-32f);
            if (ret >= 1.0f) ret = __uint_as_float(0x3f7fffffu);
            split = fadd(fmul(ret, fsub(kfloat(mx), kfloat(mn))), kfloat(mn));
            ks = __builtin_amdgcn_readfirstlane(fkey(split));
          }
          const uint64_t lm = md & ballot(sk < ks);
          if (lm == 0) {
            leaf = true;
          } else {
            if (!(MODE & NO_LDS) && lane == 0) nodes[node & 255] = make_uint2(dim + 1u, __float_as_uint(split));
            uint64_t lx = lm, ly = lm, lz = lm;
            if (!(MODE & NO_CONVERT)) {
              const int rk = dim == 0 ? rx : (dim == 1 ? ry : rz);
              const uint64_t il = ballot((lm >> rk) & 1ull);
              lx = dim == 0 ? lm : ballot((il >> px) & 1ull);
              ly = dim == 1 ? lm : ballot((il >> py) & 1ull);
              lz = dim == 2 ? lm : ballot((il >> pz) & 1ull);
            }
            const uint64_t ux = mX & ~lx, uy = mY & ~ly, uz = mZ & ~lz;
            if (!(MODE & NO_STACK)) {
              writelane(q0, (int)(uint32_t)ux, ssp);
              writelane(q1, (int)(uint32_t)(ux >> 32), ssp);
              writelane(q2, (int)(uint32_t)uy, ssp);
              writelane(q3, (int)(uint32_t)(uy >> 32), ssp);
              writelane(q4, (int)(uint32_t)uz, ssp);
              writelane(q5, (int)(uint32_t)(uz >> 32), ssp);
              writelane(q6, d + 1, ssp);
              writelane(q7, node, ssp);
              ssp++;
            }
            mX = lx;
            mY = ly;
            mZ = lz;
            d++;
            node = nn++;
            continue;
          }
        }
      }
      if (!(MODE & NO_LDS) && lane == 0) nodes[node & 255] = make_uint2((uint32_t)cn << 2, 0u);
      if (ssp == 0) break;
      ssp--;
      mX = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(q0, ssp) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(q1, ssp) << 32);
      mY = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(q2, ssp) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(q3, ssp) << 32);
      mZ = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(q4, ssp) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(q5, ssp) << 32);
      d = __builtin_amdgcn_readlane(q6, ssp);
      const int par = __builtin_amdgcn_readlane(q7, ssp);
      node = nn++;
      if (!(MODE & NO_LDS) && lane == 0) right[par & 255] = (uint16_t)node;
    }
    nn_total += nn;
    sink += node;
  }
  const unsigned long long t2 = clock64();
  if (lane == 0) {
    out[0] = t1 - t0;
    out[1] = t2 - t1;
    out[2] = nn_total;
    out[3] = sink + nodes[3].x + right[5];
  }
}

// the kernel's own subtree builder (iforest_wave.h), sort included
__global__ void k_subtree(const int* keys, int cnt, int maxDepth, int reps, unsigned long long* out) {
  __shared__ uint32_t mts[624];
  __shared__ uint2 nodes[256];
  __shared__ uint16_t ndep[256];
  const int lane = threadIdx.x;
  for (int i = lane; i < 624; i += 64) mts[i] = 0x9e3779b9u * (i + 1);
  __syncthreads();
  WaveRng g;
  g.mt = mts;
  g.idx = 0;
  g.bp = g.blen = 0;
  const int kx = keys[lane], ky = keys[64 + lane], kz = keys[128 + lane];
  long long total = 0;
  int bad = 0;
  const unsigned long long t0 = clock64();
  for (int r = 0; r < reps; r++) {
    int nn = 1;
    bad |= rank_subtree(g, kx, ky, kz, cnt, 0, maxDepth, 0, nn, nodes);
    total += nn;
  }
  const unsigned long long t1 = clock64();
  if (lane == 0) {
    out[0] = t1 - t0;
    out[1] = total;
    out[2] = bad + nodes[5].x + ndep[3];
  }
}

__global__ void k_sort(const int* keys, int reps, unsigned long long* out) {
  const int lane = threadIdx.x;
  uint64_t a = ((uint64_t)(uint32_t)keys[lane] << 32) | lane, b = ((uint64_t)(uint32_t)keys[64 + lane] << 32) | lane,
           c = ((uint64_t)(uint32_t)keys[128 + lane] << 32) | lane;
  const unsigned long long t0 = clock64();
  for (int r = 0; r < reps; r++) {
    wave_sort3(a, b, c);
    a ^= (uint64_t)(r & 1) << 40;  // keep the chain dependent
    b ^= (uint64_t)(r & 2) << 40;
    c ^= (uint64_t)(r & 1) << 41;
  }
  const unsigned long long t1 = clock64();
  if (lane == 0) {
    out[0] = t1 - t0;
    out[1] = a + b + c;
  }
}

static void run_sort(const int* d_keys, unsigned long long* d_out) {
  unsigned long long h[2];
  for (int w = 0; w < 2; w++) hipLaunchKernelGGL(k_sort, dim3(1), dim3(64), 0, 0, d_keys, 200, d_out);
  (void)hipMemcpy(h, d_out, sizeof h, hipMemcpyDeviceToHost);
  printf("wave_sort3: %.0f cyc\n", (double)h[0] / 200);
}

static void run_subtree(const int* d_keys, int cnt, int maxDepth, unsigned long long* d_out) {
  unsigned long long h[3];
  for (int w = 0; w < 2; w++)
    hipLaunchKernelGGL(k_subtree, dim3(1), dim3(64), 0, 0, d_keys, cnt, maxDepth, 200, d_out);
  (void)hipMemcpy(h, d_out, sizeof h, hipMemcpyDeviceToHost);
  printf("rank_subtree cnt %2d depth %d: %.0f cyc/subtree, %.1f nodes, %.1f cyc/node\n", cnt, maxDepth,
         (double)h[0] / 200, (double)h[1] / 200, (double)h[0] / h[1]);
}

template <int MODE>
static void run(const char* name, const int* d_keys, int cnt, unsigned long long* d_out) {
  unsigned long long h[4];
  for (int w = 0; w < 2; w++) hipLaunchKernelGGL(k_bench<MODE>, dim3(1), dim3(64), 0, 0, d_keys, cnt, 200, d_out);
  (void)hipMemcpy(h, d_out, sizeof h, hipMemcpyDeviceToHost);
  printf("%-28s cnt %2d  sort %6llu cyc  nodes %7llu  %.1f cyc/node\n", name, cnt, h[0], h[2], (double)h[1] / h[2]);
}

int main() {
  std::vector<int> keys(192);
  srand(7);
  for (int& k : keys) k = rand() % 100000;
  int* d_keys;
  unsigned long long* d_out;
  (void)hipMalloc(&d_keys, keys.size() * 4);
  (void)hipMalloc(&d_out, 64);
  (void)hipMemcpy(d_keys, keys.data(), keys.size() * 4, hipMemcpyHostToDevice);
  run_sort(d_keys, d_out);
  run_subtree(d_keys, 64, 1, d_out);
  run_subtree(d_keys, 64, 2, d_out);
  for (int cnt : {64, 40, 16, 8}) run_subtree(d_keys, cnt, 7, d_out);
  run_subtree(d_keys, 64, 12, d_out);
  for (int cnt : {64, 40}) {
    run<0>("full", d_keys, cnt, d_out);
    run<NO_LDS>("no LDS writes", d_keys, cnt, d_out);
    run<CHEAP_RNG>("cheap RNG", d_keys, cnt, d_out);
    run<INT_SPLIT>("int split", d_keys, cnt, d_out);
    run<NO_CONVERT>("no mask conversion", d_keys, cnt, d_out);
    run<NO_STACK>("no stack push", d_keys, cnt, d_out);
    run<CHEAP_RNG | INT_SPLIT>("cheap RNG + int split", d_keys, cnt, d_out);
    run<CHEAP_RNG | INT_SPLIT | NO_LDS | NO_CONVERT>("skeleton", d_keys, cnt, d_out);
  }
  return 0;
}
