// Micro-benchmark of the rank-space prologue of the isolation-forest subtree build
// (iforest_wave.h rank_subtree): per dimension, the rank of every item, the item at
// every rank and the sorted key at every rank, for <= 64 items held one per lane.
//   A: wave_sort3 (bitonic over the 64 lanes, 64-bit keys value << 32 | lane) + ds_permute
//   B: ranks by counting (rank = #smaller + #equal at a lower lane), then ds_permute
//   C: bitonic over the next power of two >= cnt lanes only (8, 16, 32 or 64)
// All must agree on the ranks of the cnt items, the items at ranks < cnt and their sorted
// keys (ties broken by lane). Development aid only.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I../../eao-slam_amd/csrc rank_bench.hip -o rank_bench
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "iforest_wave.h"

using namespace eao;

__device__ __forceinline__ void rank_count3(int kx, int ky, int kz, int& rx, int& ry, int& rz) {
  const int lane = lane_id();
  rx = ry = rz = 0;
#pragma unroll 16
  for (int j = 0; j < 64; j++) {
    const int ax = __builtin_amdgcn_readlane(kx, j), ay = __builtin_amdgcn_readlane(ky, j),
              az = __builtin_amdgcn_readlane(kz, j);
    rx += (ax < kx || (ax == kx && j < lane)) ? 1 : 0;
    ry += (ay < ky || (ay == ky && j < lane)) ? 1 : 0;
    rz += (az < kz || (az == kz && j < lane)) ? 1 : 0;
  }
}

template <int MODE>
__global__ void k_bench(const int* keys, int cnt, int reps, int* out, unsigned long long* cyc) {
  const int lane = threadIdx.x;
  const bool has = lane < cnt;
  const int kx = has ? keys[lane] : INT_MAX, ky = has ? keys[64 + lane] : INT_MAX,
            kz = has ? keys[128 + lane] : INT_MAX;
  int px = 0, py = 0, pz = 0, rx = 0, ry = 0, rz = 0, sx = 0, sy = 0, sz = 0;
  const unsigned long long t0 = clock64();
  for (int r = 0; r < reps; r++) {
    const int jx = kx + (r & 1) * 0, jy = ky, jz = kz;  // same keys each rep (kept live)
    if (MODE == 0 || MODE == 2) {
      auto sk64 = [&](int k) { return ((uint64_t)((uint32_t)k ^ 0x80000000u) << 32) | (uint32_t)lane; };
      uint64_t vx = sk64(jx), vy = sk64(jy), vz = sk64(jz);
      if (MODE == 0 || cnt > 32)
        wave_sort3(vx, vy, vz);
      else if (cnt > 16)
        bitonic_sort3<32>(vx, vy, vz);
      else if (cnt > 8)
        bitonic_sort3<16>(vx, vy, vz);
      else
        bitonic_sort3<8>(vx, vy, vz);
      sx = (int)((uint32_t)(vx >> 32) ^ 0x80000000u), px = (int)(uint32_t)vx;
      sy = (int)((uint32_t)(vy >> 32) ^ 0x80000000u), py = (int)(uint32_t)vy;
      sz = (int)((uint32_t)(vz >> 32) ^ 0x80000000u), pz = (int)(uint32_t)vz;
      rx = __builtin_amdgcn_ds_permute(px << 2, lane);
      ry = __builtin_amdgcn_ds_permute(py << 2, lane);
      rz = __builtin_amdgcn_ds_permute(pz << 2, lane);
    } else {
      rank_count3(jx, jy, jz, rx, ry, rz);
      px = __builtin_amdgcn_ds_permute(rx << 2, lane);
      py = __builtin_amdgcn_ds_permute(ry << 2, lane);
      pz = __builtin_amdgcn_ds_permute(rz << 2, lane);
      sx = __builtin_amdgcn_ds_permute(rx << 2, jx);
      sy = __builtin_amdgcn_ds_permute(ry << 2, jy);
      sz = __builtin_amdgcn_ds_permute(rz << 2, jz);
    }
  }
  const unsigned long long t1 = clock64();
  const int o[9] = {px, py, pz, rx, ry, rz, sx, sy, sz};
  for (int k = 0; k < 9; k++) out[64 * k + lane] = o[k];
  if (lane == 0) *cyc = (t1 - t0) / reps;
}

int main() {
  int *d_keys, *d_out;
  unsigned long long* d_cyc;
  hipMalloc(&d_keys, 192 * sizeof(int));
  hipMalloc(&d_out, 2 * 576 * sizeof(int));
  hipMalloc(&d_cyc, 2 * sizeof(unsigned long long));
  srand(7);
  int bad = 0;
  for (int cnt : {64, 63, 40, 16, 8}) {
    for (int ties : {0, 1}) {
      std::vector<int> keys(192);
      for (int i = 0; i < 192; i++) keys[i] = ties ? (rand() % 7) - 3 : (int)(rand() ^ (rand() << 16));
      hipMemcpy(d_keys, keys.data(), 192 * sizeof(int), hipMemcpyHostToDevice);
      hipLaunchKernelGGL(k_bench<0>, dim3(1), dim3(64), 0, 0, d_keys, cnt, 200, d_out, d_cyc);
      hipLaunchKernelGGL(k_bench<2>, dim3(1), dim3(64), 0, 0, d_keys, cnt, 200, d_out + 576, d_cyc + 1);
      std::vector<int> o(1152);
      unsigned long long c[2];
      hipMemcpy(o.data(), d_out, 1152 * sizeof(int), hipMemcpyDeviceToHost);
      hipMemcpy(c, d_cyc, sizeof c, hipMemcpyDeviceToHost);
      int diff = 0;
      for (int k = 0; k < 9; k++)
        for (int l = 0; l < cnt; l++) diff += o[64 * k + l] != o[576 + 64 * k + l];
      bad += diff;
      printf("cnt %2d ties %d: full sort %6llu cyc, sort of the next pow2 lanes %6llu cyc, differ: %d\n", cnt, ties,
             c[0], c[1], diff);
    }
  }
  printf(bad ? "MISMATCH\n" : "identical\n");
  return bad ? 1 : 0;
}
