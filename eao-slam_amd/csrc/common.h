// common.h -- shared host/device definitions of the MI355X EAO engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <cstring>
#include <string>

namespace eao {

// last error text (thread-local), exposed as eao_last_error()
void set_error(const std::string& s);

#define EAO_HIP_CHECK(expr)                                                              \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess) {                                                              \
      ::eao::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));               \
      return EAO_E_HIP;                                                                  \
    }                                                                                    \
  } while (0)

constexpr int kWave = 64;

// cvRound semantics (round half to even) -- SURVEY appendix A
__device__ __forceinline__ int dev_round(float v) { return __float2int_rn(v); }

// exact float ops, no contraction
__device__ __forceinline__ float fmul(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float fadd(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float fsub(float a, float b) { return __fsub_rn(a, b); }
__device__ __forceinline__ float fdiv(float a, float b) { return __fdiv_rn(a, b); }

// candidate keypoint packing: x (12b) | y (12b) << 12 | FAST score (8b) << 24
__host__ __device__ __forceinline__ uint32_t pack_kp(int x, int y, int s) {
  return (uint32_t)x | ((uint32_t)y << 12) | ((uint32_t)s << 24);
}
__host__ __device__ __forceinline__ int kp_x(uint32_t p) { return (int)(p & 0xfffu); }
__host__ __device__ __forceinline__ int kp_y(uint32_t p) { return (int)((p >> 12) & 0xfffu); }
__host__ __device__ __forceinline__ int kp_s(uint32_t p) { return (int)(p >> 24); }

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ int popc64(uint64_t m) { return __popcll(m); }
__device__ __forceinline__ uint64_t lanes_below() {
  int l = lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int wave_max_int(int v) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wave_min_int(int v) {
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}

// Staging of the C ABI's host-buffer (single-call) entry points: a pinned host image and its
// device mirror. Inputs are packed 16-byte aligned into the pinned image and go over in one
// DMA copy (a pageable source would be bounced through a driver buffer, copy by copy); outputs
// come back into pinned memory. Returns EAO status codes (the including file defines them).
struct HostStage {
  unsigned char* h = nullptr;
  unsigned char* d = nullptr;
  size_t cap = 0, used = 0;
  static size_t al(size_t x) { return (x + 15) & ~(size_t)15; }
  hipError_t reserve(size_t bytes) {
    used = 0;
    if (bytes <= cap) return hipSuccess;
    release();
    const size_t c = al(bytes + bytes / 4 + 4096);
    hipError_t e = hipHostMalloc((void**)&h, c, 0);
    if (e == hipSuccess) e = hipMalloc((void**)&d, c);
    if (e == hipSuccess) cap = c;
    return e;
  }
  // the next 16-aligned slot of `bytes`, filled from src when given: its offset
  size_t put(const void* src, size_t bytes) {
    const size_t at = used;
    if (src && bytes) std::memcpy(h + at, src, bytes);
    used = al(at + bytes);
    return at;
  }
  template <class T>
  T* dev(size_t off) const { return (T*)(d + off); }
  hipError_t upload(hipStream_t s) const { return used ? hipMemcpyAsync(d, h, used, hipMemcpyHostToDevice, s) : hipSuccess; }
  void release() {
    if (h) (void)hipHostFree(h);
    if (d) (void)hipFree(d);
    h = d = nullptr;
    cap = used = 0;
  }
  ~HostStage() { release(); }
};

}  // namespace eao
