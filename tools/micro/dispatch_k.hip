// Kernels of tools/micro/dispatch_lat.cpp (development aid): built twice, into the HIP
// program and as a stand-alone gfx950 code object that the HSA path loads itself.
// Neither reads blockDim / gridDim (no implicit kernel arguments needed).
#include <hip/hip_runtime.h>
#include <cstdint>

extern "C" __global__ void __launch_bounds__(64) k_nop(uint32_t* p) {
  if (threadIdx.x == 0 && p && blockIdx.x == 0xffffff) p[0] = 1;
}

// the flag store goes to pinned host memory at system scope: the host spins on it
extern "C" __global__ void __launch_bounds__(64) k_flag(uint32_t* flag, uint32_t v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// a kernel of a few microseconds (one wave spins on s_memtime): the producer of a chain
extern "C" __global__ void __launch_bounds__(64) k_busy(uint32_t* p, uint32_t cycles) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) {
  }
  if (threadIdx.x == 0 && p && blockIdx.x == 0xffffff) p[0] = 1;
}
