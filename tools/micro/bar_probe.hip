// Probe (development aid): can the host write device memory directly (large-BAR / fine-grained
// device allocations), and what does a small host->device hand-off cost each way? For each
// allocation kind: the host pointer attribute, a host memcpy of 16 KB into it, and a one-block
// kernel that sums it; versus pinned host memory read by the kernel over PCIe.
//   hipcc --offload-arch=gfx950 -O2 tools/micro/bar_probe.hip -o tools/micro/_build/bar_probe
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void k_sum(const unsigned* __restrict__ p, int n, unsigned* out) {
  unsigned s = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += p[i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  __shared__ unsigned w[16];
  if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned t = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); k++) t += w[k];
    *out = t;
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const int n = 4096;  // 16 KB
  std::vector<unsigned> src(n);
  unsigned ref = 0;
  for (int i = 0; i < n; i++) ref += (src[i] = 2654435761u * i + 7);
  unsigned* out = nullptr;
  hipHostMalloc((void**)&out, 64, 0);
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  struct Kind {
    const char* name;
    unsigned flags;
    int host;
  } kinds[] = {{"hipMalloc", 0, 0},
               {"hipExtMallocWithFlags(Finegrained)", hipDeviceMallocFinegrained, 0},
               {"hipExtMallocWithFlags(Uncached)", hipDeviceMallocUncached, 0},
               {"hipHostMalloc (pinned host)", 0, 1}};
  for (const Kind& k : kinds) {
    void* p = nullptr;
    hipError_t e;
    if (k.host) e = hipHostMalloc(&p, n * 4, 0);
    else if (k.flags == 0) e = hipMalloc(&p, n * 4);
    else e = hipExtMallocWithFlags(&p, n * 4, k.flags);
    if (e != hipSuccess) {
      printf("%-40s alloc failed: %s\n", k.name, hipGetErrorString(e));
      continue;
    }
    hipPointerAttribute_t a;
    std::memset(&a, 0, sizeof(a));
    e = hipPointerGetAttributes(&a, p);
    printf("%-40s attr %s type %d hostPointer %p devicePointer %p\n", k.name, hipGetErrorString(e), (int)a.type,
           a.hostPointer, a.devicePointer);
    void* hp = k.host ? p : a.hostPointer;
    if (!hp) {
      printf("%-40s no host mapping\n", k.name);
      if (k.host) hipHostFree(p); else hipFree(p);
      continue;
    }
    // host write then kernel read, timed as a hand-off (20 repetitions, median-ish: min)
    double best_w = 1e9, best_rt = 1e9;
    bool ok = true;
    for (int r = 0; r < 20; r++) {
      src[0] = (unsigned)r;
      unsigned ref_r = ref - (2654435761u * 0 + 7) + (unsigned)r;
      const double t0 = now_us();
      std::memcpy(hp, src.data(), n * 4);
      std::atomic_thread_fence(std::memory_order_seq_cst);
      const double t1 = now_us();
      *out = 0;
      hipLaunchKernelGGL(k_sum, dim3(1), dim3(1024), 0, s, (const unsigned*)p, n, out);
      hipStreamSynchronize(s);
      const double t2 = now_us();
      if (*out != ref_r) ok = false;
      best_w = std::min(best_w, t1 - t0);
      best_rt = std::min(best_rt, t2 - t0);
    }
    printf("%-40s host write 16 KB %.2f us | write + kernel + sync %.1f us | %s\n", k.name, best_w, best_rt,
           ok ? "sum ok" : "SUM WRONG");
    if (k.host) hipHostFree(p); else hipFree(p);
  }
  // reference: hipMemcpyAsync H2D from pinned + kernel
  {
    void *h = nullptr, *d = nullptr;
    hipHostMalloc(&h, n * 4, 0);
    hipMalloc(&d, n * 4);
    double best = 1e9;
    for (int r = 0; r < 20; r++) {
      const double t0 = now_us();
      std::memcpy(h, src.data(), n * 4);
      hipMemcpyAsync(d, h, n * 4, hipMemcpyHostToDevice, s);
      hipLaunchKernelGGL(k_sum, dim3(1), dim3(1024), 0, s, (const unsigned*)d, n, out);
      hipStreamSynchronize(s);
      best = std::min(best, now_us() - t0);
    }
    printf("%-40s memcpy + H2D DMA + kernel + sync %.1f us\n", "pinned + hipMemcpyAsync", best);
  }
  return 0;
}
