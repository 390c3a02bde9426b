// Host-side cost of the HIP calls the association engine issues per launch
// (small pinned copies, launches, events, syncs) on this box.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#define CK(x) do { if ((x) != hipSuccess) { printf("err %s line %d\n", #x, __LINE__); return 1; } } while (0)
__global__ void k_nop(int* p) { if (threadIdx.x == 0 && p) p[blockIdx.x] = 1; }
__global__ void k_write_host(double* h, int n) { int i = blockIdx.x * blockDim.x + threadIdx.x; if (i < n) h[i] = i * 0.5; }
static double now() { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main() {
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  unsigned char *h, *d; CK(hipHostMalloc((void**)&h, 1 << 20, 0)); CK(hipMalloc((void**)&d, 1 << 20));
  hipEvent_t ev; CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const int R = 2000;
  for (int w = 0; w < 2; w++) {
    double t0 = now();
    for (int i = 0; i < R; i++) CK(hipMemcpyAsync(d, h, 24000, hipMemcpyHostToDevice, s));
    double t1 = now(); CK(hipStreamSynchronize(s)); double t2 = now();
    for (int i = 0; i < R; i++) hipLaunchKernelGGL(k_nop, dim3(50), dim3(256), 0, s, (int*)d);
    double t3 = now(); CK(hipStreamSynchronize(s)); double t4 = now();
    for (int i = 0; i < R; i++) CK(hipEventRecord(ev, s));
    double t5 = now();
    double rt = 0;
    for (int i = 0; i < 200; i++) {
      double a = now();
      CK(hipMemcpyAsync(d, h, 24000, hipMemcpyHostToDevice, s));
      hipLaunchKernelGGL(k_nop, dim3(50), dim3(256), 0, s, (int*)d);
      CK(hipMemcpyAsync(h, d, 16000, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      rt += now() - a;
    }
    double rt2 = 0;
    for (int i = 0; i < 200; i++) {
      double a = now();
      hipLaunchKernelGGL(k_nop, dim3(50), dim3(256), 0, s, (int*)d);
      CK(hipStreamSynchronize(s));
      rt2 += now() - a;
    }
    double rt3 = 0;
    for (int i = 0; i < 200; i++) {
      double a = now();
      CK(hipMemcpyAsync(d, h, 24000, hipMemcpyHostToDevice, s));
      hipLaunchKernelGGL(k_write_host, dim3(8), dim3(256), 0, s, (double*)h, 2000);
      CK(hipStreamSynchronize(s));
      rt3 += now() - a;
    }
    printf("H2D async call %.2f us | launch call %.2f us (drain %.1f us/launch) | event record %.2f us | "
           "H2D+kernel+D2H+sync round trip %.1f us | kernel+sync %.1f us | H2D+kernel(write host)+sync %.1f us\n",
           (t1 - t0) / R, (t3 - t2) / R, (t4 - t2) / R, (t5 - t4) / R, rt / 200, rt2 / 200, rt3 / 200);
  }
  {  // CPU access cost of pinned (hipHostMalloc) vs pageable memory
    unsigned char* pg = (unsigned char*)malloc(1 << 20);
    float src[3] = {1.f, 2.f, 3.f};
    for (int pass = 0; pass < 2; pass++) {
      unsigned char* buf = pass ? pg : h;
      double a = now();
      for (int r = 0; r < 100; r++)
        for (int i = 0; i < 2000; i++) memcpy(buf + 12 * i, src, 12);  // 2000 packed points
      double b = now();
      hipLaunchKernelGGL(k_write_host, dim3(8), dim3(256), 0, s, (double*)h, 2000);
      CK(hipStreamSynchronize(s));
      double c = now(), acc = 0;
      for (int r = 0; r < 100; r++)
        for (int i = 0; i < 2000; i++) acc += ((double*)buf)[i];
      double e = now();
      printf("%s: write 2000 x 12 B %.2f us | read 2000 doubles %.2f us (%g)\n", pass ? "pageable" : "hipHostMalloc",
             (b - a) / 100, (e - c) / 100, acc);
    }
  }
  double* hd = (double*)h;
  printf("host sees %.1f %.1f\n", hd[2], hd[1999]);
  return 0;
}
