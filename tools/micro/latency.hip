// Single-wave instruction latency calibration on gfx950 (development aid):
// dependent chains of VALU ops, VALU->SALU->VALU round trips, readlane,
// taken scalar branches, DPP and ds_swizzle, timed with s_memtime.
#include <hip/hip_runtime.h>

#include <cstdio>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

__global__ void k_lat(unsigned long long* out, int seed) {
  int v = threadIdx.x + seed;
  int s = seed;
  unsigned long long t0, t1;
  // 1) dependent v_add_u32
  t0 = clock64();
  REP64(asm volatile("v_add_u32 %0, %0, 1" : "+v"(v));)
  t1 = clock64();
  out[0] = t1 - t0;
  // 2) dependent s_add_u32
  t0 = clock64();
  REP64(asm volatile("s_add_u32 %0, %0, 1" : "+s"(s));)
  t1 = clock64();
  out[1] = t1 - t0;
  // 3) v_readfirstlane -> s_add -> v_add (VALU->SALU->VALU)
  t0 = clock64();
  REP64(asm volatile("v_readfirstlane_b32 %1, %0\n\ts_add_u32 %1, %1, 1\n\tv_add_u32 %0, %1, %0" : "+v"(v), "+s"(s));)
  t1 = clock64();
  out[2] = t1 - t0;
  // 4) v_cmp -> s_and (vcc consumed by SALU)
  unsigned long long m = 0;
  t0 = clock64();
  REP64(asm volatile("v_cmp_gt_u32 %1, %0, 5\n\ts_and_b64 %1, %1, exec\n\tv_cndmask_b32 %0, %0, 1, %1" : "+v"(v), "+s"(m));)
  t1 = clock64();
  out[3] = t1 - t0;
  // 5) DPP chain
  t0 = clock64();
  REP64(asm volatile("s_nop 1\n\tv_add_u32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(v));)
  t1 = clock64();
  out[4] = t1 - t0;
  // 6) ds_swizzle chain
  t0 = clock64();
  REP64(asm volatile("ds_swizzle_b32 %0, %0 offset:swizzle(BITMASK_PERM,\"01pip\")\n\ts_waitcnt lgkmcnt(0)" : "+v"(v));)
  t1 = clock64();
  out[5] = t1 - t0;
  // 7) v_readlane with sgpr lane -> s_add
  t0 = clock64();
  REP64(asm volatile("s_and_b32 %1, %1, 63\n\tv_readlane_b32 %1, %0, %1" : "+v"(v), "+s"(s));)
  t1 = clock64();
  out[6] = t1 - t0;
  // 8) taken scalar branches
  t0 = clock64();
  REP64(asm volatile("s_branch 1f\n\ts_nop 0\n1:\n\ts_add_u32 %0, %0, 1" : "+s"(s));)
  t1 = clock64();
  out[7] = t1 - t0;
  // 9) v_cvt_f32 + v_mul_f32 + readfirstlane (split-like)
  float f = (float)v;
  t0 = clock64();
  REP64(asm volatile("v_mul_f32 %0, 0x3f000001, %0\n\tv_add_f32 %0, 1.0, %0\n\tv_readfirstlane_b32 %1, %0\n\tv_add_f32 %0, %1, %0" : "+v"(f), "+s"(s));)
  t1 = clock64();
  out[8] = t1 - t0;
  // 10) independent v_add (4 chains interleaved)
  int a = v, b = v + 1, c = v + 2, d = v + 3;
  t0 = clock64();
  REP64(asm volatile("v_add_u32 %0, %0, 1\n\tv_add_u32 %1, %1, 1\n\tv_add_u32 %2, %2, 1\n\tv_add_u32 %3, %3, 1" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));)
  t1 = clock64();
  out[9] = t1 - t0;
  // 11) v_writelane with m0 lane select
  int w = 0;
  t0 = clock64();
  REP64(asm volatile("s_and_b32 m0, %1, 63\n\tv_writelane_b32 %0, %1, m0\n\ts_add_u32 %1, %1, 1" : "+v"(w), "+s"(s) :: "m0");)
  t1 = clock64();
  out[10] = t1 - t0;
  out[11] = v + s + (int)m + (int)f + a + b + c + d + w;
}

int main() {
  unsigned long long* d;
  unsigned long long h[12];
  (void)hipMalloc(&d, sizeof h);
  for (int r = 0; r < 3; r++) hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, d, 3);
  (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  const char* names[] = {"v_add dep", "s_add dep", "readfirstlane+s_add+v_add", "v_cmp+s_and+v_cndmask",
                         "dpp add (+nop)", "ds_swizzle+wait", "s_and+readlane", "s_branch taken+s_add",
                         "vmul+vadd+readfirstlane+vadd", "4x indep v_add", "s_and m0+writelane+s_add"};
  for (int i = 0; i < 11; i++) printf("%-34s %6.1f cycles per rep\n", names[i], h[i] / 64.0);
  return 0;
}
