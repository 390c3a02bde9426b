// Launch cost and launch-to-host round trips: HIP streams against AQL packets written straight
// into a user-mode HSA queue (development aid; decides whether the association's launches move
// off the HIP runtime).
//   make -C tools/micro dispatch   then   tools/micro/_build/dispatch_lat tools/micro/_build/dispatch_k.hsaco
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "dispatch_k.hip"

#define HK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                         \
    }                                                                  \
  } while (0)
#define SK(x)                                                          \
  do {                                                                 \
    hsa_status_t s_ = (x);                                             \
    if (s_ != HSA_STATUS_SUCCESS) {                                    \
      const char* m_ = nullptr;                                        \
      hsa_status_string(s_, &m_);                                      \
      printf("HSA error %s at %s:%d\n", m_ ? m_ : "?", __FILE__, __LINE__); \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

static double now() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}
static double p90(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() * 9 / 10];
}
static void spin_flag(volatile uint32_t* f, uint32_t v, double t0) {
  while (*f != v)
    if (now() - t0 > 2e6) {
      printf("timeout waiting for flag %u\n", v);
      exit(2);
    }
}

// ------------------------------------------------------------------ HSA
static hsa_agent_t g_gpu, g_cpu;
static hsa_amd_memory_pool_t g_karg_pool;
static bool g_have_gpu = false, g_have_cpu = false, g_have_pool = false;

static hsa_status_t find_agents(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU && !g_have_gpu) {
    g_gpu = a;
    g_have_gpu = true;
  }
  if (t == HSA_DEVICE_TYPE_CPU && !g_have_cpu) {
    g_cpu = a;
    g_have_cpu = true;
  }
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t find_karg(hsa_amd_memory_pool_t p, void*) {
  hsa_amd_segment_t seg;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  uint32_t fl = 0;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &fl);
  if ((fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) && !g_have_pool) {
    g_karg_pool = p;
    g_have_pool = true;
  }
  return HSA_STATUS_SUCCESS;
}

struct Kern {
  uint64_t obj = 0;
  uint32_t karg = 0, group = 0, priv = 0;
};

struct Q {
  hsa_queue_t* q = nullptr;
  char* karg = nullptr;  // ring of 512-byte kernarg slots, one per packet slot
  uint32_t mask = 0;
};

static uint16_t hdr(hsa_packet_type_t t, bool barrier, hsa_fence_scope_t acq, hsa_fence_scope_t rel) {
  return (uint16_t)((t << HSA_PACKET_HEADER_TYPE) | ((barrier ? 1 : 0) << HSA_PACKET_HEADER_BARRIER) |
                    (acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                    (rel << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
}

// one kernel dispatch: 1-D grid of `groups` workgroups of 64 lanes
static hsa_fence_scope_t g_acq = HSA_FENCE_SCOPE_SYSTEM;
static void dispatch(Q& q, const Kern& k, const void* args, size_t nbytes, uint32_t groups, hsa_signal_t done,
                     hsa_fence_scope_t rel) {
  const uint64_t idx = hsa_queue_add_write_index_relaxed(q.q, 1);
  while (idx - hsa_queue_load_read_index_relaxed(q.q) >= q.q->size) {
  }
  hsa_kernel_dispatch_packet_t* p = (hsa_kernel_dispatch_packet_t*)q.q->base_address + (idx & q.mask);
  char* ka = q.karg + 512 * (idx & q.mask);
  std::memset(ka, 0, k.karg < 512 ? k.karg : 512);
  std::memcpy(ka, args, nbytes);
  p->workgroup_size_x = 64;
  p->workgroup_size_y = 1;
  p->workgroup_size_z = 1;
  p->reserved0 = 0;
  p->grid_size_x = 64 * groups;
  p->grid_size_y = 1;
  p->grid_size_z = 1;
  p->private_segment_size = k.priv;
  p->group_segment_size = k.group;
  p->kernel_object = k.obj;
  p->kernarg_address = ka;
  p->reserved2 = 0;
  p->completion_signal = done;
  const uint16_t h = hdr(HSA_PACKET_TYPE_KERNEL_DISPATCH, true, g_acq, rel);
  const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
  __atomic_store_n((uint32_t*)p, (uint32_t)h | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
  hsa_signal_store_screlease(q.q->doorbell_signal, (hsa_signal_value_t)idx);
}

static void barrier_and(Q& q, hsa_signal_t dep) {
  const uint64_t idx = hsa_queue_add_write_index_relaxed(q.q, 1);
  while (idx - hsa_queue_load_read_index_relaxed(q.q) >= q.q->size) {
  }
  hsa_barrier_and_packet_t* p = (hsa_barrier_and_packet_t*)q.q->base_address + (idx & q.mask);
  std::memset((char*)p + 4, 0, sizeof(*p) - 4);
  p->dep_signal[0] = dep;
  const uint16_t h = hdr(HSA_PACKET_TYPE_BARRIER_AND, true, HSA_FENCE_SCOPE_NONE, HSA_FENCE_SCOPE_NONE);
  __atomic_store_n((uint32_t*)p, (uint32_t)h, __ATOMIC_RELEASE);
  hsa_signal_store_screlease(q.q->doorbell_signal, (hsa_signal_value_t)idx);
}

static Q make_queue() {
  Q q;
  SK(hsa_queue_create(g_gpu, 1024, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q.q));
  SK(hsa_amd_queue_set_priority(q.q, HSA_AMD_QUEUE_PRIORITY_HIGH));
  q.mask = q.q->size - 1;
  SK(hsa_amd_memory_pool_allocate(g_karg_pool, 512 * (size_t)q.q->size, 0, (void**)&q.karg));
  SK(hsa_amd_agents_allow_access(1, &g_gpu, nullptr, q.karg));
  return q;
}

static Kern get_kern(hsa_executable_t exe, const char* name) {
  hsa_executable_symbol_t sym;
  std::string s = std::string(name) + ".kd";
  SK(hsa_executable_get_symbol_by_name(exe, s.c_str(), &g_gpu, &sym));
  Kern k;
  SK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k.obj));
  SK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k.karg));
  SK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k.group));
  SK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k.priv));
  return k;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    printf("usage: dispatch_lat <dispatch_k.hsaco>\n");
    return 1;
  }
  const int R = 400;
  HK(hipSetDevice(0));
  int lo = 0, hi = 0;
  HK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  hipStream_t s1, s2;
  HK(hipStreamCreateWithPriority(&s1, hipStreamNonBlocking, hi));
  HK(hipStreamCreateWithPriority(&s2, hipStreamNonBlocking, hi));
  hipEvent_t ev;
  HK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  uint32_t* hflag;
  HK(hipHostMalloc((void**)&hflag, 4096, 0));
  volatile uint32_t* vf = hflag;
  *hflag = 0;
  uint32_t seq = 0;
  const uint32_t busy = 500;  // wall_clock64 ticks (100 MHz): 5 us

  // ---------------- HIP
  for (int w = 0; w < 20; w++) hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, s1, hflag, ++seq);
  HK(hipStreamSynchronize(s1));
  std::vector<double> a, b, c, d, e, f;
  for (int i = 0; i < R; i++) {
    double t0 = now();
    hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, s1, (uint32_t*)nullptr);
    a.push_back(now() - t0);
  }
  HK(hipStreamSynchronize(s1));
  for (int i = 0; i < R; i++) {
    double t0 = now();
    hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, s1, hflag, ++seq);
    spin_flag(vf, seq, t0);
    b.push_back(now() - t0);
  }
  HK(hipStreamSynchronize(s1));
  for (int i = 0; i < R; i++) {  // busy (5 us) -> flag on the same stream
    double t0 = now();
    hipLaunchKernelGGL(k_busy, dim3(1), dim3(64), 0, s1, (uint32_t*)nullptr, busy);
    hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, s1, hflag, ++seq);
    spin_flag(vf, seq, t0);
    c.push_back(now() - t0);
  }
  HK(hipStreamSynchronize(s1));
  for (int i = 0; i < R; i++) {  // busy on s1 -> event -> s2 waits -> flag on s2
    double t0 = now();
    hipLaunchKernelGGL(k_busy, dim3(1), dim3(64), 0, s1, (uint32_t*)nullptr, busy);
    HK(hipEventRecord(ev, s1));
    HK(hipStreamWaitEvent(s2, ev, 0));
    hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, s2, hflag, ++seq);
    d.push_back(now() - t0);
    spin_flag(vf, seq, t0);
    e.push_back(now() - t0);
  }
  HK(hipDeviceSynchronize());
  for (int i = 0; i < R; i++) {
    double t0 = now();
    (void)hipEventQuery(ev);
    f.push_back(now() - t0);
  }
  printf("HIP  launch call                      med %6.2f p90 %6.2f us\n", med(a), p90(a));
  printf("HIP  launch -> flag seen               med %6.2f p90 %6.2f us\n", med(b), p90(b));
  printf("HIP  busy(5us) -> flag, one stream     med %6.2f p90 %6.2f us\n", med(c), p90(c));
  printf("HIP  busy -> event -> other stream flag: calls %6.2f us, flag seen med %6.2f p90 %6.2f us\n", med(d),
         med(e), p90(e));
  printf("HIP  hipEventQuery                     med %6.2f us\n", med(f));

  // ---------------- HSA
  SK(hsa_init());
  SK(hsa_iterate_agents(find_agents, nullptr));
  if (!g_have_gpu || !g_have_cpu) {
    printf("no agents\n");
    return 1;
  }
  SK(hsa_amd_agent_iterate_memory_pools(g_cpu, find_karg, nullptr));
  if (!g_have_pool) {
    printf("no kernarg pool\n");
    return 1;
  }
  std::ifstream in(argv[1], std::ios::binary);
  std::stringstream ss;
  ss << in.rdbuf();
  std::string co = ss.str();
  if (co.empty()) {
    printf("cannot read %s\n", argv[1]);
    return 1;
  }
  hsa_code_object_reader_t rd;
  SK(hsa_code_object_reader_create_from_memory(co.data(), co.size(), &rd));
  hsa_executable_t exe;
  SK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe));
  SK(hsa_executable_load_agent_code_object(exe, g_gpu, rd, nullptr, nullptr));
  SK(hsa_executable_freeze(exe, nullptr));
  Kern kn = get_kern(exe, "k_nop"), kf = get_kern(exe, "k_flag"), kb = get_kern(exe, "k_busy");
  printf("HSA  kernarg sizes: nop %u flag %u busy %u; group %u priv %u\n", kn.karg, kf.karg, kb.karg, kf.group,
         kf.priv);
  Q q1 = make_queue(), q2 = make_queue();
  hsa_signal_t sg, none{0};
  SK(hsa_signal_create(1, 0, nullptr, &sg));
  struct {
    uint32_t* p;
  } an{nullptr};
  struct {
    uint32_t* f;
    uint32_t v;
  } af;
  struct {
    uint32_t* p;
    uint32_t c;
  } ab{nullptr, busy};
  for (int w = 0; w < 20; w++) {
    af = {hflag, ++seq};
    dispatch(q1, kf, &af, sizeof af, 1, none, HSA_FENCE_SCOPE_SYSTEM);
    spin_flag(vf, seq, now());
  }
  for (int rel = 0; rel < 4; rel++) {
    const hsa_fence_scope_t rs = rel ? HSA_FENCE_SCOPE_AGENT : HSA_FENCE_SCOPE_SYSTEM;
    g_acq = rel == 0 || rel == 1 ? HSA_FENCE_SCOPE_SYSTEM : rel == 2 ? HSA_FENCE_SCOPE_AGENT : HSA_FENCE_SCOPE_NONE;
    const char* names[] = {"acq sys rel sys  ", "acq sys rel agent", "acq agt rel agent", "acq none rel agent"};
    const char* rn = names[rel];
    a.clear(); b.clear(); c.clear(); d.clear(); e.clear();
    for (int i = 0; i < R; i++) {
      double t0 = now();
      dispatch(q1, kn, &an, sizeof an, 1, none, rs);
      a.push_back(now() - t0);
    }
    for (int i = 0; i < R; i++) {
      double t0 = now();
      af = {hflag, ++seq};
      dispatch(q1, kf, &af, sizeof af, 1, none, rs);
      spin_flag(vf, seq, t0);
      b.push_back(now() - t0);
    }
    for (int i = 0; i < R; i++) {
      double t0 = now();
      dispatch(q1, kb, &ab, sizeof ab, 1, none, rs);
      af = {hflag, ++seq};
      dispatch(q1, kf, &af, sizeof af, 1, none, rs);
      spin_flag(vf, seq, t0);
      c.push_back(now() - t0);
    }
    for (int i = 0; i < R; i++) {
      double t0 = now();
      hsa_signal_store_relaxed(sg, 1);
      dispatch(q1, kb, &ab, sizeof ab, 1, sg, rs);
      barrier_and(q2, sg);
      af = {hflag, ++seq};
      dispatch(q2, kf, &af, sizeof af, 1, none, rs);
      d.push_back(now() - t0);
      spin_flag(vf, seq, t0);
      e.push_back(now() - t0);
      while (hsa_signal_load_scacquire(sg) != 0) {
      }
    }
    printf("HSA  %s dispatch call            med %6.2f p90 %6.2f us\n", rn, med(a), p90(a));
    printf("HSA  %s dispatch -> flag seen    med %6.2f p90 %6.2f us\n", rn, med(b), p90(b));
    printf("HSA  %s busy(5us) -> flag, 1 q   med %6.2f p90 %6.2f us\n", rn, med(c), p90(c));
    printf("HSA  %s busy -> barrier-AND -> other queue flag: calls %6.2f us, flag seen med %6.2f p90 %6.2f us\n",
           rn, med(d), med(e), p90(e));
  }
  // drain both queues before teardown
  hsa_signal_store_relaxed(sg, 1);
  dispatch(q1, kn, &an, sizeof an, 1, sg, HSA_FENCE_SCOPE_SYSTEM);
  while (hsa_signal_load_scacquire(sg) != 0) {
  }
  hsa_signal_store_relaxed(sg, 1);
  dispatch(q2, kn, &an, sizeof an, 1, sg, HSA_FENCE_SCOPE_SYSTEM);
  while (hsa_signal_load_scacquire(sg) != 0) {
  }
  hsa_queue_destroy(q1.q);
  hsa_queue_destroy(q2.q);
  hsa_signal_destroy(sg);
  hsa_executable_destroy(exe);
  hsa_code_object_reader_destroy(rd);
  hsa_shut_down();
  printf("done\n");
  return 0;
}
