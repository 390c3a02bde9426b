// hsa_lane.h -- launch lanes of the association chain.
//
// A Lane is either a HIP stream or a user-mode HSA queue that the engine writes AQL packets into
// itself (hsa_lane.cpp). The replay's forest batches and frame starts are a latency chain of
// small launches: a hipLaunchKernel costs ~2.3 us of host time and a cross-stream
// launch / event record / event wait / launch sequence ~12 us, against ~0.2 us per AQL packet and
// ~0.6 us for the same sequence with a barrier-AND packet, and the packets' agent-scope acquire
// starts a dependent kernel ~1-4 us sooner (profiles/r05_dispatch_lat.txt, tools/micro/dispatch_lat.cpp).
// A Done is the matching completion marker: a HIP event, or a use of an HSA signal of the lane's
// ring, attached to the lane's last packet.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstring>

namespace eao {

struct HsaQueue;
struct Lane {
  hipStream_t s = nullptr;
  HsaQueue* q = nullptr;
  Lane() = default;
  Lane(hipStream_t st) : s(st) {}
  bool hsa() const { return q != nullptr; }
};
struct Done {
  hipEvent_t e = nullptr;
  uint64_t sig = 0;  // hsa_signal_t handle (HSA lanes)
  HsaQueue* q = nullptr;  // the lane whose signal ring holds it,
  uint32_t slot = 0;      // the ring slot
  uint64_t use = 0;       // and the slot's use it marks (a later use of the slot: this one completed)
};

// HSA lanes usable on HIP device `dev` (the code object loaded, an agent matched by PCI address);
// EAO_HSA_LANES=0 turns them off (A/B switch)
bool hsa_lanes_available(int dev);
// open n lanes of the chosen kind (HIP: non-blocking streams at the highest priority)
int lanes_open(Lane* l, int n, bool hsa, int dev);
void lane_close(Lane& l);  // drains an HSA queue first
int lane_sync(const Lane& l);  // wait until everything launched on l has completed
void done_close(Done& d);
// record d on lane l (after everything launched on l so far); d takes the lane's kind
int lane_record(const Lane& l, Done& d);
// everything launched on l after this call waits for d (a Done of the same kind)
int lane_wait(const Lane& l, const Done& d);
// hipSuccess (complete), hipErrorNotReady, or an error
hipError_t done_query(const Done& d);
// device memory the host writes directly through the BAR (write-combined; never read it back on
// the host): nullptr when the device's memory is not host-visible
void* bar_alloc(int dev, size_t bytes);
void bar_free(void* p);
// the host wrote BAR memory ending at `last` that launches on lane l read: the lane's next commit
// flushes it (write-combining fence, HDP flush, read-back) before its doorbell
void lane_bar_written(const Lane& l, const void* last);

// the generated kernel table (gen_co.py)
struct CoKernel {
  const char* name;  // demangled
  const char* sym;   // symbol of the kernel descriptor
  uint32_t karg, group, priv;
  int nargs;
  int off[32], size[32];
  int hidden[14];  // offsets of block_count xyz, group_size xyz, remainder xyz, global_offset xyz, grid_dims,
                   // dynamic_lds_size (-1: not declared)
};
// index of the kernel whose demangled name starts with `prefix` (-1: none)
int hsa_kernel_id(const char* prefix);
const CoKernel* hsa_kernel_meta(int id);
// one dispatch of kernel `id` on q: grid g (workgroups) x block b, `dyn_lds` bytes of dynamic LDS,
// explicit arguments laid out in `args` at the kernel's offsets
int hsa_submit(HsaQueue* q, int id, dim3 g, dim3 b, uint32_t dyn_lds, const unsigned char* args);
int hsa_arg_mismatch(int id, int i, int size);  // sets the error, returns EAO_E_STATE
// self-test of the HSA lanes' markers and commits (eao_lane_selftest); report[0] = packets written
int lane_selftest(int dev, int* report);

// hipLaunchKernelGGL's counterpart on an HSA lane: the arguments are placed at the offsets the
// code object declares, each checked against the declared size (pass them as the kernel's
// parameter types)
template <class... A>
int hsa_launch(HsaQueue* q, int id, dim3 g, dim3 b, uint32_t dyn_lds, const A&... a) {
  const CoKernel* k = hsa_kernel_meta(id);
  alignas(16) unsigned char buf[512];
  std::memset(buf, 0, sizeof(buf));
  if (!k || k->nargs != (int)sizeof...(A)) return hsa_arg_mismatch(id, -1, (int)sizeof...(A));
  int i = 0, bad = -1, bad_size = 0;
  auto put = [&](const void* p, int n) {
    if (bad < 0 && (k->size[i] != n || k->off[i] + n > (int)sizeof(buf))) {
      bad = i;
      bad_size = n;
    }
    if (bad < 0) std::memcpy(buf + k->off[i], p, (size_t)n);
    i++;
  };
  (put(&a, (int)sizeof(A)), ...);
  if (bad >= 0) return hsa_arg_mismatch(id, bad, bad_size);
  return hsa_submit(q, id, g, b, dyn_lds, buf);
}

}  // namespace eao
