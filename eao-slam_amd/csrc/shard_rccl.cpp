// shard_rccl.cpp -- RCCL exchanger of the sharded association.
//
// One communicator per replay; each exchange is a single ncclAllGather of the
// ranks' fixed-size result records over xGMI. The records (64-byte NP
// statistics, 17-byte projected rects, per-point outlier bit masks) are written
// by the engine's kernels straight into device memory; the collective reads
// them there after a GPU-side wait on the producing stream's event, gathers into
// device memory, and only the gathered records the host's decisions need come
// back, in one copy. The exchange is latency bound (a few KB).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/eao_accel.h"
#include "common.h"
#include "shard.h"

namespace eao {
namespace {

#define EAO_NCCL_CHECK(expr)                                                      \
  do {                                                                            \
    ncclResult_t _r = (expr);                                                     \
    if (_r != ncclSuccess) {                                                      \
      ::eao::set_error(std::string(#expr) + ": " + ncclGetErrorString(_r));       \
      return EAO_E_HIP;                                                           \
    }                                                                             \
  } while (0)

// The gathered records' way back to the host: one workgroup behind the all-gather on its stream
// copies them into pinned host memory and then publishes the call's sequence number in a flag
// word after them (every thread's stores drained system-wide before the barrier; the flag stored
// last), so the host waits on that word instead of a DMA copy plus an event.
__global__ __launch_bounds__(256) void k_recv_out(const unsigned char* __restrict__ d, unsigned char* h, size_t n,
                                                  unsigned* flag, unsigned seq) {
  const size_t n16 = n / 16;
  for (size_t i = threadIdx.x; i < n16; i += blockDim.x) ((uint4*)h)[i] = ((const uint4*)d)[i];
  for (size_t i = 16 * n16 + threadIdx.x; i < n; i += blockDim.x) h[i] = d[i];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct RcclExchanger : Exchanger {
  int dev = 0, world = 1;
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;  // the latest copy-back (its errors)
  unsigned char* d_recv = nullptr;
  size_t dcap = 0;   // bytes of d_recv
  unsigned seq = 0;  // k_recv_out's flag value of the latest exchange
  // pinned landing slots of the exchanges in flight: [world][bytes] records + the flag word
  struct Slot {
    unsigned char* h = nullptr;
    size_t cap = 0;
    unsigned want = 0;
    bool busy = false;
    unsigned* flag() const { return (unsigned*)(h + cap); }
  };
  std::vector<Slot> slots;
  uint64_t* rflag[8] = {};  // producer lanes' ready flags (signal memory), made on first use

  ~RcclExchanger() override {
    if (stream) (void)hipStreamSynchronize(stream);
    for (uint64_t* f : rflag)
      if (f) (void)hipFree(f);
    if (done) (void)hipEventDestroy(done);
    if (comm) (void)ncclCommDestroy(comm);
    if (stream) (void)hipStreamDestroy(stream);
    for (Slot& sl : slots)
      if (sl.h) (void)hipHostFree(sl.h);
    if (d_recv) (void)hipFree(d_recv);
  }
  int init(int d, int rank, int w, const void* uid) {
    dev = d;
    world = w;
    EAO_HIP_CHECK(hipSetDevice(dev));
    EAO_HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof id);
    EAO_NCCL_CHECK(ncclCommInitRank(&comm, world, id, rank));
    return EAO_OK;
  }
  // the gathered records' device buffer: exchanges on the stream run one after the other, so one
  // buffer serves them all (growing it waits for those in flight)
  int grow_dev(size_t n) {
    if (n <= dcap) return EAO_OK;
    const size_t c = std::max(n, 2 * dcap);
    EAO_HIP_CHECK(hipStreamSynchronize(stream));
    if (d_recv) (void)hipFree(d_recv);
    d_recv = nullptr;
    dcap = 0;
    EAO_HIP_CHECK(hipMalloc((void**)&d_recv, c));
    dcap = c;
    return EAO_OK;
  }
  // a free landing slot of >= n bytes (a free slot that is too small is regrown)
  int take_slot(size_t n, int* out) {
    int k = -1;
    for (int i = 0; i < (int)slots.size() && k < 0; i++)
      if (!slots[i].busy && slots[i].cap >= n) k = i;
    for (int i = 0; i < (int)slots.size() && k < 0; i++)
      if (!slots[i].busy) k = i;
    if (k < 0) {
      slots.emplace_back();
      k = (int)slots.size() - 1;
    }
    Slot& sl = slots[k];
    if (sl.cap < n) {
      const size_t c = std::max<size_t>(std::max(n, 2 * sl.cap), 4096);
      if (sl.h) (void)hipHostFree(sl.h);
      sl.h = nullptr;
      sl.cap = 0;
      EAO_HIP_CHECK(hipHostMalloc((void**)&sl.h, c + 64, 0));  // + the flag word
      sl.cap = c;
      *(volatile unsigned*)sl.flag() = 0;
    }
    *out = k;
    return EAO_OK;
  }
  int allgather(const void*, void*, size_t) override {
    set_error("rccl exchanger: records are exchanged from device memory (allgather_device)");
    return EAO_E_ARG;
  }
  bool device_form() const override { return true; }
  uint64_t* ready_flag(int i) override {
    if (i < 0 || i >= 8) return nullptr;
    if (!rflag[i]) {
      void* p = nullptr;
      if (hipSetDevice(dev) != hipSuccess || hipExtMallocWithFlags(&p, sizeof(uint64_t), hipMallocSignalMemory) != hipSuccess)
        return nullptr;
      if (hipMemset(p, 0, sizeof(uint64_t)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        (void)hipFree(p);
        return nullptr;
      }
      rflag[i] = (uint64_t*)p;  // 0: below every published value (>= 1)
    }
    return rflag[i];
  }
  int start_device(const void* d_send, const ExReady& ready, size_t bytes, int* ticket) override {
    if (bytes == 0) return EAO_E_ARG;
    if (int rc = grow_dev(bytes * world)) return rc;
    int k = -1;
    if (int rc = take_slot(bytes * world, &k)) return rc;
    Slot& sl = slots[k];
    if (ready.ev) EAO_HIP_CHECK(hipStreamWaitEvent(stream, ready.ev, 0));
    if (ready.flag)  // the HSA lane's k_publish stores the value once the record is complete
      EAO_HIP_CHECK(hipStreamWaitValue64(stream, (void*)ready.flag, ready.value, hipStreamWaitValueGte));
    EAO_NCCL_CHECK(ncclAllGather(d_send, d_recv, bytes, ncclUint8, comm, stream));
    sl.want = ++seq;
    hipLaunchKernelGGL(k_recv_out, dim3(1), dim3(256), 0, stream, d_recv, sl.h, bytes * world, sl.flag(), sl.want);
    EAO_HIP_CHECK(hipGetLastError());
    if (!done) EAO_HIP_CHECK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
    EAO_HIP_CHECK(hipEventRecord(done, stream));
    sl.busy = true;
    *ticket = k;
    return EAO_OK;
  }
  int wait_device(int ticket, const unsigned char** out) override {
    if (ticket < 0 || ticket >= (int)slots.size() || !slots[ticket].busy) {
      set_error("rccl exchanger: wait on an unknown exchange");
      return EAO_E_STATE;
    }
    Slot& sl = slots[ticket];
    const unsigned* flag = sl.flag();
    // the replay thread spins (a blocking synchronisation may park it and pay a wake-up per
    // exchange) on the flag; the latest event reports a failed launch (queried every 64 spins)
    for (unsigned k = 1;; k++) {
      if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == sl.want) break;
      if ((k & 63) == 0) {
        const hipError_t r = hipEventQuery(done);
        if (r != hipSuccess && r != hipErrorNotReady) EAO_HIP_CHECK(r);
        if (r == hipSuccess && __atomic_load_n(flag, __ATOMIC_ACQUIRE) != sl.want) {
          set_error("rccl exchanger: copy-back completed without its flag");
          return EAO_E_HIP;
        }
      }
      __builtin_ia32_pause();
    }
    sl.busy = false;  // its bytes stay until a later start_device takes the slot
    *out = sl.h;
    return EAO_OK;
  }
};

}  // namespace

Exchanger* make_rccl_exchanger(int dev, int rank, int world, const void* unique_id, int* rc) {
  RcclExchanger* x = new RcclExchanger();
  *rc = x->init(dev, rank, world, unique_id);
  if (*rc) {
    delete x;
    return nullptr;
  }
  return x;
}

}  // namespace eao

namespace {
__global__ void k_selftest_pattern(unsigned char* d, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) d[i] = (unsigned char)(i * 131 + 7);
}
}  // namespace

// one-rank RCCL exchange self-test: a world-1 communicator from a fresh unique id, one
// all-gather of a byte pattern through the replay's exchanger in its device form (the
// pattern in device memory, ready behind an event; ncclAllGather device to device; one
// copy back), result compared with the pattern
extern "C" int eao_rccl_selftest(int device, int bytes) {
  if (bytes <= 0) return EAO_E_ARG;
  if (!eao_device_ok(device)) {
    eao::set_error("no usable gfx950 device");
    return EAO_E_NODEVICE;
  }
  uint8_t uid[128];
  if (int rc = eao_rccl_unique_id(uid)) return rc;
  int rc = 0;
  eao::Exchanger* x = eao::make_rccl_exchanger(device, 0, 1, uid, &rc);
  if (!x) return rc;
  unsigned char* d_send = nullptr;
  hipEvent_t ev = nullptr;
  // the requested size, then one past the initial 4 KB (grow() reallocates)
  for (size_t n : {(size_t)bytes, (size_t)bytes + 4097}) {
    std::string send(n, '\0');
    for (size_t i = 0; i < n; i++) send[i] = (char)(i * 131 + 7);
    if (d_send) (void)hipFree(d_send);
    d_send = nullptr;
    if (hipMalloc((void**)&d_send, n) != hipSuccess ||
        (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess)) {
      eao::set_error("eao_rccl_selftest: test buffer setup failed");
      rc = EAO_E_HIP;
      break;
    }
    // the pattern is written on the device (as the engine's kernels write their records)
    hipLaunchKernelGGL(k_selftest_pattern, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, d_send, n);
    if (hipGetLastError() != hipSuccess || hipEventRecord(ev, 0) != hipSuccess) {
      eao::set_error("eao_rccl_selftest: pattern kernel failed");
      rc = EAO_E_HIP;
      break;
    }
    const unsigned char* recv = nullptr;
    eao::ExReady rd;
    rd.ev = ev;
    rc = x->allgather_device(d_send, rd, n, &recv);
    if (!rc && std::memcmp(recv, send.data(), n) != 0) {
      eao::set_error("eao_rccl_selftest: gathered bytes differ");
      rc = EAO_E_HIP;
    }
    if (rc) break;
  }
  if (d_send) (void)hipFree(d_send);
  if (ev) (void)hipEventDestroy(ev);
  delete x;
  return rc;
}

extern "C" int eao_rccl_unique_id(uint8_t* out) {
  if (!out) return EAO_E_ARG;
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) {
    eao::set_error(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    return EAO_E_HIP;
  }
  std::memcpy(out, &id, sizeof id);
  return EAO_OK;
}
