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

struct RcclExchanger : Exchanger {
  int dev = 0, world = 1;
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;  // the gathered records' copy-back
  unsigned char *h_recv = nullptr, *d_recv = nullptr;
  size_t cap = 0;  // bytes per rank

  ~RcclExchanger() override {
    if (stream) (void)hipStreamSynchronize(stream);
    if (done) (void)hipEventDestroy(done);
    if (comm) (void)ncclCommDestroy(comm);
    if (stream) (void)hipStreamDestroy(stream);
    if (h_recv) (void)hipHostFree(h_recv);
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
    return grow(4096);
  }
  int grow(size_t bytes) {
    if (bytes <= cap) return EAO_OK;
    const size_t c = std::max(bytes, 2 * cap);
    // every pointer is released and cleared before reallocating, so a failed
    // allocation below never leaves the destructor a stale pointer to free again
    if (stream) EAO_HIP_CHECK(hipStreamSynchronize(stream));
    if (h_recv) (void)hipHostFree(h_recv);
    if (d_recv) (void)hipFree(d_recv);
    h_recv = d_recv = nullptr;
    cap = 0;
    EAO_HIP_CHECK(hipHostMalloc((void**)&h_recv, c * world, 0));
    EAO_HIP_CHECK(hipMalloc((void**)&d_recv, c * world));
    cap = c;
    return EAO_OK;
  }
  int allgather(const void*, void*, size_t) override {
    set_error("rccl exchanger: records are exchanged from device memory (allgather_device)");
    return EAO_E_ARG;
  }
  bool device_form() const override { return true; }
  int allgather_device(const void* d_send, hipEvent_t ready, size_t bytes, const unsigned char** out) override {
    if (bytes == 0) return EAO_E_ARG;
    if (int rc = grow(bytes)) return rc;
    if (ready) EAO_HIP_CHECK(hipStreamWaitEvent(stream, ready, 0));
    EAO_NCCL_CHECK(ncclAllGather(d_send, d_recv, bytes, ncclUint8, comm, stream));
    EAO_HIP_CHECK(hipMemcpyAsync(h_recv, d_recv, bytes * world, hipMemcpyDeviceToHost, stream));
    // the replay thread spins on the copy's event, as on its own launches: a blocking
    // synchronisation may park the thread and pay a wake-up per exchange
    if (!done) EAO_HIP_CHECK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
    EAO_HIP_CHECK(hipEventRecord(done, stream));
    for (;;) {
      const hipError_t r = hipEventQuery(done);
      if (r == hipSuccess) break;
      if (r != hipErrorNotReady) EAO_HIP_CHECK(r);
      __builtin_ia32_pause();
    }
    *out = h_recv;
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
    rc = x->allgather_device(d_send, ev, n, &recv);
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
