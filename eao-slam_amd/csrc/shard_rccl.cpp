// shard_rccl.cpp -- RCCL exchanger of the sharded association.
//
// One communicator per replay; each exchange is a single ncclAllGather of
// the ranks' fixed-size result records over xGMI. The records are a few KB
// (64-byte NP statistics, 20-byte projected rects, per-point outlier bit
// masks), so the exchange is latency bound; it runs on its own non-blocking
// stream through pinned host staging.
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
  unsigned char *h_send = nullptr, *h_recv = nullptr, *d_send = nullptr, *d_recv = nullptr;
  size_t cap = 0;  // bytes per rank

  ~RcclExchanger() override {
    if (stream) (void)hipStreamSynchronize(stream);
    if (comm) (void)ncclCommDestroy(comm);
    if (stream) (void)hipStreamDestroy(stream);
    if (h_send) (void)hipHostFree(h_send);
    if (h_recv) (void)hipHostFree(h_recv);
    if (d_send) (void)hipFree(d_send);
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
    if (h_send) (void)hipHostFree(h_send);
    if (h_recv) (void)hipHostFree(h_recv);
    if (d_send) (void)hipFree(d_send);
    if (d_recv) (void)hipFree(d_recv);
    EAO_HIP_CHECK(hipHostMalloc((void**)&h_send, c, 0));
    EAO_HIP_CHECK(hipHostMalloc((void**)&h_recv, c * world, 0));
    EAO_HIP_CHECK(hipMalloc((void**)&d_send, c));
    EAO_HIP_CHECK(hipMalloc((void**)&d_recv, c * world));
    cap = c;
    return EAO_OK;
  }
  int allgather(const void* send, void* recv, size_t bytes) override {
    if (bytes == 0) return EAO_OK;
    if (int rc = grow(bytes)) return rc;
    std::memcpy(h_send, send, bytes);
    EAO_HIP_CHECK(hipMemcpyAsync(d_send, h_send, bytes, hipMemcpyHostToDevice, stream));
    EAO_NCCL_CHECK(ncclAllGather(d_send, d_recv, bytes, ncclUint8, comm, stream));
    EAO_HIP_CHECK(hipMemcpyAsync(h_recv, d_recv, bytes * world, hipMemcpyDeviceToHost, stream));
    EAO_HIP_CHECK(hipStreamSynchronize(stream));
    std::memcpy(recv, h_recv, bytes * world);
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
