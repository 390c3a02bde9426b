// shard.h -- the association's cross-rank exchange (Config C).
//
// Objects are owned by rank id mod world. Every rank replays the identical
// host decisions; the GPU work of an object (its NP pairs, its projected rect
// and its isolation forest) runs on the owner only, and the fixed-layout
// result records are all-gathered so that every rank applies the same
// outcome. The exchanger is the one collective of that data path.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace eao {

// when a device-form record is complete: after a HIP event (records written on HIP streams), or
// once the word *flag holds >= value (records written on an HSA lane, whose k_publish stores the
// value after them; the flag is signal memory from the exchanger's ready_flag)
struct ExReady {
  hipEvent_t ev = nullptr;
  const uint64_t* flag = nullptr;
  uint64_t value = 0;
};

struct Exchanger {
  virtual ~Exchanger() {}
  // host form (the gloo callback of eao_replay_shard_callback): all-gather of host
  // buffers, recv[r * bytes, (r + 1) * bytes) = rank r's send
  virtual int allgather(const void* send, void* recv, size_t bytes) = 0;
  // device form (RCCL): the records are gathered from device memory into device memory.
  // d_send holds this rank's `bytes` once `ready` holds (the kernels that wrote it were
  // recorded on its event, or published its flag value); the collective waits on the GPU, and the
  // [world][bytes] result is copied to the host once: *h_recv points at it (pinned,
  // valid until the next exchange).
  virtual bool device_form() const { return false; }
  // the GPU-side ready flag of producer lane `i` (0..7; nullptr: none): signal memory holding the
  // last value published on that lane, monotone per lane
  virtual uint64_t* ready_flag(int i) {
    (void)i;
    return nullptr;
  }
  virtual int allgather_device(const void* d_send, const ExReady& ready, size_t bytes, const unsigned char** h_recv) {
    int t = -1;
    if (int rc = start_device(d_send, ready, bytes, &t)) return rc;
    return wait_device(t, h_recv);
  }
  // the same in two halves: start_device enqueues the exchange (the GPU waits for `ready`, gathers,
  // copies back) and returns at once with a ticket; wait_device(ticket) returns the gathered
  // records (valid until the next start_device). Tickets may be waited in any order; every rank
  // starts its exchanges in the same order (the collectives' order).
  virtual int start_device(const void* d_send, const ExReady& ready, size_t bytes, int* ticket) {
    (void)d_send;
    (void)ready;
    (void)bytes;
    (void)ticket;
    return -1;
  }
  virtual int wait_device(int ticket, const unsigned char** h_recv) {
    (void)ticket;
    (void)h_recv;
    return -1;
  }
};

// RCCL over xGMI (shard_rccl.cpp): a communicator of `world` ranks on device `dev`
Exchanger* make_rccl_exchanger(int dev, int rank, int world, const void* unique_id, int* rc);

}  // namespace eao
