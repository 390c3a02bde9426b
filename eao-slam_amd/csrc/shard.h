// shard.h -- the association's cross-rank exchange (Config C).
//
// Objects are owned by rank id mod world. Every rank replays the identical
// host decisions; the GPU work of an object (its NP pairs, its projected rect
// and its isolation forest) runs on the owner only, and the fixed-layout
// result records are all-gathered so that every rank applies the same
// outcome. The exchanger is the one collective of that data path.
#pragma once
#include <cstddef>

namespace eao {

struct Exchanger {
  virtual ~Exchanger() {}
  // all-gather of host buffers: recv[r * bytes, (r + 1) * bytes) = rank r's send
  virtual int allgather(const void* send, void* recv, size_t bytes) = 0;
};

// RCCL over xGMI (shard_rccl.cpp): a communicator of `world` ranks on device `dev`
Exchanger* make_rccl_exchanger(int dev, int rank, int world, const void* unique_id, int* rc);

}  // namespace eao
