"""Multi-GPU plumbing for the frame-parallel path.

Frames (and the association replays of independent camera streams) are
independent units: each rank owns a contiguous block of them and no data-path
collective is needed.  The only cross-rank operations are the benchmark's
barrier and the max-over-ranks of the timed region.  One process per GPU,
torch.distributed over RCCL ("nccl") on the GPU box, gloo on CPU tests.
"""
import os

import torch
import torch.distributed as dist


def env_rank():
    """(rank, world, local_rank) from the torchrun environment (1-process default)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(n_units, rank, world):
    """Contiguous block [begin, end) of n_units owned by `rank` (sizes differ by <= 1)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(n_units, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def max_over_ranks(value, device=None):
    """Maximum of a float over all ranks (identity without a process group)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    if dist.get_backend() == "gloo":
        device = None  # gloo reduces host tensors
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value, device=None):
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    if dist.get_backend() == "gloo":
        device = None
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def barrier():
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


# ---------------------------------------------------------------- Config C
# Object-sharded association: objects are owned by id mod
# world; every rank replays the same stream and the owners' result records are
# all-gathered once per exchange step (eao_replay_shard_*).

def allgather_bytes_gloo(group=None):
    """An allgather(bytes) -> bytes over a CPU (gloo) process group, for
    Replay.shard(..., allgather=...). World order, equal lengths."""
    def ag(data):
        world = dist.get_world_size(group)
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8)
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t, group=group)
        return b"".join(o.numpy().tobytes() for o in out)
    return ag


def broadcast_bytes(data, src=0, group=None):
    """Broadcast a small byte string (e.g. the 128-byte RCCL id) from `src`."""
    obj = [data]
    dist.broadcast_object_list(obj, src=src, group=group)
    return obj[0]
