"""World-size-2 gloo tests of the object-sharded association (SURVEY.md §8e,
Config C): eao_replay_shard_callback on the host harness (tests/native, the
engine's replay.cpp with oracle-served primitives), two processes, objects
owned by id mod 2, result records all-gathered through gloo. Every rank must
return the association ids and object statistics of the unsharded oracle
replay. CPU only; the RCCL exchanger is covered by tests/test_gpu_shard.py."""
import ctypes
import os
import socket
import subprocess

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import eao_accel as ea
import eao_dist
import pyoracle as orc
from tools import synth

NATIVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")
HARNESS = os.path.join(NATIVE, "_build", "libreplay_host.so")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stream(kind, n):
    return synth.assoc_stream_config_c(n) if kind == "C" else synth.assoc_stream(n)


def _device_exchange(H, world):
    """The harness's stand-in for the RCCL exchanger (device form) over gloo: the replay
    writes its records into "device" buffers and gathers them from there."""
    gather = eao_dist.allgather_bytes_gloo() if world > 1 else None

    def fn(ctx, send, recv, nbytes):
        try:
            data = gather(ctypes.string_at(send, nbytes))
            ctypes.memmove(recv, data, len(data))
            return 0
        except Exception:  # noqa: BLE001 -- reported through the C status
            return -1
    cb = ea.Replay.ALLGATHER(fn)
    H.harness_set_device_exchange(cb, None)
    return cb


def _worker(rank, world, port, flag, kind, n, q, form="host"):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        H = ctypes.CDLL(HARNESS)
        H.harness_assoc_create.restype = ctypes.c_void_p
        ea._lib = H  # this process only talks to the harness build of the engine

        class A:
            pass
        a = A()
        a.h = ctypes.c_void_p(H.harness_assoc_create())
        g = ea.Replay(a, flag)
        if form == "device":
            keep = _device_exchange(H, world)  # noqa: F841 -- the callback must outlive the replay
            g.shard(rank, world, unique_id=bytes(128))
        else:
            g.shard(rank, world, allgather=eao_dist.allgather_bytes_gloo())
        outs = []
        for i, f in enumerate(_stream(kind, n)):
            outs.append(g.frame(i + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"]))
            if f["kf"]:
                g.local_mapping()
        ints, fl, pts = g.objects()
        st = g.shard_stats()
        dist.destroy_process_group()
        q.put((rank, outs, ints, fl, [p.tolist() for p in pts], st, None))
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        q.put((rank, None, None, None, None, None, repr(e)))


def _oracle(flag, kind, n):
    o = orc.Replay(flag)
    outs = []
    for i, f in enumerate(_stream(kind, n)):
        outs.append(o.frame(i + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"]))
        if f["kf"]:
            o.local_mapping()
    return outs, o.objects()


@pytest.mark.parametrize("kind,n,flag,form,world", [("C", 40, "EAO", "host", 2), ("fr3", 60, "iForest", "host", 2),
                                                   ("fr3", 30, "NP", "host", 2), ("C", 40, "EAO", "device", 2),
                                                   ("fr3", 40, "EAO", "device", 2), ("C", 30, "EAO", "device", 1)])
def test_sharded_replay_world2_matches_oracle(kind, n, flag, form, world):
    """form "device": the RCCL exchanger's device form (records written by the kernels into
    device buffers, gathered from there); world 1 runs the whole exchange path on one rank."""
    orc.lib()
    subprocess.check_call(["make", "-s", "-C", NATIVE])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, flag, kind, n, q, form)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=600) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    assert all(r[6] is None for r in res), [r[6] for r in res]
    assert all(p.exitcode == 0 for p in procs)
    ref_outs, (ri, rf, rp) = _oracle(flag, kind, n)
    for rank, outs, ints, fl, pts, st, _ in res:
        for t, (a, b) in enumerate(zip(outs, ref_outs)):
            assert np.array_equal(a, b), (rank, t, a.tolist(), b.tolist())
        assert np.array_equal(ints, ri)
        assert np.allclose(fl, rf, rtol=1e-5, atol=1e-5, equal_nan=True)
        assert pts == [p.tolist() for p in rp]
        assert st["exchanges"] > 0
    # both ranks saw the same exchanges
    assert res[0][5]["exchanges"] == res[-1][5]["exchanges"]


def _worker_capacity(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        H = ctypes.CDLL(HARNESS)
        H.harness_assoc_create.restype = ctypes.c_void_p
        H.eao_last_error.restype = ctypes.c_char_p
        ea._lib = H

        class A:
            pass
        a = A()
        a.h = ctypes.c_void_p(H.harness_assoc_create())
        g = ea.Replay(a, "iForest")
        g.shard(rank, world, allgather=eao_dist.allgather_bytes_gloo())
        err = None
        for i, f in enumerate(synth.assoc_stream(12, classes=[39, 56], pts_range=(9000, 9001))):
            try:
                g.frame(i + 1, f["T"], f["boxes"], f["ids"], f["pos"], f["uv"], f["bad"])
            except ea.EaoError as e:
                err = str(e)
                break
        dist.destroy_process_group()
        q.put((rank, err, None))
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


def test_sharded_capacity_error_reaches_every_rank():
    """An object over the isolation-forest capacity (9000 points > IF_MAXN): the capacity
    verdict is taken over the whole batch before the ownership filter, so both ranks fail
    the same frame with the same error instead of one rank waiting in an exchange."""
    subprocess.check_call(["make", "-s", "-C", NATIVE])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_capacity, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    assert all(r[2] is None for r in res), [r[2] for r in res]
    assert all(r[1] is not None and "capacity" in r[1] for r in res), [r[1] for r in res]
