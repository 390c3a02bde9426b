"""World-size-2 gloo tests of the frame-parallel plumbing used by bench.py
(eao-slam_amd/python/eao_dist.py): disjoint shards that cover every unit, and
max/sum reductions of the per-rank timings/counts. CPU only."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import eao_dist


def test_shard_covers_all_units():
    for n in (0, 1, 7, 405, 1000):
        for world in (1, 2, 3, 8):
            got = []
            for r in range(world):
                b, e = eao_dist.shard(n, r, world)
                assert 0 <= b <= e <= n
                got.extend(range(b, e))
            assert got == list(range(n))
    with pytest.raises(ValueError):
        eao_dist.shard(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r, w, lr = eao_dist.env_rank()
    b, e = eao_dist.shard(405, r, w)
    eao_dist.barrier()
    mx = eao_dist.max_over_ranks(1.5 + r)
    tot = eao_dist.sum_over_ranks(e - b)
    dist.destroy_process_group()
    q.put((r, w, b, e, mx, tot))


def test_gloo_world2_shards_and_reductions():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [(r[2], r[3]) for r in res] == [(0, 203), (203, 405)]
    assert all(r[4] == 2.5 and r[5] == 405 for r in res)


_RANK_SCRIPT = r'''
import os, sys, torch, torch.distributed as dist
dist.init_process_group("gloo")
r, w = dist.get_rank(), dist.get_world_size()
assert (r, w) == (int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])) and os.environ["LOCAL_RANK"] == str(r)
t = torch.tensor([float(r + 1)])
dist.all_reduce(t)
dist.barrier()
dist.destroy_process_group()
if r == 0:
    print("ranks-ok %d %.0f %s" % (w, t.item(), " ".join(sys.argv[1:])), flush=True)
'''


def test_bench_launcher_world2(tmp_path, capfd):
    """bench.py --gpus 2 outside torchrun starts two fresh rank processes (launch_ranks) that
    rendezvous on 127.0.0.1 with the torchrun environment; rank 0 reports."""
    import bench
    script = tmp_path / "rank.py"
    script.write_text(_RANK_SCRIPT)
    env_before = {k: os.environ.get(k) for k in ("RANK", "WORLD_SIZE")}
    rc = bench.launch_ranks(2, ["--gpus", "2", "--steps", "1"], script=str(script))
    assert rc == 0
    out = capfd.readouterr().out
    assert "ranks-ok 2 3 --gpus 2 --steps 1" in out
    assert {k: os.environ.get(k) for k in env_before} == env_before  # the parent's environment is untouched
