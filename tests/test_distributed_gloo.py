"""World-size-2 gloo tests of the instance sharding and the final gather (CPU, no GPU)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed import gather_rows, max_over_ranks, shard_ids


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ids = shard_ids(total, world, rank)
        # per-instance "results": x rows whose entries encode the global id
        local = torch.stack([torch.full((5,), float(i), dtype=torch.float64) for i in ids]) if ids \
            else torch.zeros((0, 5), dtype=torch.float64)
        g = gather_rows(local, total, world, rank)
        tmax = max_over_ranks(1.0 + rank, torch.device("cpu"))
        q.put((rank, g.numpy().tolist(), tmax))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("total", [1, 2, 7, 128])
def test_gather_rows_world2(total):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, g, tmax in res:
        assert [row[0] for row in g] == [float(i) for i in range(total)]
        assert tmax == 2.0


def test_shard_ids_partition():
    for total in (1, 5, 128, 1024):
        for world in (1, 2, 3, 8):
            allids = sorted(i for r in range(world) for i in shard_ids(total, world, r))
            assert allids == list(range(total))
            sizes = [len(shard_ids(total, world, r)) for r in range(world)]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_ids(4, 2, 2)


def _census_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, bench.rank_census(dist, world, rank, torch.device("cpu"))))
    finally:
        dist.destroy_process_group()


def test_bench_rank_census_world2():
    """bench.rank_census: every rank's view of the world, gathered with one all_gather (what the
    driver's multi-GPU line reports under config.ranks)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_census_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, census in res:
        assert [c["rank"] for c in census] == [0, 1]
        assert all(c["world_size_seen"] == 2 and not c["rccl"] for c in census)
