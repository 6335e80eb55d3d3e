"""CPU, world_size 2 (gloo): the multi-GPU path's host logic -- image sharding (image i -> rank i mod N),
the single context broadcast from rank 0, max-over-ranks timing."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from f_lite.distributed import broadcast_context, image_indices, max_over_ranks

    ctx = torch.full((1, 8, 16), float(rank + 1))
    if rank == 0:
        ctx = torch.arange(128, dtype=torch.float32).reshape(1, 8, 16)
    broadcast_context(ctx, src=0)
    mine = image_indices(8, rank, world)
    t = max_over_ranks(1.0 + rank)
    q.put((rank, ctx.sum().item(), mine, t))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharding_and_broadcast(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
    expect = float(sum(range(128)))
    shards = []
    for rank, s, mine, t in res:
        assert s == expect  # every rank sees rank 0's context
        assert t == float(world)  # slowest rank's time
        shards += mine
    assert sorted(shards) == list(range(8))  # every image exactly once
