"""CPU, world_size 2 (gloo): the multi-GPU path's host logic -- image sharding (image i -> rank i mod N),
the single context broadcast from rank 0, max-over-ranks timing."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from _mp import pack, unpack  # tensors by value: a worker may exit before the parent reads its result


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from f_lite.distributed import image_indices, max_over_ranks, process_group_info, timed_broadcast_context

    ctx = torch.full((1, 8, 16), float(rank + 1))
    if rank == 0:
        ctx = torch.arange(128, dtype=torch.float32).reshape(1, 8, 16)
    # bench.py's path: the timed context broadcast, then what the process group reports about itself
    ms = timed_broadcast_context(ctx, src=0)
    mine = image_indices(8, rank, world)
    t = max_over_ranks(1.0 + rank)
    q.put((rank, ctx.sum().item(), mine, t, ms, process_group_info()))
    dist.destroy_process_group()


def _rows_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from f_lite.distributed import all_gather_rows

    send = torch.full((5,), rank + 1, dtype=torch.uint8)
    recv = torch.empty(5 * world, dtype=torch.uint8)
    all_gather_rows(send, recv)
    q.put((rank, recv.tolist()))
    dist.destroy_process_group()


def _ring_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from f_lite.distributed import ring_shift_rows

    # the engine's buffer protocol (flite.h, flite_dit_sp_set_ring): shift k sends kv_send (k = 1) or ring slot
    # (k - 2) & 1 and receives into slot (k - 1) & 1; the attention of step k reads slot (k - 1) & 1
    send = torch.full((6,), rank + 1, dtype=torch.uint8)
    slots = torch.zeros(2 * 6, dtype=torch.uint8)
    slot = lambda i: slots[6 * i:6 * (i + 1)]  # noqa: E731
    seen = []
    for k in range(1, world):
        ring_shift_rows(send if k == 1 else slot((k - 2) & 1), slot((k - 1) & 1))
        seen.append(int(slot((k - 1) & 1)[0]) - 1)
    q.put((rank, seen))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_ring_shift_rows(world):
    """The ring exchange of the sequence-parallel mode (distributed.ring_shift_rows): after shift k every rank
    holds the block of rank (r - k) mod N, so the N - 1 steps visit every other rank's keys exactly once."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ring_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=60) for _ in range(world))
    for p in procs:
        p.join(30)
    for r in range(world):
        assert res[r] == [(r - k) % world for k in range(1, world)]


@pytest.mark.parametrize("world", [2, 3])
def test_all_gather_rows(world):
    """The sequence-parallel exchange (distributed.all_gather_rows): rank-ordered concatenation."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rows_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=60) for _ in range(world))
    for p in procs:
        p.join(30)
    want = [r + 1 for r in range(world) for _ in range(5)]
    assert all(res[r] == want for r in range(world))


def _cfg_parallel_worker(rank, world, port, q):
    """One rank of the CFG-parallel loop; the branch forward is the fp32 oracle (test infrastructure)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from f_lite.distributed import cfg_parallel_loop
    from oracle import flite_ref as R

    lat, pos, neg = _cfg_inputs()
    ref = R.RefDiT.random(R.PRESETS["tiny"], dtype=torch.float32)
    sched = R.schedule(4, 128, 128)
    ctx = neg if rank == 0 else pos  # uncond on rank 0 (pipeline.py:266)

    def forward_branch(x, i):
        return ref(x, ctx, None, torch.tensor([sched[i][0]] * x.shape[0], dtype=torch.float32))

    def update(x, u, c, dt):
        x += dt * (u + 6.0 * (c - u))

    acc = cfg_parallel_loop(lat.clone(), [t for t, _ in sched], [dt for _, dt in sched], forward_branch, update)
    q.put((rank, pack(acc)))
    dist.destroy_process_group()


def _cfg_inputs():
    g = torch.Generator().manual_seed(11)
    lat = torch.randn(1, 16, 16, 16, generator=g)
    pos = torch.randn(1, 24, 128, generator=g)
    neg = torch.randn(1, 24, 128, generator=g)
    return lat, pos, neg


def test_cfg_parallel_loop_matches_batched_oracle():
    """CFG-parallel host logic: 2 ranks, one branch each, one all-gather per step; both
    ranks end with the same latents, equal to the batched CFG loop of pipeline.py:250-297 (fp32 oracle)."""
    from oracle import flite_ref as R

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cfg_parallel_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: unpack(v) for r, v in (q.get(timeout=180) for _ in range(2))}
    for p in procs:
        p.join(60)
    assert torch.equal(res[0], res[1])
    lat, pos, neg = _cfg_inputs()
    ref = R.sample(R.RefDiT.random(R.PRESETS["tiny"], dtype=torch.float32), lat, pos, neg, num_steps=4,
                   guidance_scale=6.0, height=128, width=128, t_dtype=torch.float32, acc_dtype=torch.float32)
    assert torch.allclose(res[0], ref, rtol=1e-4, atol=1e-4), (res[0] - ref).abs().max()


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
    for rank, s, mine, t, ms, pg in res:
        assert s == expect  # every rank sees rank 0's context
        assert t == float(world)  # slowest rank's time
        assert ms >= 0.0
        assert pg == {"backend": "gloo", "world_size_seen": world, "rank_seen": rank}
        shards += mine
    assert sorted(shards) == list(range(8))  # every image exactly once


def _dp_apg_worker(rank, world, port, q):
    """One rank of the data-parallel loop with APG: its images of the batch, the branch forward by the fp32
    oracle (test infrastructure), APG's sums all-reduced between the two phases (distributed.apg_step)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from f_lite.distributed import all_reduce_sum_, apg_step, data_parallel_loop, gather_images, image_indices
    from oracle import flite_ref as R

    lat, pos, neg = _dp_inputs()
    mine = image_indices(lat.shape[0], rank, world)
    ref = R.RefDiT.random(R.PRESETS["tiny"], dtype=torch.float32)
    sched = R.schedule(4, 128, 128)
    ctx = torch.cat([neg[mine], pos[mine]])

    def forward_pair(x, i):
        out = ref(torch.cat([x, x]), ctx, None, torch.tensor([sched[i][0]] * 2 * x.shape[0]))
        return out.chunk(2)

    def sums(u, c, k, phase):
        if phase == 0:
            return torch.stack([(c * (c - u)).sum(), (c * c).sum()])
        o = (c - u) - k * c
        return torch.stack([o.sum(), (o * o).sum()])

    def update(a, u, c, gs, k, sc, dt):
        a += dt * (c + (gs - 1) * sc * ((c - u) - k * c))

    n_total = lat.numel()

    def combine(x, u, c, dt):
        apg_step(x, u, c, dt, 6.0, 0.03, n_total, sums, update, reduce=all_reduce_sum_)

    acc = data_parallel_loop(lat[mine].clone(), [dt for _, dt in sched], forward_pair, combine)
    q.put((rank, pack(gather_images(acc, lat.shape[0]))))
    dist.destroy_process_group()


def _dp_inputs():
    g = torch.Generator().manual_seed(12)
    lat = torch.randn(3, 16, 16, 16, generator=g)
    pos = torch.randn(3, 24, 128, generator=g)
    neg = torch.randn(3, 24, 128, generator=g)
    return lat, pos, neg


@pytest.mark.parametrize("world", [2, 3])
def test_data_parallel_apg_matches_batched_oracle(world):
    """one reference batch (3 images) sharded over the ranks (image i -> rank i mod N) with APG on;
    the batch-global sums are all-reduced twice per step, and every rank ends with the batched APG loop's
    latents (pipeline.py:250-297, fp32 oracle)."""
    from oracle import flite_ref as R

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_apg_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: unpack(v) for r, v in (q.get(timeout=240) for _ in range(world))}
    for p in procs:
        p.join(60)
    for r in range(1, world):
        assert torch.equal(res[0], res[r])
    lat, pos, neg = _dp_inputs()
    ref = R.sample(R.RefDiT.random(R.PRESETS["tiny"], dtype=torch.float32), lat, pos, neg, num_steps=4,
                   guidance_scale=6.0, apg=R.APG(enabled=True), height=128, width=128, t_dtype=torch.float32,
                   acc_dtype=torch.float32)
    assert torch.allclose(res[0], ref, rtol=1e-4, atol=1e-4), (res[0] - ref).abs().max()
