"""Multi-GPU sampling: independent images sharded one per GPU (replica data parallelism).

The reference has no multi-GPU inference; its torch.distributed use is training-only
(f_lite/distributed.py:71-80, NCCL). Here every rank holds a full copy of the weights (22 GB of bf16 for the
10B model, far below the 288 GB of HBM) and generates its own images; the only collective is one broadcast of
the shared text embedding from rank 0 (RCCL over xGMI with the "nccl" backend), before the denoise loop.
No per-step communication. APG's batch-global reductions (pipeline.py:281-285) couple the images of one
reference batch: `data_parallel_sample` shards ONE batch over the ranks and all-reduces APG's partial sums
twice per step (2 floats each), so the result is the batched loop's.

Second mode, for single-image latency: CFG-parallel, the uncond and cond branches of the
same image on two ranks with one all-gather of the branch outputs per step (`cfg_parallel_sample`).

Third mode, single-image latency over any number of GPUs ("ring attention over T"):
sequence parallelism (`sequence_parallel_sample`). Each rank holds a 1/N slice of the token rows of both CFG
sequences; the native engine all-gathers the K/V rows once per block (the only data the self-attention needs
from other ranks) and the output rows once per step, through `all_gather_rows`.
"""
from __future__ import annotations

import os
from typing import Callable, List, Optional

import numpy as np
import torch


def world() -> "tuple[int, int, int]":
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("LOCAL_RANK", "0"))


def image_indices(n_images: int, rank: int, world_size: int) -> List[int]:
    """Global image indices owned by `rank`: image i -> rank i mod world_size."""
    return list(range(rank, n_images, world_size))


def broadcast_context(ctx: torch.Tensor, src: int = 0, group=None) -> torch.Tensor:
    """The one collective of the path: the shared text embedding from rank `src` to every rank (in place)."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        if dist.get_backend(group) == "gloo" and ctx.device.type != "cpu":  # CPU tests / ranks sharing a GPU
            host = ctx.detach().cpu()
            dist.broadcast(host, src=src, group=group)
            ctx.copy_(host)
        else:
            dist.broadcast(ctx, src=src, group=group)
    return ctx


def timed_broadcast_context(ctx: torch.Tensor, src: int = 0, group=None) -> float:
    """broadcast_context with its wall time in ms (device synchronised on both sides when ctx is on a GPU; the first
    collective of a process group includes the communicator's set-up). bench.py records it per rank."""
    import time

    sync = torch.cuda.synchronize if ctx.device.type == "cuda" else (lambda: None)
    sync()
    t0 = time.perf_counter()
    broadcast_context(ctx, src=src, group=group)
    sync()
    return (time.perf_counter() - t0) * 1000.0


def process_group_info(group=None):
    """What the process group itself reports (None without one): backend, world size and rank as seen by
    torch.distributed, and the RCCL version under the nccl backend; bench.py puts it in the line's "distributed" so a
    multi-GPU run says what it actually ran over."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return None
    info = {"backend": dist.get_backend(group), "world_size_seen": dist.get_world_size(group),
            "rank_seen": dist.get_rank(group)}
    if info["backend"] == "nccl":
        try:
            info["rccl_version"] = ".".join(map(str, torch.cuda.nccl.version()))
        except Exception:  # pragma: no cover - version query unsupported
            pass
    return info


def broadcast_from_group_root(t: torch.Tensor, group=None) -> torch.Tensor:
    """In-place broadcast of `t` from rank 0 OF `group` (its global rank resolved) to the group's ranks. With
    gloo (CPU tests, or two ranks sharing one GPU) a device tensor is staged through the host."""
    import torch.distributed as dist

    src = 0 if group is None else dist.get_global_rank(group, 0)
    if dist.get_backend(group) == "gloo" and t.device.type != "cpu":
        host = t.detach().cpu()
        dist.broadcast(host, src=src, group=group)
        t.copy_(host)
    else:
        dist.broadcast(t, src=src, group=group)
    return t


def exchange_branches(out: torch.Tensor, group=None) -> "List[torch.Tensor]":
    """All-gather of the per-rank CFG branch outputs: [uncond (rank 0), cond (rank 1)]. With the "nccl"
    backend (RCCL over xGMI) device tensors move directly; gloo (CPU tests) stages through the host."""
    import torch.distributed as dist

    staged = out.cpu() if dist.get_backend(group) == "gloo" else out
    bufs = [torch.empty_like(staged) for _ in range(dist.get_world_size(group))]
    dist.all_gather(bufs, staged.contiguous(), group=group)
    return [b.to(out.device) for b in bufs]


def cfg_parallel_loop(acc: torch.Tensor, t_list, dt_list, forward_branch, update, group=None) -> torch.Tensor:
    """The denoise loop of FLitePipeline.__call__ (pipeline.py:250-297) with the CFG pair split over the two
    ranks of `group`: rank 0 runs the uncond branch, rank 1 the cond branch (the batch order of
    pipeline.py:264-268). Per step each rank runs forward_branch(acc, step) -> [B, C, h, w] fp32, the two
    outputs are exchanged (one all-gather of B*C*h*w fp32: 1 MiB per image at 1024^2), and both ranks apply the
    same update(acc, u, c, dt), so their accumulators stay identical."""
    import torch.distributed as dist

    if dist.get_world_size(group) != 2:
        raise ValueError("CFG-parallel sampling needs a group of exactly 2 ranks (uncond, cond)")
    for i, dt in enumerate(dt_list):
        u, c = exchange_branches(forward_branch(acc, i), group)
        update(acc, u, c, dt)
    return acc


def all_reduce_sum_(t: torch.Tensor, group=None) -> torch.Tensor:
    """In-place SUM over the group's ranks (RCCL on device tensors; gloo stages a device tensor via the host)."""
    import torch.distributed as dist

    if dist.get_backend(group) == "gloo" and t.device.type != "cpu":
        host = t.detach().cpu()
        dist.all_reduce(host, group=group)
        t.copy_(host)
    else:
        dist.all_reduce(t, group=group)
    return t


def apg_step(acc, u, c, dt: float, guidance: float, threshold: float, n_total: int,
             sums: Callable, update: Callable, reduce: Optional[Callable] = None):
    """One APG + Euler update (pipeline.py:276-287,296) with the batch-global sums taken in two phases:
    sums(u, c, k, phase) -> 2 floats (phase 0: [sum dy*dd, sum dy^2]; phase 1: [sum o, sum o^2]), each optionally
    all-reduced by reduce() (ranks holding different images of the batch), then update(acc, u, c, g, k, s, dt).
    The scalar algebra is the fp32 arithmetic of the single-launch APG kernel (elementwise.hip
    apg_euler_kernel): k = dydd / dyy, unbiased variance (soo - mean so) / (n - 1), s = min(1, thr / std)."""
    f32 = np.float32
    s0 = sums(u, c, 0.0, 0)
    if reduce is not None:
        reduce(s0)
    dydd, dyy = (f32(v) for v in s0.tolist())
    k = dydd / dyy if dyy > 0 else f32(0)
    s1 = sums(u, c, float(k), 1)
    if reduce is not None:
        reduce(s1)
    so, soo = (f32(v) for v in s1.tolist())
    mean = so / f32(n_total)
    var = np.maximum(soo - mean * so, f32(0)) / f32(n_total - 1) if n_total > 1 else f32(0)
    sd = np.sqrt(f32(var))
    sc = np.minimum(f32(1), f32(threshold) / sd) if sd > 0 else f32(1)
    update(acc, u, c, guidance, float(k), float(sc), dt)
    return acc


def apg_step_device(acc, u, c, dt: float, guidance: float, threshold: float, n_total: int, ws: torch.Tensor,
                    reduce: Optional[Callable] = None):
    """apg_step with the scalars kept on the device (include/flite.h flite_apg_sums_dev / flite_apg_euler_dev):
    the two partial sums of each phase land in the 4-float device tensor `ws`, are optionally all-reduced IN PLACE
    (RCCL on the device tensor: stream-ordered, no host round trip), and the kernels derive k and the orthogonal
    scale from them with the fp32 expressions of the single-launch APG kernel. A rank without images (u empty)
    joins the reductions with zeros."""
    from . import _native

    have = u.numel() > 0
    for phase in (0, 1):
        if have:
            _native.apg_sums_dev(u, c, phase, ws)
        else:
            ws[2 * phase: 2 * phase + 2].zero_()
        if reduce is not None:
            reduce(ws[2 * phase: 2 * phase + 2])
    if have:
        _native.apg_euler_dev_(acc, u, c, guidance, threshold, n_total, ws, dt)
    return acc


def _broadcast_inputs(group, *ts):
    """Private contiguous copies of the inputs, overwritten with the group root's values (the caller's tensors
    are never modified)."""
    out = [t.clone(memory_format=torch.contiguous_format) for t in ts]
    for t in out:
        broadcast_from_group_root(t, group)
    return out


def cfg_parallel_sample(dit, latents: torch.Tensor, prompt_embeds: torch.Tensor,
                        negative_prompt_embeds: Optional[torch.Tensor] = None, num_inference_steps: int = 30,
                        guidance_scale: float = 6.0, alpha: Optional[float] = None, group=None,
                        apg=None) -> torch.Tensor:
    """Single-image latency mode: the two CFG branches of the same images run on two GPUs
    (B = n_img per launch instead of 2 n_img), exchanging their outputs once per step; the native CFG + Euler
    update (flite_cfg_euler) runs on both ranks. Every rank passes the same latents and embeddings and gets
    the final fp32 latents [n_img, 16, h, w]. Weights are replicated; the branch context (negative on rank 0,
    positive on rank 1) feeds the step-invariant cross-attention K/V cache once. With `apg` (an APGConfig
    with enabled=True) the update is APG: after the exchange every rank holds both branches of every image, so
    the batch-global sums need no collective, and they equal the batched kernel's bit for bit."""
    import torch.distributed as dist

    from . import _native
    from .pipeline import flow_schedule

    if guidance_scale < 1.0:
        raise ValueError("CFG-parallel sampling needs classifier-free guidance (guidance_scale >= 1)")
    rank = dist.get_rank(group)
    eng = dit.engine()
    dev = dit.device
    n_img, _, lh, lw = latents.shape
    pos = prompt_embeds.to(device=dev, dtype=torch.bfloat16)
    neg = torch.zeros_like(pos) if negative_prompt_embeds is None else \
        negative_prompt_embeds.to(device=dev, dtype=torch.bfloat16)  # pipeline.py:160-161
    if neg.shape != pos.shape or pos.shape[0] != n_img:
        raise ValueError("prompt / negative embeddings must both be [n_img, L, C_ctx]")
    # Both branches must integrate the SAME noise and embeddings: ranks that drew their own latents (e.g.
    # seeded with seed + rank, or after uneven RNG use) would otherwise each return a wrong image silently.
    # One broadcast from the group's first rank before the loop, like broadcast_context.
    lat, pos, neg = _broadcast_inputs(group, latents.to(device=dev, dtype=torch.bfloat16), pos, neg)
    ctx = neg if rank == 0 else pos
    L = ctx.shape[1]
    sched = flow_schedule(num_inference_steps, lh, lw, alpha)
    t_list = [t for t, _ in sched]
    dt_list = [dt for _, dt in sched]
    eng.prepare(n_img, lh, lw, n_img * L, num_inference_steps)
    eng.set_context(ctx.reshape(n_img * L, -1), [i * L for i in range(n_img + 1)])
    # one timestep row per step, shared by the batch (pipeline.py:260,268), as in flite_dit_sample
    eng.set_timesteps(torch.tensor(t_list, dtype=torch.float32, device=dev), bool(eng.cfg.bf16_timestep_quant))
    acc = lat.float().contiguous()
    out = torch.empty_like(acc)

    def forward_branch(x, i):
        return eng.forward(x, out, i, 0)

    if apg is not None and apg.enabled:
        ws = torch.zeros(4, device=dev, dtype=torch.float32)

        def update(x, u, c, dt):
            apg_step_device(x, u, c, dt, guidance_scale, apg.orthogonal_threshold, x.numel(), ws)
    else:
        def update(x, u, c, dt):
            _native.cfg_euler_(x, u, c, guidance_scale, dt)

    return cfg_parallel_loop(acc, t_list, dt_list, forward_branch, update, group)


def gather_images(local: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """Inverse of image_indices: every rank's images (rank r holds images r, r + N, ...) -> the whole batch
    [n_total, ...] on every rank (one all-gather of equal, zero-padded blocks)."""
    import torch.distributed as dist

    rank, n = dist.get_rank(group), dist.get_world_size(group)
    per = -(-n_total // n)
    blk = torch.zeros((per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    blk[: local.shape[0]] = local
    if dist.get_backend(group) == "gloo" and local.device.type != "cpu":
        host = blk.cpu()
        parts = [torch.empty_like(host) for _ in range(n)]
        dist.all_gather(parts, host, group=group)
        parts = [p.to(local.device) for p in parts]
    else:
        parts = [torch.empty_like(blk) for _ in range(n)]
        dist.all_gather(parts, blk, group=group)
    out = torch.empty((n_total,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    for r in range(n):
        idx = image_indices(n_total, r, n)
        if idx:
            out[idx[0]::n] = parts[r][: len(idx)]
    return out


def data_parallel_loop(acc, dt_list, forward_pair: Callable, combine: Callable):
    """The denoise loop with this rank's images of the batch: forward_pair(acc, step) -> (u, c) of the local
    images, combine(acc, u, c, dt) the CFG / APG update (APG all-reduces its sums inside, see apg_step)."""
    for i, dt in enumerate(dt_list):
        u, c = forward_pair(acc, i)
        combine(acc, u, c, dt)
    return acc


def data_parallel_sample(dit, latents: torch.Tensor, prompt_embeds: torch.Tensor,
                         negative_prompt_embeds: Optional[torch.Tensor] = None, num_inference_steps: int = 30,
                         guidance_scale: float = 6.0, alpha: Optional[float] = None, group=None,
                         apg=None) -> torch.Tensor:
    """ONE reference batch of images sharded over the ranks of `group` (image i -> rank i mod N):
    each rank runs the CFG batch of its own images; with APG the batch-global sums of pipeline.py:281-285 are
    all-reduced (two 2-float all-reduces per step), so the images equal the batched loop's up to the order of
    the fp32 partial sums. Every rank passes the same inputs and gets the whole batch's final fp32 latents
    (one all-gather at the end). The DiT launches run eagerly (the per-step collective sits between them)."""
    import torch.distributed as dist

    from . import _native
    from .pipeline import flow_schedule

    if guidance_scale < 1.0:
        raise ValueError("data_parallel_sample runs the CFG loop (guidance_scale >= 1)")
    rank, n = dist.get_rank(group), dist.get_world_size(group)
    eng = dit.engine()
    dev = dit.device
    n_img, C, lh, lw = latents.shape
    pos = prompt_embeds.to(device=dev, dtype=torch.bfloat16)
    neg = torch.zeros_like(pos) if negative_prompt_embeds is None else \
        negative_prompt_embeds.to(device=dev, dtype=torch.bfloat16)  # pipeline.py:160-161
    if neg.shape != pos.shape or pos.shape[0] != n_img:
        raise ValueError("prompt / negative embeddings must both be [n_img, L, C_ctx]")
    lat, pos, neg = _broadcast_inputs(group, latents.to(device=dev, dtype=torch.bfloat16), pos, neg)
    mine = image_indices(n_img, rank, n)
    b = len(mine)
    sched = flow_schedule(num_inference_steps, lh, lw, alpha)
    dt_list = [dt for _, dt in sched]
    acc = lat[mine].float().contiguous()
    use_apg = apg is not None and apg.enabled
    if b:
        L = pos.shape[1]
        ctx = torch.cat([neg[mine], pos[mine]]).reshape(2 * b * L, -1).contiguous()  # uncond first
        eng.prepare(2 * b, lh, lw, 2 * b * L, num_inference_steps)
        eng.set_context(ctx, [i * L for i in range(2 * b + 1)])
        eng.set_timesteps(torch.tensor([t for t, _ in sched], dtype=torch.float32, device=dev),
                          bool(eng.cfg.bf16_timestep_quant))
        x2 = torch.empty((2 * b, C, lh, lw), device=dev, dtype=torch.float32)
        out = torch.empty_like(x2)

        def forward_pair(x, i):
            x2[:b].copy_(x)
            x2[b:].copy_(x)
            eng.forward(x2, out, i, 0)
            return out[:b], out[b:]
    else:  # more ranks than images: this rank still joins APG's all-reduces with zero partial sums
        zero = torch.zeros((0, C, lh, lw), device=dev, dtype=torch.float32)

        def forward_pair(x, i):
            return zero, zero

    if use_apg:
        n_total = n_img * C * lh * lw
        ws = torch.zeros(4, device=dev, dtype=torch.float32)

        def combine(x, u, c, dt):  # two 2-float all-reduces per step, on the device (no .tolist())
            apg_step_device(x, u, c, dt, guidance_scale, apg.orthogonal_threshold, n_total, ws,
                            reduce=lambda t: all_reduce_sum_(t, group))
    else:
        def combine(x, u, c, dt):
            if b:
                _native.cfg_euler_(x, u, c, guidance_scale, dt)

    data_parallel_loop(acc, dt_list, forward_pair, combine)
    return gather_images(acc, n_img, group)


def all_gather_rows(send: torch.Tensor, recv: torch.Tensor, group=None) -> None:
    """recv = cat over the group's ranks (rank order) of `send` (flat device buffers). RCCL all-gather over
    xGMI with the "nccl" backend; gloo (tests, ranks sharing one GPU) stages through the host."""
    import torch.distributed as dist

    if dist.get_backend(group) == "gloo":
        host = send.cpu()
        parts = [torch.empty_like(host) for _ in range(dist.get_world_size(group))]
        dist.all_gather(parts, host, group=group)
        recv.copy_(torch.cat(parts))
    else:
        dist.all_gather_into_tensor(recv, send, group=group)


def ring_shift_rows(send: torch.Tensor, recv: torch.Tensor, group=None) -> None:
    """One ring step: send `send` to the next rank of the group and receive the previous rank's block into `recv`
    (equal sizes). RCCL send/recv over one xGMI link with "nccl"; gloo stages through the host."""
    import torch.distributed as dist

    n = dist.get_world_size(group)
    r = dist.get_rank(group)
    nxt = dist.get_global_rank(group, (r + 1) % n) if group is not None else (r + 1) % n
    prv = dist.get_global_rank(group, (r - 1) % n) if group is not None else (r - 1) % n
    if dist.get_backend(group) == "gloo":
        host = send.cpu()
        buf = torch.empty_like(host)
        reqs = [dist.isend(host, nxt, group=group), dist.irecv(buf, prv, group=group)]
        for q in reqs:
            q.wait()
        recv.copy_(buf)
    else:
        ops = [dist.P2POp(dist.isend, send, nxt, group), dist.P2POp(dist.irecv, recv, prv, group)]
        for q in dist.batch_isend_irecv(ops):
            q.wait()


def sequence_parallel_sample(dit, latents: torch.Tensor, prompt_embeds: torch.Tensor,
                             negative_prompt_embeds: Optional[torch.Tensor] = None, num_inference_steps: int = 30,
                             guidance_scale: float = 6.0, alpha: Optional[float] = None, group=None,
                             ring: bool = False, apg=None) -> torch.Tensor:
    """Single-image latency mode over the N ranks of `group`: the denoise loop of
    FLitePipeline.__call__ (pipeline.py:250-297) with every DiT launch split by token rows. Rank r computes rows
    [r*Tl, (r+1)*Tl) of each sequence of the CFG batch (Tl = ceil(T / N)); per block its K/V rows are
    all-gathered (2 x T x D bf16 per sequence), per step the output rows. Every rank ends each step with the
    full model output and applies the same native CFG + Euler update, so all ranks return the same final fp32
    latents [n_img, 16, h, w]. Weights are replicated. Latents and embeddings are broadcast from the group's
    first rank first (ranks may have drawn different noise). ring=True moves the self-attention's keys as N - 1
    neighbour shifts (ring attention), each overlapped with the attention over the previous block, instead of
    one all-gather. With `apg` enabled the update is APG; every rank holds the whole model output after the
    per-step gather, so its batch-global sums need no further collective."""
    import torch.distributed as dist

    from .pipeline import flow_schedule

    rank, n = dist.get_rank(group), dist.get_world_size(group)
    eng = dit.engine()
    dev = dit.device
    n_img, _, lh, lw = latents.shape
    pos = prompt_embeds.to(device=dev, dtype=torch.bfloat16).contiguous()
    do_cfg = guidance_scale >= 1.0
    neg = torch.zeros_like(pos) if negative_prompt_embeds is None else \
        negative_prompt_embeds.to(device=dev, dtype=torch.bfloat16).contiguous()  # pipeline.py:160-161
    if neg.shape != pos.shape or pos.shape[0] != n_img:
        raise ValueError("prompt / negative embeddings must both be [n_img, L, C_ctx]")
    lat, pos, neg = _broadcast_inputs(group, latents.to(device=dev, dtype=torch.bfloat16), pos, neg)
    use_apg = bool(apg is not None and apg.enabled and do_cfg)
    ctx = torch.cat([neg, pos]) if do_cfg else pos  # uncond first (pipeline.py:266)
    nseq, L = ctx.shape[0], ctx.shape[1]
    sched = flow_schedule(num_inference_steps, lh, lw, alpha)
    acc = lat.float().contiguous()
    eng.set_sequence_parallel(rank, n, lambda s, r: all_gather_rows(s, r, group),
                              (lambda s, r: ring_shift_rows(s, r, group)) if ring else None)
    try:
        eng.prepare(nseq, lh, lw, nseq * L, num_inference_steps, device=dev)
        eng.set_context(ctx.reshape(nseq * L, -1).contiguous(), [i * L for i in range(nseq + 1)])
        eng.sample(acc, n_img, [t for t, _ in sched], [dt for _, dt in sched], guidance_scale, do_cfg,
                   apg=use_apg, apg_thr=apg.orthogonal_threshold if use_apg else 0.03, use_graph=False)
    finally:
        eng.set_sequence_parallel(0, 1)
    return acc


def max_over_ranks(seconds: float, device=None, group=None) -> float:
    """Job wall time = the slowest rank's time (bench.py contract)."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return seconds
    if dist.get_backend(group) == "gloo":
        device = "cpu"  # CPU tests / ranks sharing a GPU
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
