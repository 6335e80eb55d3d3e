"""GPU: the CFG-parallel latency mode through the native engine and flite_cfg_euler.

Two ranks share the box's one GPU (gloo carries the per-step exchange here; RCCL does on a multi-GPU node).
Each rank runs one CFG branch at batch 1. Bars: both ranks end bit-identical, bit-identical to a one-process
run of the same two batch-1 branches, and within 60 dB PSNR of the batched CFG loop (flite_dit_sample), whose
GEMMs run at twice the rows.
"""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no ROCm device", allow_module_level=True)

import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402
from _mp import pack, unpack  # noqa: E402

from f_lite import DiT, FLitePipeline  # noqa: E402
from f_lite import _native  # noqa: E402
from f_lite.model import PRESETS  # noqa: E402
from f_lite.pipeline import flow_schedule  # noqa: E402
from oracle import flite_ref as R  # noqa: E402

STEPS = 4
G = 6.0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs():
    g = torch.Generator().manual_seed(21)
    lat = torch.randn(1, 16, 16, 16, generator=g).bfloat16()
    pos = torch.randn(1, 24, 128, generator=g).bfloat16()
    neg = torch.randn(1, 24, 128, generator=g).bfloat16()
    return lat, pos, neg


def _worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2")
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=2)
        from f_lite.distributed import cfg_parallel_sample

        lat, pos, neg = _inputs()
        m = DiT.random(seed=0, device="cuda", **PRESETS["tiny"])
        acc = cfg_parallel_sample(m, lat.cuda(), pos.cuda(), neg.cuda(), num_inference_steps=STEPS,
                                  guidance_scale=G)
        pipe = FLitePipeline(m)
        pipe.enable_cfg_parallel()
        via_pipe = pipe(prompt_embeds=pos.cuda(), negative_prompt_embeds=neg.cuda(), latents=lat.cuda(),
                        height=128, width=128, num_inference_steps=STEPS, guidance_scale=G,
                        output_type="latent").images
        # latents=None with a DIFFERENT seed per rank: the ranks must still integrate rank 0's noise
        own = pipe(prompt_embeds=pos.cuda(), negative_prompt_embeds=neg.cuda(), height=128, width=128,
                   num_inference_steps=STEPS, guidance_scale=G, output_type="latent",
                   generator=torch.Generator().manual_seed(100 + rank)).images
        lat0 = torch.randn(1, 16, 16, 16, generator=torch.Generator().manual_seed(100), dtype=torch.bfloat16)
        explicit = cfg_parallel_sample(m, lat0.cuda(), pos.cuda(), neg.cuda(), num_inference_steps=STEPS,
                                       guidance_scale=G)
        torch.cuda.synchronize()
        q.put(pack((rank, acc.cpu())))
        q.put(pack((rank + 2, via_pipe.cpu())))
        q.put(pack((rank + 4, own.cpu())))
        q.put(pack((rank + 6, explicit.cpu())))
        dist.destroy_process_group()
    except Exception as e:  # report instead of leaving the parent waiting
        q.put((rank, repr(e)))


@pytest.fixture(scope="module")
def two_rank_result():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    while len(res) < 8 and not any(isinstance(v, str) for v in res.values()):
        k, v = unpack(q.get(timeout=100))
        res[k] = v
    for p in procs:
        p.join(30)
        if p.is_alive():  # a rank stuck in the exchange after its peer failed
            p.kill()
            p.join(10)
    for r in sorted(res):
        assert isinstance(res[r], torch.Tensor), f"rank {r}: {res[r]}"
    return res


def _one_process_branches():
    """The same two batch-1 branches in one process, one engine per branch."""
    lat, pos, neg = _inputs()
    mu = DiT.random(seed=0, device="cuda", **PRESETS["tiny"])
    mc = DiT.random(seed=0, device="cuda", **PRESETS["tiny"])
    sched = flow_schedule(STEPS, 16, 16)
    t = torch.tensor([s for s, _ in sched], dtype=torch.float32, device="cuda")
    engs = []
    for m, ctx in ((mu, neg), (mc, pos)):
        e = m.engine()
        e.prepare(1, 16, 16, 24, STEPS)
        e.set_context(ctx.cuda().reshape(24, -1).contiguous(), [0, 24])
        e.set_timesteps(t, True)
        engs.append(e)
    acc = lat.cuda().float().contiguous()
    u = torch.empty_like(acc)
    c = torch.empty_like(acc)
    for i, (_, dt) in enumerate(sched):
        engs[0].forward(acc, u, i, 0)
        engs[1].forward(acc, c, i, 0)
        _native.cfg_euler_(acc, u, c, G, dt)
    return acc.cpu()


def test_ranks_agree_and_match_one_process(two_rank_result):
    assert torch.equal(two_rank_result[0], two_rank_result[1])
    assert torch.equal(two_rank_result[0], _one_process_branches())


def test_pipeline_surface(two_rank_result):
    """FLitePipeline.enable_cfg_parallel(): the same latents through the reference's __call__ surface."""
    assert torch.equal(two_rank_result[2], two_rank_result[0].bfloat16())
    assert torch.equal(two_rank_result[3], two_rank_result[2])


def test_per_rank_seeds_are_unified(two_rank_result):
    """Ranks seeded differently (latents=None, generator seed 100 + rank) integrate rank 0's noise and end
    equal to each other and to an explicit run on rank 0's latents (broadcast before the loop)."""
    assert torch.equal(two_rank_result[4], two_rank_result[5])
    assert torch.equal(two_rank_result[4], two_rank_result[6].bfloat16())
    assert torch.equal(two_rank_result[6], two_rank_result[7])


def test_matches_batched_cfg_loop_and_oracle(two_rank_result):
    lat, pos, neg = _inputs()
    m = DiT.random(seed=0, device="cuda", **PRESETS["tiny"])
    pipe = FLitePipeline(m)
    batched = pipe(prompt_embeds=pos.cuda(), negative_prompt_embeds=neg.cuda(), latents=lat.cuda(), height=128,
                   width=128, num_inference_steps=STEPS, guidance_scale=G, output_type="latent").images.float().cpu()
    got = two_rank_result[0]
    p_b = R.psnr(got, batched)
    ref = R.sample(R.RefDiT.random(R.PRESETS["tiny"], dtype=torch.float32), lat.float(), pos.float(), neg.float(),
                   num_steps=STEPS, guidance_scale=G, height=128, width=128, t_dtype=torch.bfloat16,
                   acc_dtype=torch.float32)
    p_o = R.psnr(got, ref)
    print(f"CFG-parallel vs batched loop: {p_b:.2f} dB; vs fp32 oracle: {p_o:.2f} dB")
    assert p_b >= 60.0
    assert p_o >= 35.0


def test_cfg_euler_matches_torch():
    g = torch.Generator().manual_seed(3)
    acc0, u, c = (torch.randn(2, 16, 8, 8, generator=g) for _ in range(3))
    acc = acc0.cuda()
    _native.cfg_euler_(acc, u.cuda(), c.cuda(), 6.0, 0.125)
    torch.testing.assert_close(acc.cpu(), acc0 + 0.125 * (u + 6.0 * (c - u)), rtol=1e-6, atol=1e-6)
    acc = acc0.cuda()
    _native.cfg_euler_(acc, None, c.cuda(), 6.0, 0.125, use_cfg=False)
    torch.testing.assert_close(acc.cpu(), acc0 + 0.125 * c, rtol=1e-6, atol=1e-6)
