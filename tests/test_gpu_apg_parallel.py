"""GPU: APG (pipeline.py:276-287) in the multi-rank modes, through the native engine.

APG's sums and its std run over the WHOLE batch tensor, so they couple the CFG branches and the images of a
reference batch:
  * CFG-parallel: after the per-step exchange each rank holds both branches of every image, so the split APG
    kernels (flite_apg_sums / flite_apg_euler) run locally -- same expressions and summation order as the
    batched loop's single-launch APG kernel;
  * sequence parallel: every rank holds the whole model output after the per-step gather; the engine's own APG
    kernel runs on it;
  * data parallel (one batch of 3 images sharded over 2 ranks, image i -> rank i mod 2): the partial sums are
    all-reduced between APG's two phases.
Two ranks share the box's one GPU; gloo carries the exchanges (RCCL does on a multi-GPU node). Bars: ranks
bit-identical; >= 50 dB vs the single-process batched APG loop (the launches differ in rows, so GEMM tiles and
summation order differ); >= 40 dB vs the fp32 oracle's batched APG loop.
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

from f_lite import APGConfig, DiT, FLitePipeline  # noqa: E402
from f_lite import _native  # noqa: E402
from f_lite.model import PRESETS  # noqa: E402
from oracle import flite_ref as R  # noqa: E402

STEPS = 4
G = 6.0
MODES = ("cfg", "dp", "sp")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(n):
    g = torch.Generator().manual_seed(31)
    lat = torch.randn(n, 16, 16, 16, generator=g).bfloat16()
    pos = torch.randn(n, 24, 128, generator=g).bfloat16()
    neg = torch.randn(n, 24, 128, generator=g).bfloat16()
    return lat, pos, neg


def _worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2")
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=2)
        from f_lite.distributed import cfg_parallel_sample, data_parallel_sample, sequence_parallel_sample

        apg = APGConfig(enabled=True)
        m = DiT.random(seed=0, device="cuda", **PRESETS["tiny"])
        lat, pos, neg = _inputs(2)
        q.put(pack(("cfg", rank, cfg_parallel_sample(m, lat.cuda(), pos.cuda(), neg.cuda(), STEPS, G, apg=apg).cpu())))
        lat3, pos3, neg3 = _inputs(3)
        q.put(pack(("dp", rank, data_parallel_sample(m, lat3.cuda(), pos3.cuda(), neg3.cuda(), STEPS, G,
                                                     apg=apg).cpu())))
        # the pipeline surface of the data-parallel mode
        pipe = FLitePipeline(m)
        pipe.enable_data_parallel()
        out = pipe(prompt_embeds=pos3.cuda(), negative_prompt_embeds=neg3.cuda(), latents=lat3.cuda(), height=128,
                   width=128, num_inference_steps=STEPS, guidance_scale=G, apg_config=apg,
                   output_type="latent").images
        q.put(pack(("dp_pipe", rank, out.float().cpu())))
        q.put(pack(("sp", rank, sequence_parallel_sample(m, lat.cuda(), pos.cuda(), neg.cuda(), STEPS, G,
                                                         apg=apg).cpu())))
        torch.cuda.synchronize()
        dist.destroy_process_group()
    except Exception as e:  # report instead of leaving the parent waiting
        import traceback

        q.put(("error", rank, traceback.format_exc() + repr(e)))


@pytest.fixture(scope="module")
def results():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    while len(res) < 8:
        kind, rank, v = unpack(q.get(timeout=110))
        if kind == "error":
            for p in procs:
                p.kill()
            pytest.fail(f"rank {rank}: {v}")
        res[(kind, rank)] = v
    for p in procs:
        p.join(30)
        if p.is_alive():
            p.kill()
            p.join(10)
    return res


def _batched(n):
    """The single-process batched APG loop (flite_dit_sample's in-launch APG kernel) on the same inputs."""
    lat, pos, neg = _inputs(n)
    m = DiT.random(seed=0, device="cuda", **PRESETS["tiny"])
    return FLitePipeline(m)(prompt_embeds=pos.cuda(), negative_prompt_embeds=neg.cuda(), latents=lat.cuda(),
                            height=128, width=128, num_inference_steps=STEPS, guidance_scale=G,
                            apg_config=APGConfig(enabled=True), output_type="latent",
                            use_graph=False).images.float().cpu()


def _oracle(n):
    lat, pos, neg = _inputs(n)
    ref = R.RefDiT.random(R.PRESETS["tiny"], dtype=torch.float32)
    with torch.no_grad():
        return R.sample(ref, lat.float(), pos.float(), neg.float(), num_steps=STEPS, guidance_scale=G,
                        apg=R.APG(enabled=True), height=128, width=128, t_dtype=torch.bfloat16,
                        acc_dtype=torch.float32)


@pytest.mark.parametrize("mode", MODES + ("dp_pipe",))
def test_apg_parallel_mode(results, mode):
    a, b = results[(mode, 0)], results[(mode, 1)]
    assert torch.equal(a, b), f"{mode}: ranks differ"
    n = 3 if mode.startswith("dp") else 2
    assert a.shape == (n, 16, 16, 16)
    batched = _batched(n)
    ora = _oracle(n)
    p_b, p_o = R.psnr(a, batched), R.psnr(a, ora)
    print(f"APG {mode}: {p_b:.2f} dB vs the batched native loop, {p_o:.2f} dB vs the fp32 oracle "
          f"(batched native vs oracle {R.psnr(batched, ora):.2f} dB)")
    assert p_b >= 50.0 and p_o >= 40.0


def test_apg_split_kernels_match_single_launch():
    """flite_apg_sums + flite_apg_euler (distributed.apg_step, no reduction) == the reference APG expression,
    and == the single-launch kernel inside flite_dit_sample for one rank holding the whole batch (checked
    through the CFG-parallel result above)."""
    from f_lite.distributed import apg_step

    g = torch.Generator().manual_seed(4)
    u = torch.randn(2, 16, 64, 64, generator=g)
    c = u + 0.2 * torch.randn(2, 16, 64, 64, generator=g)
    acc = torch.randn(2, 16, 64, 64, generator=g)
    got = acc.cuda()
    apg_step(got, u.cuda(), c.cuda(), 0.05, G, 0.03, u.numel(), _native.apg_sums,
             lambda a, uu, cc, gs, k, sc, dt: _native.apg_euler_(a, uu, cc, gs, k, sc, dt))
    dy, dd = c.double(), (c - u).double()
    orth = dd - (dy * dd).sum() / (dy * dy).sum() * dy
    want = acc.double() + 0.05 * (dy + (G - 1) * orth * min(1.0, 0.03 / orth.std().item()))
    torch.testing.assert_close(got.cpu().double(), want, rtol=1e-4, atol=1e-5)


def test_apg_device_scalars_match_host_algebra():
    """distributed.apg_step_device (flite_apg_sums_dev / flite_apg_euler_dev: k and the orthogonal scale derived on
    the device, no host round trip) == apg_step's host fp32 algebra to rounding, == the reference expression, and a
    split of the batch over two "ranks" whose partial sums are added in place reproduces the whole-batch step."""
    from f_lite.distributed import apg_step, apg_step_device

    g = torch.Generator().manual_seed(5)
    u = torch.randn(3, 16, 64, 64, generator=g)
    c = u + 0.2 * torch.randn(3, 16, 64, 64, generator=g)
    acc = torch.randn(3, 16, 64, 64, generator=g)
    host = acc.cuda()
    apg_step(host, u.cuda(), c.cuda(), 0.05, G, 0.03, u.numel(), _native.apg_sums,
             lambda a, uu, cc, gs, k, sc, dt: _native.apg_euler_(a, uu, cc, gs, k, sc, dt))
    dev = acc.cuda()
    ws = torch.zeros(4, device="cuda")
    apg_step_device(dev, u.cuda(), c.cuda(), 0.05, G, 0.03, u.numel(), ws)
    torch.testing.assert_close(dev, host, rtol=1e-6, atol=1e-6)
    dy, dd = c.double(), (c - u).double()
    orth = dd - (dy * dd).sum() / (dy * dy).sum() * dy
    want = acc.double() + 0.05 * (dy + (G - 1) * orth * min(1.0, 0.03 / orth.std().item()))
    torch.testing.assert_close(dev.cpu().double(), want, rtol=1e-4, atol=1e-5)
    # two shards (images {0, 2} and {1}); "reduce" adds the other shard's partial sums in place
    parts = [[0, 2], [1]]
    accs = [acc[p].cuda() for p in parts]
    wss = [torch.zeros(4, device="cuda") for _ in parts]
    for phase in (0, 1):
        for p, w in zip(parts, wss):
            _native.apg_sums_dev(u[p].cuda(), c[p].cuda(), phase, w)
        tot = wss[0][2 * phase: 2 * phase + 2] + wss[1][2 * phase: 2 * phase + 2]
        for w in wss:
            w[2 * phase: 2 * phase + 2] = tot
    for p, a, w in zip(parts, accs, wss):
        _native.apg_euler_dev_(a, u[p].cuda(), c[p].cuda(), G, 0.03, u.numel(), w, 0.05)
        torch.testing.assert_close(a.cpu().double(), want[p], rtol=1e-4, atol=1e-5)
