"""GPU: replica data parallelism -- image i on rank i mod N, one context broadcast, no per-step
collective. Two ranks share the box's one GPU (gloo carries the broadcast; RCCL does on a multi-GPU node).

Bar (§4 item 5 of SURVEY): every rank's images are BIT-EQUAL to a single-process run of the same image
indices -- the kernels are deterministic and a rank computes exactly what one process would.
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

WORLD = 2
N_IMAGES = 4
H = W = 128
STEPS = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make_pipe():
    from f_lite.vae import AutoencoderKL

    m = DiT.random(seed=0, device="cuda", **PRESETS["tiny"])
    return FLitePipeline(m, AutoencoderKL.random(seed=0, device="cuda"))


def _image(pipe, ctx, i):
    lat = torch.empty(1, 16, H // 8, W // 8, device="cuda", dtype=torch.bfloat16)
    _native.init_param_(lat, f"synthetic.latents.{i}", seed=2, std=1.0)
    return pipe(prompt_embeds=ctx, latents=lat, height=H, width=W, num_inference_steps=STEPS, guidance_scale=6.0,
                output_type="uint8").images.cpu()


def _ctx(rank):
    ctx = torch.zeros(1, 24, 128, device="cuda", dtype=torch.bfloat16)
    if rank == 0:
        _native.init_param_(ctx, "synthetic.t5_context", seed=1, std=1.0)
    return ctx


def _worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD))
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        from f_lite.distributed import broadcast_context, image_indices

        pipe = _make_pipe()
        ctx = broadcast_context(_ctx(rank), src=0)
        out = {i: _image(pipe, ctx, i) for i in image_indices(N_IMAGES, rank, WORLD)}
        torch.cuda.synchronize()
        q.put(pack((rank, out)))
        dist.destroy_process_group()
    except Exception as e:  # report instead of leaving the parent waiting
        q.put((rank, repr(e)))


@pytest.fixture(scope="module")
def ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = {}
    while len(res) < WORLD and not any(isinstance(v, str) for v in res.values()):
        k, v = unpack(q.get(timeout=100))
        res[k] = v
    for p in procs:
        p.join(30)
        if p.is_alive():
            p.kill()
            p.join(10)
    for r in sorted(res):
        assert isinstance(res[r], dict), f"rank {r}: {res[r]}"
    return res


def test_each_image_once_and_bit_equal_to_single_process(ranks):
    merged = {}
    for r, imgs in ranks.items():
        assert sorted(imgs) == list(range(r, N_IMAGES, WORLD))  # image i -> rank i mod N
        merged.update(imgs)
    assert sorted(merged) == list(range(N_IMAGES))
    pipe = _make_pipe()
    ctx = _ctx(0)
    for i in range(N_IMAGES):
        ref = _image(pipe, ctx, i)
        assert ref.shape == (1, H, W, 3) and ref.dtype == torch.uint8
        assert torch.equal(merged[i], ref), f"image {i}: rank output differs from the single-process image"
    # the images really differ per index (the latents are per image)
    assert not torch.equal(merged[0], merged[1])
