"""GPU: the RCCL ("nccl" backend) branches of f_lite.distributed, executed on the box's one MI355X.

Every multi-rank test elsewhere runs gloo, because RCCL refuses two ranks on one device, so the device-tensor
branches (RCCL broadcast / all-gather / all-reduce / send-recv of CUDA tensors) never ran on hardware
(VERDICT r04 weak 6). A process group of ONE rank over RCCL executes exactly those branches: communicator set-up,
every collective the sampling modes use, and the data-parallel APG loop whose two 2-float all-reduces per step go
through RCCL on device tensors. World size 1 makes every result checkable: each collective must return its input,
and the data-parallel sample must match the single-process batched loop on the same images (>= 50 dB).
"""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no ROCm device", allow_module_level=True)

import torch.multiprocessing as mp  # noqa: E402
from _mp import pack, unpack  # noqa: E402

from f_lite import APGConfig, DiT, FLitePipeline  # noqa: E402
from f_lite.model import PRESETS  # noqa: E402
from oracle import flite_ref as R  # noqa: E402

STEPS = 3
G = 6.0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(n):
    g = torch.Generator().manual_seed(5)
    return (torch.randn(n, 16, 16, 16, generator=g).bfloat16(), torch.randn(n, 24, 128, generator=g).bfloat16(),
            torch.randn(n, 24, 128, generator=g).bfloat16())


def _worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    try:
        import torch.distributed as dist

        from f_lite import distributed as D

        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        res = {"info": D.process_group_info()}
        g = torch.Generator(device=dev).manual_seed(3)
        ctx = torch.randn(1, 512, 4096, device=dev, generator=g).bfloat16()
        got = D.broadcast_context(ctx.clone())
        res["bcast"] = bool(torch.equal(got, ctx))
        res["bcast_ms"] = D.timed_broadcast_context(ctx.clone())
        t = torch.randn(4, device=dev, generator=g)
        res["allreduce"] = bool(torch.equal(D.all_reduce_sum_(t.clone()), t))
        out = torch.randn(2, 16, 16, 16, device=dev, generator=g)
        ex = D.exchange_branches(out)
        res["exchange"] = len(ex) == 1 and bool(torch.equal(ex[0], out))
        res["gather_images"] = bool(torch.equal(D.gather_images(out, 2), out))
        send = torch.randn(3 * 4096, device=dev, generator=g).bfloat16()
        recv = torch.empty_like(send)
        D.all_gather_rows(send, recv)
        res["all_gather_rows"] = bool(torch.equal(recv, send))
        recv2 = torch.empty_like(send)
        D.ring_shift_rows(send, recv2)  # to and from itself
        res["ring_shift"] = bool(torch.equal(recv2, send))
        res["max_over_ranks"] = D.max_over_ranks(1.25, device=dev)
        # the data-parallel sampling mode (APG's batch sums all-reduced on the device between its two phases)
        m = DiT.random(seed=0, device="cuda", **PRESETS["tiny"])
        lat, pos, neg = _inputs(2)
        res["dp"] = D.data_parallel_sample(m, lat.cuda(), pos.cuda(), neg.cuda(), STEPS, G,
                                           apg=APGConfig(enabled=True)).float().cpu()
        torch.cuda.synchronize()
        dist.destroy_process_group()
        q.put(pack(("ok", res)))
    except Exception as e:  # report instead of leaving the parent waiting
        import traceback

        q.put(("error", traceback.format_exc() + repr(e)))


@pytest.fixture(scope="module")
def results():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    kind, v = unpack(q.get(timeout=150))
    p.join(30)
    if p.is_alive():
        p.kill()
        p.join(10)
    if kind == "error":
        pytest.fail(v)
    return v


def test_rccl_process_group_reports_itself(results):
    info = results["info"]
    print("process group:", info, "broadcast ms", results["bcast_ms"])
    assert info["backend"] == "nccl" and info["world_size_seen"] == 1 and info["rank_seen"] == 0
    assert "rccl_version" in info
    assert results["bcast_ms"] > 0.0


@pytest.mark.parametrize("op", ["bcast", "allreduce", "exchange", "gather_images", "all_gather_rows", "ring_shift"])
def test_rccl_collective_returns_its_input(results, op):
    assert results[op], f"{op} over RCCL changed a world-size-1 tensor"


def test_rccl_max_over_ranks(results):
    assert results["max_over_ranks"] == 1.25


def test_rccl_data_parallel_apg_matches_batched_loop(results):
    lat, pos, neg = _inputs(2)
    m = DiT.random(seed=0, device="cuda", **PRESETS["tiny"])
    ref = FLitePipeline(m)(prompt_embeds=pos.cuda(), negative_prompt_embeds=neg.cuda(), latents=lat.cuda(),
                           height=128, width=128, num_inference_steps=STEPS, guidance_scale=G,
                           apg_config=APGConfig(enabled=True), output_type="latent",
                           use_graph=False).images.float().cpu()
    dp = results["dp"]
    assert dp.shape == ref.shape and torch.isfinite(dp).all()
    p = R.psnr(dp, ref)
    print(f"data-parallel APG over RCCL (1 rank) vs the batched loop: {p:.2f} dB")
    # the data-parallel mode launches the DiT per image and splits APG's sums around the all-reduce, so GEMM tiles
    # and the fp32 partial-sum order differ from the batched launch: the bar of test_gpu_apg_parallel's dp mode
    assert p >= 50.0
