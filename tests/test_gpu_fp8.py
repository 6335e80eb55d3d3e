"""GPU: the MXFP8 path (BASELINE.json configs[4]: fp8 weights + activations on the gfx950 block-scaled MFMA).

The reference has no fp8 path, so the oracle is a FAKE-QUANT restatement (oracle/flite_ref.py: mx_quant /
mx_quant_bytes / RefDiT(fp8=True)): the same MXFP8 rounding applied at the same points of the fp32 forward.
Bars:
  - quantisation kernels (flite_quant_fp8_rows, the fp8-output RMSNorm): bit-exact e4m3 bytes and E8M0 scales;
  - fp8 GEMM: vs an fp64 product of the dequantised operands, rel-L2 <= 1e-4 (measured 1.4e-5: the
    block-scaled MFMA's internal accumulation; 1000x below the e4m3 rounding of the operands);
  - fp8 DiT forward: >= 30 dB PSNR vs the fake-quant oracle (quantiser inputs differ by bf16 roundings, which
    can move an element by one e4m3 step); the distance to the un-quantised fp32 oracle is reported.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no ROCm device", allow_module_level=True)

from f_lite import DiT  # noqa: E402
from f_lite import _native as nat  # noqa: E402
from f_lite.model import PRESETS  # noqa: E402
from oracle import flite_ref as R  # noqa: E402

DEV = "cuda"


def dequant(q: torch.Tensor, sc: torch.Tensor) -> torch.Tensor:
    """uint8 e4m3 [rows, K] + scales [K/128, rows_pad, 4] -> fp32."""
    rows, K = q.shape
    v = q.cpu().view(torch.float8_e4m3fn).float()
    e = sc.cpu()[:, :rows, :].permute(1, 0, 2).reshape(rows, K // 32).to(torch.int32) - 127
    return (v.reshape(rows, K // 32, 32) * torch.ldexp(torch.ones(()), e)[..., None]).reshape(rows, K)


def psnr(a, ref):
    mse = (a.double() - ref.double()).pow(2).mean().item()
    return float("inf") if mse == 0 else 10 * math.log10(ref.double().abs().max().item() ** 2 / mse)


def test_e4m3_conversion_matches_torch():
    """v_cvt_pk_fp8_f32 on gfx950 is OCP e4m3fn with round-to-nearest-even (incl. subnormals and ties)."""
    g = torch.Generator().manual_seed(1)
    x = torch.cat([torch.randn(64, 1024, generator=g) * s for s in (1e-3, 0.1, 1.0, 30.0)])
    x[0, :8] = torch.tensor([0.0, -0.0, 1e-30, 448.0, -448.0, 2 ** -9, 3 * 2 ** -10, 1.0 + 2 ** -4])
    x = x.bfloat16()
    q, sc = nat.quant_fp8_rows(x.to(DEV))
    qr, scr = R.mx_quant_bytes(x.float())
    assert torch.equal(sc.cpu()[:, : x.shape[0]], scr[:, : x.shape[0]])
    assert torch.equal(q.cpu(), qr)


@pytest.mark.parametrize("rows,K", [(300, 512), (8224, 3072)])
def test_quant_rows_bit_exact(rows, K):
    g = torch.Generator().manual_seed(rows)
    x = (torch.randn(rows, K, generator=g) * torch.logspace(-3, 2, K)[None]).bfloat16()
    q, sc = nat.quant_fp8_rows(x.to(DEV))
    qr, scr = R.mx_quant_bytes(x.float())
    assert torch.equal(q.cpu(), qr)
    assert torch.equal(sc.cpu()[:, :rows], scr[:, :rows])
    torch.testing.assert_close(dequant(q, sc), R.mx_quant(x.float()), rtol=0, atol=0)


def test_rmsnorm_fp8_output():
    rows, D, T = 600, 3072, 300
    g = torch.Generator().manual_seed(2)
    x = torch.randn(rows, D, generator=g) * 3
    w = (1 + 0.1 * torch.randn(D, generator=g)).bfloat16()
    shift = torch.randn(2, D, generator=g) * 0.1
    scale = torch.randn(2, D, generator=g) * 0.1
    y8, sc = nat.rmsnorm_modulate_fp8(x.to(DEV), w.to(DEV), shift.to(DEV), scale.to(DEV), seg_rows=T)
    seg = torch.arange(rows) // T
    ref = R.liger_rmsnorm(x, w.float()) * (1 + scale[seg]) + shift[seg]
    got = dequant(y8, sc)
    want = R.mx_quant(ref)
    mism = (got != want).float().mean().item()
    print(f"fp8 RMSNorm: {mism * 100:.4f} % of elements differ from the fake-quant oracle (rsqrt/sum order)")
    assert mism < 1e-3
    assert psnr(got, want) > 60


@pytest.mark.parametrize("M,N,K,epi", [(300, 256, 512, "resid"), (8224, 3072, 3072, "resid"),
                                       (1000, 1536, 512, "store"), (8224, 9216, 3072, "store")])
def test_gemm_fp8(M, N, K, epi):
    g = torch.Generator().manual_seed(M + N)
    a = torch.randn(M, K, generator=g).bfloat16()
    w = (torch.randn(N, K, generator=g) * 0.02).bfloat16()
    bias = (torch.randn(N, generator=g) * 0.1).bfloat16()
    a8, asc = nat.quant_fp8_rows(a.to(DEV))
    w8, wsc = nat.quant_fp8_rows(w.to(DEV))
    ref = dequant(a8, asc).double() @ dequant(w8, wsc).double().t() + bias.double()
    if epi == "resid":
        gate = torch.ones(1, N, device=DEV)
        out = torch.zeros(M, N, device=DEV)
        nat.gemm_fp8(a8, asc, w8, wsc, bias.to(DEV), out=out, epilogue=nat.EPI8_RESID_F32, gate=gate,
                     gate_seg_stride=0, rows_per_seg=M)
        err = (out.cpu().double() - ref).norm() / ref.norm()
        assert err < 1e-4, err  # measured 1.4e-5 at K = 512 and 3072 (the block-scaled MFMA's accumulation)
    else:
        out = nat.gemm_fp8(a8, asc, w8, wsc, bias.to(DEV))
        err = (out.cpu().double() - ref).norm() / ref.norm()
        assert err < 4e-3, err  # bf16 output rounding


# Stream-K (flite_gemm_fp8_ws, stream_k.h): a partial last wave of 256x256 tiles cut into k-ranges over the CUs
# (the 10B down projection at 1024^2, and a 12-tile grid split ~4 ways per tile). Every epilogue runs in the
# finisher: fp32 residual, bf16 store, SwiGLU -> e4m3.
@pytest.mark.parametrize("M,N,K", [(8224, 3072, 12288), (1000, 768, 16384)])
def test_gemm_fp8_stream_k(M, N, K):
    g = torch.Generator().manual_seed(K + M)
    a8, asc = nat.quant_fp8_rows(torch.randn(M, K, generator=g).bfloat16().to(DEV))
    w8, wsc = nat.quant_fp8_rows((torch.randn(N, K, generator=g) * 0.02).bfloat16().to(DEV))
    bias = (torch.randn(N, generator=g) * 0.1).bfloat16().to(DEV)
    ws = nat.gemm_workspace(DEV)
    ref = dequant(a8, asc).double() @ dequant(w8, wsc).double().t() + bias.cpu().double()
    gate = torch.ones(1, N, device=DEV)
    outs = []
    for w_ in (None, ws, ws):
        x = torch.zeros(M, N, device=DEV)
        nat.gemm_fp8(a8, asc, w8, wsc, bias, out=x, epilogue=nat.EPI8_RESID_F32, gate=gate, gate_seg_stride=0,
                     rows_per_seg=M, workspace=w_)
        outs.append(x.cpu())
    dp, sk, sk2 = outs
    for o in (dp, sk):
        assert ((o.double() - ref).norm() / ref.norm()).item() < 1e-4
    assert not torch.equal(sk, dp)  # the split ran (another fp32 summation order)
    assert torch.equal(sk, sk2)  # deterministic
    n_cu = ws.numel() // (256 * 256 * 4 + 4)
    assert int(ws[n_cu * 256 * 256 * 4:].view(torch.int32).abs().sum().item()) == 0  # flags back to 0
    st = nat.gemm_fp8(a8, asc, w8, wsc, bias, workspace=ws)
    assert ((st.cpu().double() - ref).norm() / ref.norm()).item() < 4e-3
    F = N // 2
    gu8, gusc = nat.quant_fp8_gateup((torch.randn(F, K, generator=g) * 0.02).bfloat16().to(DEV),
                                     (torch.randn(F, K, generator=g) * 0.02).bfloat16().to(DEV))
    h_dp, s_dp = nat.gemm_fp8(a8, asc, gu8, gusc, epilogue=nat.EPI8_SWIGLU_FP8)
    h_sk, s_sk = nat.gemm_fp8(a8, asc, gu8, gusc, epilogue=nat.EPI8_SWIGLU_FP8, workspace=ws)
    assert psnr(dequant(h_sk, s_sk), dequant(h_dp, s_dp)) > 40


def test_gemm_fp8_swiglu():
    M, F, K = 1000, 1024, 512
    g = torch.Generator().manual_seed(9)
    a = torch.randn(M, K, generator=g).bfloat16()
    wg = (torch.randn(F, K, generator=g) * 0.05).bfloat16()
    wu = (torch.randn(F, K, generator=g) * 0.05).bfloat16()
    a8, asc = nat.quant_fp8_rows(a.to(DEV))
    gu8, gusc = nat.quant_fp8_gateup(wg.to(DEV), wu.to(DEV))
    h8, hsc = nat.gemm_fp8(a8, asc, gu8, gusc, epilogue=nat.EPI8_SWIGLU_FP8)
    ad = dequant(a8, asc).double()
    gd = ad @ R.mx_quant(wg.float()).double().t()
    ud = ad @ R.mx_quant(wu.float()).double().t()
    h = (torch.nn.functional.silu(gd) * ud).float()
    got = dequant(h8, hsc)
    want = R.mx_quant(h)
    p = psnr(got, want)
    mism = (got != want).float().mean().item()
    print(f"fp8 SwiGLU GEMM: {p:.1f} dB vs fake-quant fp64; {mism * 100:.3f} % elements differ")
    assert p > 45 and mism < 0.02
    # the bf16-output epilogue (an MXFP8 gate/up feeding a bf16 down): the same fp32 h rounded once, 16-B stores
    hb = nat.gemm_fp8(a8, asc, gu8, gusc, epilogue=nat.EPI8_SWIGLU_BF16)
    assert hb.dtype == torch.bfloat16 and hb.shape == (M, F)
    assert ((hb.cpu().double() - h.double()).norm() / h.double().norm()).item() < 4e-3
    assert (hb.cpu() != h.bfloat16()).float().mean().item() < 0.05
    # a strided output (row stride F + 8: 16-B aligned rows) and one that is not 16-B aligned (8-B stores)
    for pad in (8, 4):
        buf = torch.zeros(M, F + pad, device=DEV, dtype=torch.bfloat16)
        nat.gemm_fp8(a8, asc, gu8, gusc, epilogue=nat.EPI8_SWIGLU_BF16, out=buf[:, :F])
        assert torch.equal(buf[:, :F], hb) and not buf[:, F:].any()


@pytest.mark.parametrize("preset", ["tiny", "tiny_v2"])
def test_dit_fp8_forward_vs_fake_quant_oracle(golden, preset):
    m = DiT.random(seed=0, device=DEV, **PRESETS[preset])
    x = golden["in.x"].bfloat16()
    ctx = golden["in.ctx"].bfloat16()
    t = golden["in.t"]
    bf = m(x.to(DEV), ctx.to(DEV), None, t.to(DEV), output_dtype=torch.float32).cpu()
    m.enable_fp8(True)
    out = m(x.to(DEV), ctx.to(DEV), None, t.to(DEV), output_dtype=torch.float32).cpu()
    m.enable_fp8(False)
    again = m(x.to(DEV), ctx.to(DEV), None, t.to(DEV), output_dtype=torch.float32).cpu()
    assert torch.equal(bf, again)  # back on the bf16 path
    with torch.no_grad():
        fq = R.RefDiT.random(R.PRESETS[preset], dtype=torch.float32, fp8=True)(x.float(), ctx.float(), None, t)
        f32 = R.RefDiT.random(R.PRESETS[preset], dtype=torch.float32)(x.float(), ctx.float(), None, t)
    p_fq, p_32, p_bf = psnr(out, fq), psnr(out, f32), psnr(bf, f32)
    print(f"{preset} fp8 forward: {p_fq:.2f} dB vs fake-quant oracle, {p_32:.2f} dB vs fp32 oracle "
          f"(bf16 path: {p_bf:.2f} dB; fake-quant oracle vs fp32 oracle {psnr(fq, f32):.2f} dB)")
    assert p_fq >= 30.0


def test_dit_fp8_sampling_loop_graph_equals_eager(golden):
    from f_lite import FLitePipeline

    m = DiT.random(seed=0, device=DEV, **PRESETS["tiny"]).enable_fp8(True)
    pipe = FLitePipeline(m)
    lat = golden["pipe.in.latents"].bfloat16().to(DEV)
    pos = golden["pipe.in.pos"].bfloat16().to(DEV)
    run = [pipe(prompt_embeds=pos, latents=lat, height=128, width=128, num_inference_steps=4, guidance_scale=6.0,
                output_type="latent", use_graph=gr).images.float().cpu() for gr in (False, True, True)]
    assert torch.isfinite(run[0]).all()
    assert torch.equal(run[0], run[1]) and torch.equal(run[1], run[2])


@pytest.mark.parametrize("depth", [1, 2])
def test_10b_fp8_full_width_vs_fake_quant_oracle(depth):
    """configs[4] at full width: the 10B layout at the reference's default 1344x896 (T = 4720, 112-row attention
    tails), a 512-token context, depth 1-2, fp8 mode vs the fake-quant oracle (RefDiT(fp8=True): the same MXFP8
    rounding at the same points of the fp32 forward). Covers the shapes the 512-wide presets never reach: the
    gate/up interleave at F = 12288, the SwiGLU -> e4m3 epilogue of full-size tiles, the attention's MXFP8
    output at the T = 4720 tails, the 224-row tiles. Also reports MXFP8's intrinsic cost (fake-quant oracle vs
    the fp32 oracle) and the bf16 path's distance at the same shape."""
    import dataclasses

    cfg = dict(PRESETS["10b"], depth=depth)
    m = DiT.random(seed=0, device=DEV, **cfg)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 16, 112, 168, generator=g).bfloat16()
    ctx = torch.randn(2, 512, 4096, generator=g).bfloat16()
    t = torch.tensor([0.75, 0.75]).bfloat16()
    bf = m(x.to(DEV), ctx.to(DEV), None, t.to(DEV), output_dtype=torch.float32).cpu()
    m.enable_fp8(True)
    f8 = m(x.to(DEV), ctx.to(DEV), None, t.to(DEV), output_dtype=torch.float32).cpu()
    rc = dataclasses.replace(R.PRESETS["10b"], depth=depth)
    with torch.no_grad():
        fq = R.RefDiT.random(rc, dtype=torch.float32, fp8=True)(x.float(), ctx.float(), None, t)
        f32 = R.RefDiT.random(rc, dtype=torch.float32)(x.float(), ctx.float(), None, t)
    p_fq, p_32, p_bf, p_int = psnr(f8, fq), psnr(f8, f32), psnr(bf, f32), psnr(fq, f32)
    print(f"10B 1344x896 depth {depth} fp8: {p_fq:.2f} dB vs fake-quant oracle, {p_32:.2f} dB vs fp32 oracle; "
          f"MXFP8 intrinsic (fake-quant vs fp32 oracle) {p_int:.2f} dB; bf16 path vs fp32 oracle {p_bf:.2f} dB; "
          f"fp8 vs bf16 path {psnr(f8, bf):.2f} dB")
    assert p_fq >= 30.0


def test_10b_fp8_full_size_forward():
    """The configs[4] model at the reference's default 1344x896 (T = 4720), full depth: fp8 vs the bf16 path.
    The bar sits 3 dB under the measured value (24.98 dB, round 2): the distance is MXFP8's own cost compounded
    over 40 blocks (tools/fp8_depth_decay.py measures it against the fake-quant and fp32 oracles by depth)."""
    m = DiT.random(seed=0, device=DEV, **PRESETS["10b"])
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 16, 112, 168, generator=g).bfloat16().to(DEV)
    ctx = torch.randn(2, 512, 4096, generator=g).bfloat16().to(DEV)
    t = torch.tensor([0.75, 0.75]).bfloat16().to(DEV)
    bf = m(x, ctx, None, t, output_dtype=torch.float32).cpu()
    m.enable_fp8(True)
    f8 = m(x, ctx, None, t, output_dtype=torch.float32).cpu()
    f8b = m(x, ctx, None, t, output_dtype=torch.float32).cpu()
    assert torch.isfinite(f8).all() and torch.equal(f8, f8b)
    p = psnr(f8, bf)
    print(f"10B 1344x896 full-depth forward: fp8 vs bf16 path {p:.2f} dB")
    assert p > 22.0


@pytest.mark.parametrize("preset,hw", [("tiny", (16, 16)), ("10b_d2", (112, 168))])
def test_fp8_attention_mx_output_matches_quant_rows(monkeypatch, preset, hw):
    """The fp8 path's attention writes the proj GEMM's MXFP8 operand itself (attention.hip, AttnParams.o8):
    bit-identical to the bf16 attention output + quant_rows_fp8 (FLITE_FP8_ATTN_UNFUSED=1). The 10B-layout case
    (depth 2, 1344x896: T = 4720, 112-row tails) also covers the tail-split rows, quantised after the reduce."""
    cfg = dict(PRESETS["10b"], depth=2) if preset == "10b_d2" else PRESETS[preset]
    m = DiT.random(seed=0, device=DEV, **cfg)
    g = torch.Generator().manual_seed(9)
    x = torch.randn(2, 16, *hw, generator=g).bfloat16().to(DEV)
    ctx = torch.randn(2, 64, cfg["cross_attn_input_size"], generator=g).bfloat16().to(DEV)
    t = torch.tensor([0.6, 0.6]).bfloat16().to(DEV)
    monkeypatch.setenv("FLITE_FP8_ATTN_UNFUSED", "1")
    m.enable_fp8(True)
    unfused = m(x, ctx, None, t, output_dtype=torch.float32).cpu()
    m.enable_fp8(False)
    monkeypatch.delenv("FLITE_FP8_ATTN_UNFUSED")
    m.enable_fp8(True)
    fused = m(x, ctx, None, t, output_dtype=torch.float32).cpu()
    assert torch.isfinite(fused).all()
    assert torch.equal(fused, unfused)


def test_fp8_bf16_block_policy():
    """flite_dit_set_fp8_bf16_blocks: with every block kept bf16 the fp8-mode loop IS the bf16 loop (bit for bit:
    same kernels, the blocks are self-contained between fp32 residual reads and writes); keeping the first and last
    block bf16 lands between all-fp8 and bf16."""
    from f_lite import FLitePipeline

    cfg = dict(PRESETS["10b"], depth=4)
    m = DiT.random(seed=0, device=DEV, **cfg)
    g = torch.Generator().manual_seed(8)
    lat = torch.randn(1, 16, 32, 32, generator=g).bfloat16().to(DEV)
    pos = torch.randn(1, 64, 4096, generator=g).bfloat16().to(DEV)

    def run():
        return FLitePipeline(m)(prompt_embeds=pos, latents=lat, height=256, width=256, num_inference_steps=4,
                                guidance_scale=6.0, output_type="latent").images.float().cpu()

    bf = run()
    m.enable_fp8(True, bf16_blocks=range(4))
    assert torch.equal(run(), bf)
    m.enable_fp8(True, bf16_blocks=(0, 3))
    ends = run()
    m.enable_fp8(True)
    all8 = run()
    m.enable_fp8(False)
    p_all, p_ends = psnr(all8, bf), psnr(ends, bf)
    print(f"fp8 policy, 10B layout depth 4, 256^2, 4 CFG-6 steps: all fp8 {p_all:.2f} dB, first+last bf16 "
          f"{p_ends:.2f} dB vs bf16")
    assert p_ends > p_all


def test_fp8_gemm_class_policy():
    """flite_dit_set_fp8_gemm_classes: with no class on MXFP8 the fp8-mode loop IS the bf16 loop
    (bit for bit); every mixed set (the SwiGLU output produced as bf16 by the fp8 gate/up epilogue, or quantised for
    an fp8 down; the attention writing bf16 for a bf16 proj; bf16 norms for bf16 consumers) is finite, graph ==
    eager, and no further from bf16 than all-fp8 (+0.5 dB slack); the MLP-only and gate/up-only policies are
    closer to bf16 than all-fp8 is. The zero negative prompt exercises the uniform-context collapse's bf16 / fp8
    cross-proj choice."""
    from f_lite import FLitePipeline

    cfg = dict(PRESETS["10b"], depth=3)
    m = DiT.random(seed=0, device=DEV, **cfg)
    g = torch.Generator().manual_seed(9)
    lat = torch.randn(1, 16, 32, 32, generator=g).bfloat16().to(DEV)
    pos = torch.randn(1, 64, 4096, generator=g).bfloat16().to(DEV)

    def run(graph=True):
        return FLitePipeline(m)(prompt_embeds=pos, latents=lat, height=256, width=256, num_inference_steps=4,
                                guidance_scale=6.0, output_type="latent", use_graph=graph).images.float().cpu()

    bf = run()
    m.enable_fp8(True, gemm_classes=0)
    assert torch.equal(run(), bf)
    m.enable_fp8(True)
    p_all = psnr(run(), bf)
    res = {}
    for classes in (("gate_up",), ("down",), ("gate_up", "down"), ("qkv", "proj"), ("cross_q", "cross_proj"),
                    ("qkv", "proj", "cross_q", "cross_proj"), ("proj", "down"), ("qkv", "cross_q", "gate_up")):
        m.enable_fp8(True, gemm_classes=classes)
        out = run()
        assert torch.isfinite(out).all(), classes
        assert torch.equal(out, run(graph=False)), classes
        res[classes] = psnr(out, bf)
        print(f"fp8 classes {'+'.join(classes)}: {res[classes]:.2f} dB vs bf16 (all fp8 {p_all:.2f} dB)")
        assert res[classes] >= p_all - 0.5, classes
    m.enable_fp8(False)
    assert res[("gate_up",)] > p_all and res[("gate_up", "down")] > p_all


@pytest.fixture(scope="module")
def gold3():
    import json
    from pathlib import Path

    from safetensors.torch import load_file

    d = Path(__file__).resolve().parent / "golden"
    if not (d / "golden_full3.safetensors").exists():
        pytest.skip("golden_full3.safetensors not generated")
    return load_file(str(d / "golden_full3.safetensors")), json.loads((d / "golden_full3_meta.json").read_text())


# REGRESSION PINS, not parity bars (the reference has no fp8 path): measured on the MI355X (profiles/r04a/pytest.log:
# 16.80 / 19.31 dB at CFG 6, 35.12 / 35.92 dB at CFG 1, 7B / 10B); the pins sit 3 dB under them. bf16 on the same fixtures: 37.72 / 35.47 dB at CFG 6 and 56.28 / 56.56 dB at CFG 1
# (test_gpu_full_depth.py::test_256_free_running_30_steps); the reference's own bf16 run: 30.66 / 30.60 and
# 47.51 / 48.21 dB. MXFP8's e4m3 elements carry 3 mantissa bits (bf16: 8), so its forward error is ~2^5 larger
# and CFG 6 amplifies it over the trajectory (DESIGN §4, fp8 policies)
FP8_P3_BARS = {("7b", 6.0): 13.8, ("7b", 1.0): 32.1, ("10b", 6.0): 16.3, ("10b", 1.0): 32.9}


@pytest.mark.parametrize("name", ["7b", "10b"])
@pytest.mark.parametrize("g", [6.0, 1.0])
def test_fp8_256_free_running_30_steps(gold3, name, g):
    """The MXFP8 configuration on the P3 scale of the bf16 path: the 30-step native fp8 loop's
    final latents vs the reference's fp32 trajectory at 256^2 (golden_full3, the stub-loaded reference), beside
    the reference's own bf16 run."""
    from f_lite import FLitePipeline

    gd, meta = gold3
    key = f"{name}.256.s30.g{g:g}"
    m = DiT.random(seed=0, device=DEV, **PRESETS[name])
    m.enable_fp8(True)
    ctx = torch.empty(*meta["inputs"]["ctx"][1], device=DEV, dtype=torch.bfloat16)
    nat.init_param_(ctx, meta["inputs"]["ctx"][0], seed=0, std=1.0)
    lat = torch.empty(*meta["inputs"]["latents_256"][1], device=DEV, dtype=torch.bfloat16)
    nat.init_param_(lat, meta["inputs"]["latents_256"][0], seed=0, std=1.0)
    out = FLitePipeline(m)(prompt_embeds=ctx, latents=lat, height=256, width=256, num_inference_steps=30,
                           guidance_scale=g, output_type="latent").images.float().cpu()
    p = psnr(out / 0.3611 + 0.1159, gd[f"{key}.f32.final"])
    print(f"fp8 {name} 256^2 30-step CFG-{g:g} final latents: {p:.2f} dB vs reference fp32 (reference's own bf16 "
          f"run: {meta[f'{key}.bf16_vs_f32_psnr']:.2f} dB)")
    assert p >= FP8_P3_BARS[(name, g)]


@pytest.mark.parametrize("name", ["7b", "10b"])
def test_fp8_first_blocks_bf16_policy_reaches_40db_at_cfg1(gold3, name):
    """The quality-leaning MXFP8 policy (DESIGN §5 "fp8 against the reference"): blocks 0-7 keep their bf16 GEMMs, every
    GEMM class of blocks 8-39 runs MXFP8 (1.40x the bf16 image at 1344x896, profiles/r05m/fp8_block_speed.log). The
    MXFP8 error enters through the first blocks (bf16 in the LAST four blocks gains 0.1 dB, in the first four 4.9 dB),
    so this policy meets north_star's 40 dB bar against the reference's fp32 30-step trajectory where CFG noise is
    absent (CFG 1, 256^2, golden_full3): measured 41.59 / 42.52 dB (7B / 10B) against 35.02 / 35.92 dB all-fp8.
    At CFG 6 no fp8 policy reaches the reference's own bf16 floor (30.6 dB); that case stays pinned above."""
    from f_lite import FLitePipeline

    gd, meta = gold3
    key = f"{name}.256.s30.g1"
    m = DiT.random(seed=0, device=DEV, **PRESETS[name])
    m.enable_fp8(True, bf16_blocks=list(range(8)))
    ctx = torch.empty(*meta["inputs"]["ctx"][1], device=DEV, dtype=torch.bfloat16)
    nat.init_param_(ctx, meta["inputs"]["ctx"][0], seed=0, std=1.0)
    lat = torch.empty(*meta["inputs"]["latents_256"][1], device=DEV, dtype=torch.bfloat16)
    nat.init_param_(lat, meta["inputs"]["latents_256"][0], seed=0, std=1.0)
    out = FLitePipeline(m)(prompt_embeds=ctx, latents=lat, height=256, width=256, num_inference_steps=30,
                           guidance_scale=1.0, output_type="latent").images.float().cpu()
    p = psnr(out / 0.3611 + 0.1159, gd[f"{key}.f32.final"])
    print(f"fp8 (bf16 blocks 0-7) {name} 256^2 30-step CFG-1 final latents: {p:.2f} dB vs reference fp32 "
          f"(reference's own bf16 run: {meta[f'{key}.bf16_vs_f32_psnr']:.2f} dB)")
    assert p >= 40.0


def test_fp8_10b_1344x896_30_steps_full_loop():
    """BASELINE configs[4] at full size: the 10B MXFP8 loop at 1344x896, 30 CFG-6 steps, tiled VAE
    decode to uint8, as bench.py --fp8 runs it: hipGraph == eager bit for bit, finite, and the uint8 image within a
    REGRESSION PIN of the bf16 path's image (measured 19.46 dB on the MI355X, profiles/r05j/fp8_policy.log; pin 3 dB
    under it). Not a parity bar: the reference has no fp8 path, and CFG 6 amplifies MXFP8's per-GEMM rounding over the
    30 steps (every GEMM-class policy stays <= 25 dB, DESIGN §5 "fp8 precision policies")."""
    from f_lite import FLitePipeline
    from f_lite.vae import AutoencoderKL

    m = DiT.random(seed=0, device=DEV, **PRESETS["10b"])
    pipe = FLitePipeline(m, vae=AutoencoderKL.random(seed=0, device=DEV))
    pipe.enable_vae_tiling()
    ctx = torch.empty(1, 512, 4096, device=DEV, dtype=torch.bfloat16)
    nat.init_param_(ctx, "synthetic.t5_context", seed=1, std=1.0)
    lat = torch.empty(1, 16, 112, 168, device=DEV, dtype=torch.bfloat16)
    nat.init_param_(lat, "synthetic.latents.0", seed=2, std=1.0)
    kw = dict(prompt_embeds=ctx, latents=lat, height=896, width=1344, num_inference_steps=30, guidance_scale=6.0,
              output_type="uint8")
    bf = pipe(**kw).images.cpu()
    m.enable_fp8(True)
    graph = pipe(**kw, use_graph=True).images.cpu()
    eager = pipe(**kw, use_graph=False).images.cpu()
    m.enable_fp8(False)
    assert graph.shape == (1, 896, 1344, 3)
    assert torch.equal(graph, eager)
    p = 10 * math.log10(255.0 ** 2 / max((graph.double() - bf.double()).pow(2).mean().item(), 1e-12))
    print(f"MXFP8 10B 1344x896 30-step CFG-6 image vs the bf16 image: {p:.2f} dB (regression pin 16.5 dB)")
    assert graph.float().std() > 1.0 and p >= 16.5
