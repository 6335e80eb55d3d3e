"""GPU parity at FULL size and depth against the reference itself (SURVEY §8c fixture set iii).

tests/golden/golden_full.safetensors was produced by tests/golden/make_golden_full.py from the stub-loaded
reference (f_lite/model.py, model_v2.py, pipeline.py; all 40 blocks, fp32, bf16 timesteps as a bf16 pipeline
feeds them). Weights and inputs are regenerated here bit-identically by flite_init_param (the hash generator
of oracle/weights.py), so only the reference outputs are stored.

Bars (SURVEY §8d parity protocol):
  P2  teacher-forced: for each step of the 7B 256^2 4-step CFG-6 trajectory, the native forward on the
      reference's own fp32 input reaches >= 40 dB PSNR per CFG branch (raw DiT output, peak = max|ref|);
      the same for one CFG-batched 7B and 10B forward at 1024^2 (T = 4112 tokens per sample).
  P3  free-running: the native 4-step pipeline's final latents vs the reference's fp32 ones, reported beside
      the reference's OWN bf16-vs-fp32 figure on the same run (golden_full_meta.json), which they must beat.
Plus a full 10B 1024^2 30-step CFG-6 run: finite, hipGraph replay bit-equal to eager, bit-deterministic.
"""
import json
import math
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no ROCm device", allow_module_level=True)

from f_lite import DiT, FLitePipeline  # noqa: E402
from f_lite import _native  # noqa: E402
from f_lite.model import PRESETS  # noqa: E402

GOLD = Path(__file__).resolve().parent / "golden"
DEV = "cuda"
SCALING, SHIFT = 0.3611, 0.1159  # the stub VAE config of the fixture run (pipeline.py:301-304)


def psnr(a, ref):
    a = a.double().cpu()
    ref = ref.double().cpu()
    mse = (a - ref).pow(2).mean().item()
    return float("inf") if mse == 0 else 10 * math.log10(ref.abs().max().item() ** 2 / mse)


@pytest.fixture(scope="module")
def gold():
    from safetensors.torch import load_file

    f = GOLD / "golden_full.safetensors"
    if not f.exists():
        pytest.skip("golden_full.safetensors not generated")
    return load_file(str(f)), json.loads((GOLD / "golden_full_meta.json").read_text())


def hashed(meta, key):
    name, shape = meta["inputs"][key]
    t = torch.empty(*shape, device=DEV, dtype=torch.bfloat16)
    return _native.init_param_(t, name, seed=0, std=1.0)


@pytest.fixture(scope="module")
def m7b():
    return DiT.random(seed=0, device=DEV, **PRESETS["7b"])


@pytest.fixture(scope="module")
def m10b():
    return DiT.random(seed=0, device=DEV, **PRESETS["10b"])


def _cfg_forward(model, x, pos, t):
    ctx2 = torch.cat([torch.zeros_like(pos), pos])  # uncond first (pipeline.py:266)
    return model(x.to(DEV), ctx2, t.to(DEV), output_dtype=torch.float32).cpu()


def _check_branches(out, ref, what, bar=40.0):
    pu, pc = psnr(out[0], ref[0]), psnr(out[1], ref[1])
    print(f"{what}: PSNR uncond {pu:.2f} dB, cond {pc:.2f} dB")
    assert pu >= bar and pc >= bar, (pu, pc)
    return pu, pc


@pytest.mark.parametrize("step", range(4))
def test_7b_256_teacher_forced_step(gold, m7b, step):
    g, meta = gold
    pos = hashed(meta, "ctx")
    x = g[f"7b.256.step{step}.x"]
    t = g[f"7b.256.step{step}.t"].to(torch.bfloat16)
    out = _cfg_forward(m7b, x, pos, t)
    ref = g[f"7b.256.step{step}.out"]
    _check_branches(out, ref, f"7B 256^2 step {step} (t={float(t[0]):.4f}) teacher-forced")
    comb = out[0] + 6.0 * (out[1] - out[0])
    comb_ref = ref[0] + 6.0 * (ref[1] - ref[0])
    print(f"  CFG-6 combined output: {psnr(comb, comb_ref):.2f} dB")


def test_7b_256_free_running_4_steps(gold, m7b):
    g, meta = gold
    pos = hashed(meta, "ctx")
    lat = hashed(meta, "latents_256")
    pipe = FLitePipeline(m7b)
    out = pipe(prompt_embeds=pos, latents=lat, height=256, width=256, num_inference_steps=4, guidance_scale=6.0,
               output_type="latent").images.float()
    got = out / SCALING + SHIFT
    ref = g["7b.256.f32.final"]
    p = psnr(got, ref)
    floor = meta["7b.256.bf16_vs_f32_psnr"]
    print(f"7B 256^2 4-step CFG-6 final latents: {p:.2f} dB vs reference fp32 "
          f"(reference's own bf16 run: {floor:.2f} dB)")
    assert p >= floor
    # 3 dB above the reference's own bf16 run (36.3 dB with the fp32 residual stream, 34.5 with the bf16 default)
    assert p >= floor + 3.0


def test_7b_1024_forward(gold, m7b):
    g, meta = gold
    lat = hashed(meta, "latents_1024").float().cpu()
    x = torch.cat([lat, lat])
    t = torch.tensor([meta["t_1024"]] * 2).to(torch.bfloat16)
    out = _cfg_forward(m7b, x, hashed(meta, "ctx"), t)
    _check_branches(out, g["7b.1024.out"], "7B 1024^2 full-depth forward (T=4112)")


def test_10b_1024_forward(gold, m10b):
    g, meta = gold
    lat = hashed(meta, "latents_1024").float().cpu()
    x = torch.cat([lat, lat])
    t = torch.tensor([meta["t_1024"]] * 2).to(torch.bfloat16)
    out = _cfg_forward(m10b, x, hashed(meta, "ctx"), t)
    _check_branches(out, g["10b.1024.out"], "10B 1024^2 full-depth forward (T=4112)")


def test_10b_1024_30_steps_graph_eager_deterministic(m10b):
    """The metric workload's DiT loop at full size: finite; hipGraph replay == eager; bit-reproducible."""
    ctx = torch.empty(1, 512, 4096, device=DEV, dtype=torch.bfloat16)
    _native.init_param_(ctx, "synthetic.t5_context", seed=1, std=1.0)
    lat = torch.empty(1, 16, 128, 128, device=DEV, dtype=torch.bfloat16)
    _native.init_param_(lat, "synthetic.latents.0", seed=2, std=1.0)
    pipe = FLitePipeline(m10b)

    def run(graph):
        return pipe(prompt_embeds=ctx, latents=lat, height=1024, width=1024, num_inference_steps=30,
                    guidance_scale=6.0, output_type="latent", use_graph=graph).images.float().cpu()

    a = run(True)
    b = run(True)  # replay of the cached graph
    c = run(False)
    assert torch.isfinite(a).all()
    assert a.abs().max() > 0.1 and a.std() > 0.1
    assert torch.equal(a, b) and torch.equal(a, c)


# ---- SURVEY §8c fixture set (iv) / §8d "re-measure P2 at T = 4112" (tests/golden/make_golden_full2.py) ----
@pytest.fixture(scope="module")
def gold2():
    from safetensors.torch import load_file

    f = GOLD / "golden_full2.safetensors"
    if not f.exists():
        pytest.skip("golden_full2.safetensors not generated")
    return load_file(str(f)), json.loads((GOLD / "golden_full2_meta.json").read_text())


def _teacher_input(meta, t):
    """x_t = bf16(t * noise + (1 - t) * x0) in fp32 arithmetic, as make_golden_full2.teacher_input."""
    noise = hashed(meta, "latents_1024").float().cpu()
    x0 = hashed(meta, "x0_1024").float().cpu()
    return (noise * t + x0 * (1.0 - t)).to(torch.bfloat16).float()


@pytest.mark.parametrize("name", ["7b", "10b"])
@pytest.mark.parametrize("t", [1.0, 0.5, 0.1])
def test_1024_teacher_forced_step(gold2, m7b, m10b, name, t):
    """P2 at T = 4112: the CFG-batched raw output on the reference's input at t, >= 40 dB per branch; the
    CFG-6-combined output is reported (the reference's own bf16 run sits at 38-40 dB there at 256^2)."""
    g, meta = gold2
    key = f"{name}.1024.tf{t}.out"
    if key not in g:
        pytest.skip(f"{key} not in the fixture file")
    model = m7b if name == "7b" else m10b
    x = _teacher_input(meta, t)
    out = _cfg_forward(model, torch.cat([x, x]), hashed(meta, "ctx"), torch.tensor([t, t]).to(torch.bfloat16))
    ref = g[key]
    _check_branches(out, ref, f"{name} 1024^2 teacher-forced t={t}")
    comb = out[0] + 6.0 * (out[1] - out[0])
    comb_ref = ref[0] + 6.0 * (ref[1] - ref[0])
    print(f"  CFG-6 combined output: {psnr(comb, comb_ref):.2f} dB")


@pytest.mark.parametrize("name", ["7b", "10b"])
def test_1024_free_running_4_steps(gold2, m7b, m10b, name):
    """P3 at 1024^2: the native 4-step CFG-6 pipeline's final latents vs the reference's fp32 ones, beside (and
    above) the reference's own bf16 run on the same trajectory."""
    g, meta = gold2
    key = f"{name}.1024.f32.final"
    if key not in g:
        pytest.skip(f"{key} not in the fixture file")
    model = m7b if name == "7b" else m10b
    pos = hashed(meta, "ctx")
    lat = hashed(meta, "latents_1024")
    out = FLitePipeline(model)(prompt_embeds=pos, latents=lat, height=1024, width=1024, num_inference_steps=4,
                               guidance_scale=6.0, output_type="latent").images.float()
    got = out / SCALING + SHIFT
    p = psnr(got, g[key])
    floor = meta[f"{name}.1024.bf16_vs_f32_psnr"]
    print(f"{name} 1024^2 4-step CFG-6 final latents: {p:.2f} dB vs reference fp32 (reference's own bf16 run: "
          f"{floor:.2f} dB)")
    assert p >= floor


def test_10b_1344x896_30_steps_tiled_vae(m10b):
    """BASELINE configs[2] at full size: 10B layout, the reference's generate.py default 1344x896 (T = 4720),
    30 CFG-6 steps, then the diffusers tiled decode that generate.py:77-78 turns on (112 x 168 latents exceed the
    128-latent tile) to uint8. Finite; hipGraph replay == eager bit for bit; the whole image bit-reproducible
    (the tiled decode's parity against the oracle at this grid: test_gpu_vae.py::test_vae_decode_tiled_default_grid)."""
    from f_lite.vae import AutoencoderKL

    ctx = torch.empty(1, 512, 4096, device=DEV, dtype=torch.bfloat16)
    _native.init_param_(ctx, "synthetic.t5_context", seed=1, std=1.0)
    lat = torch.empty(1, 16, 112, 168, device=DEV, dtype=torch.bfloat16)
    _native.init_param_(lat, "synthetic.latents.0", seed=2, std=1.0)
    pipe = FLitePipeline(m10b, vae=AutoencoderKL.random(seed=0))
    pipe.enable_vae_tiling()
    kw = dict(prompt_embeds=ctx, latents=lat, height=896, width=1344, num_inference_steps=30, guidance_scale=6.0)
    a = pipe(**kw, output_type="latent", use_graph=True).images.float().cpu()
    b = pipe(**kw, output_type="latent", use_graph=False).images.float().cpu()
    assert torch.isfinite(a).all() and a.std() > 0.1
    assert torch.equal(a, b)
    img = pipe(**kw, output_type="uint8").images
    assert img.shape == (1, 896, 1344, 3) and img.dtype == torch.uint8
    img2 = pipe(**kw, output_type="uint8").images
    assert torch.equal(img, img2)
    assert img.float().std() > 1.0  # a non-degenerate picture


# ---- P3 at the metric's 30 steps, CFG 6 and CFG 1 (tests/golden/make_golden_full3.py) ----
@pytest.fixture(scope="module")
def gold3():
    from safetensors.torch import load_file

    f = GOLD / "golden_full3.safetensors"
    if not f.exists():
        pytest.skip("golden_full3.safetensors not generated")
    return load_file(str(f)), json.loads((GOLD / "golden_full3_meta.json").read_text())


@pytest.mark.parametrize("name", ["7b", "10b"])
@pytest.mark.parametrize("g", [6.0, 1.0])
def test_256_free_running_30_steps(gold3, m7b, m10b, name, g):
    """P3 over the full 30-step schedule at 256^2: the native pipeline's final latents vs the reference's fp32
    trajectory, beside (and above) the reference's own bf16 run; at CFG 1, where the CFG-6 noise amplification
    is absent, the SURVEY §8d bar of 40 dB applies as stated."""
    gd, meta = gold3
    key = f"{name}.256.s30.g{g:g}"
    if f"{key}.f32.final" not in gd:
        pytest.skip(f"{key} not in the fixture file")
    model = m7b if name == "7b" else m10b
    out = FLitePipeline(model)(prompt_embeds=hashed(meta, "ctx"), latents=hashed(meta, "latents_256"), height=256,
                               width=256, num_inference_steps=30, guidance_scale=g,
                               output_type="latent").images.float()
    p = psnr(out / SCALING + SHIFT, gd[f"{key}.f32.final"])
    floor = meta[f"{key}.bf16_vs_f32_psnr"]
    print(f"{name} 256^2 30-step CFG-{g:g} final latents: {p:.2f} dB vs reference fp32 (reference's own bf16 run: "
          f"{floor:.2f} dB)")
    assert p >= floor
    if g == 1.0:
        assert p >= 40.0


# ---- the METRIC configuration pinned end to end (tests/golden/make_golden_full4.py) ----
@pytest.fixture(scope="module")
def gold4():
    from safetensors.torch import load_file

    f = GOLD / "golden_full4.safetensors"
    if not f.exists():
        pytest.skip("golden_full4.safetensors not generated")
    return load_file(str(f)), json.loads((GOLD / "golden_full4_meta.json").read_text())


@pytest.mark.parametrize("name,g", [("10b", 6.0), ("10b", 1.0), ("7b", 1.0), ("7b", 6.0)])
def test_10b_1024_30_steps_vs_reference(gold4, m7b, m10b, name, g):
    """BASELINE's metric workload end to end against the reference itself: 10B (model_v2 layout), 1024^2, 30 steps,
    the hipGraph-captured loop the bench times (and configs[1]'s 7B, model.py layout, where the fixture holds it).
    P3 final latents vs the reference's fp32 trajectory, beside (and above) the reference's own bf16 run; at CFG 1
    the SURVEY §8d bar of 40 dB. Then the uint8 image of the product path (HIP loop + HIP VAE) vs oracle/vae_ref.py's
    decode of the reference's fp32 latents (peak 255): >= 40 dB at CFG 1; at CFG 6 at least the reference's own
    bf16 run's image (decoded the same way)."""
    from f_lite.vae import AutoencoderKL

    gd, meta = gold4
    key = f"{name}.1024.s30.g{g:g}"
    assert f"{key}.f32.final" in gd, f"{key}.f32.final missing from golden_full4.safetensors"
    pipe = FLitePipeline(m7b if name == "7b" else m10b, vae=AutoencoderKL.random(seed=0))
    assert (pipe.vae.config.scaling_factor, pipe.vae.config.shift_factor) == (SCALING, SHIFT)
    kw = dict(prompt_embeds=hashed(meta, "ctx"), latents=hashed(meta, "latents_1024"), height=1024, width=1024,
              num_inference_steps=30, guidance_scale=g, use_graph=True)
    lat = pipe(**kw, output_type="latent").images.float()
    p = psnr(lat / SCALING + SHIFT, gd[f"{key}.f32.final"])
    floor = meta.get(f"{key}.bf16_vs_f32_psnr")
    print(f"{name} 1024^2 30-step CFG-{g:g} final latents: {p:.2f} dB vs reference fp32 (reference's own bf16 run: "
          f"{'n/a' if floor is None else f'{floor:.2f} dB'})")
    if g == 1.0:
        assert p >= 40.0  # SURVEY §8d as stated; the reference's own bf16 run, where generated, as well
        if floor is not None:
            assert p >= floor
    else:
        # CFG 6 amplifies every rounding along the trajectory, so the bar is the reference's own bf16 run of the same
        # 30 steps; a CFG-6 case without that floor is a missing fixture, never "no assertion" 
        assert floor is not None, f"{key}.bf16_vs_f32_psnr missing: run make_golden_full4.py --only {key}.bf16"
        assert p >= floor
    assert f"{key}.f32.image" in gd, f"{key}.f32.image missing: run make_golden_full4.py (it decodes every final)"
    img = pipe(**kw, output_type="uint8").images.cpu()
    ref = gd[f"{key}.f32.image"]
    assert img.shape == ref.shape == (1, 1024, 1024, 3)
    pi = 10 * math.log10(255.0 ** 2 / max((img.double() - ref.double()).pow(2).mean().item(), 1e-12))
    ifloor = meta.get(f"{key}.image_bf16_vs_f32_psnr")
    print(f"  uint8 image (HIP loop + HIP VAE) vs oracle VAE on the reference latents: {pi:.2f} dB (the "
          f"reference's own bf16 run: {'n/a' if ifloor is None else f'{ifloor:.2f} dB'})")
    if g == 1.0:
        assert pi >= 40.0  # the bar applies as stated where CFG 6 does not amplify the noise
    else:
        assert ifloor is not None, f"{key}.image_bf16_vs_f32_psnr missing: the bf16 trajectory's image"
        assert pi >= ifloor


@pytest.mark.parametrize("name", ["10b", "7b"])
def test_fp8_first_blocks_bf16_1024_cfg1_vs_reference(gold4, m7b, m10b, name):
    """BASELINE configs[4]'s MXFP8 path at the metric's size against the reference itself (DESIGN §5 "fp8 against the
    reference"): 1024^2, 30 steps, CFG 1 (no CFG amplification), final latents vs the reference's fp32 trajectory.
    The quality-leaning policy (blocks 0-7 bf16, every GEMM class MXFP8 in blocks 8-39; 1.40x the bf16 image) must
    meet the SURVEY §8d bar of 40 dB. The all-fp8 policy is printed beside it; it is the BASELINE row and the default,
    and no bar applies to it here."""
    gd, meta = gold4
    key = f"{name}.1024.s30.g1"
    if f"{key}.f32.final" not in gd:
        pytest.skip(f"{key} not in the fixture file")
    model = m7b if name == "7b" else m10b
    kw = dict(prompt_embeds=hashed(meta, "ctx"), latents=hashed(meta, "latents_1024"), height=1024, width=1024,
              num_inference_steps=30, guidance_scale=1.0, output_type="latent")
    res = {}
    try:
        for label, blocks in (("all fp8", []), ("bf16 blocks 0-7", list(range(8)))):
            model.enable_fp8(True, bf16_blocks=blocks)
            lat = FLitePipeline(model)(**kw).images.float()
            res[label] = psnr(lat / SCALING + SHIFT, gd[f"{key}.f32.final"])
    finally:
        model.enable_fp8(False, bf16_blocks=[])
    print(f"fp8 {name} 1024^2 30-step CFG-1 final latents vs reference fp32: " +
          ", ".join(f"{k} {v:.2f} dB" for k, v in res.items()))
    assert res["bf16 blocks 0-7"] >= 40.0


def test_fp8_7b_cfg6_policy_meets_reference_floor(gold4, m7b):
    """MXFP8 at the BASELINE row's guidance (CFG 6) against the reference itself (VERDICT r05 missing 2; DESIGN §5
    "Per-block fp8 policies"): for 7B (configs[1]'s model) the policy "blocks 0-15 bf16, every class MXFP8 in 16-39"
    keeps the 30-step 1024^2 final latents at least as close to the reference's fp32 run as the reference's own bf16
    run (27.37 dB; measured 27.87 dB). No such policy exists for 10B (the table there)."""
    gd, meta = gold4
    key = "7b.1024.s30.g6"
    floor = meta.get(f"{key}.bf16_vs_f32_psnr")
    if f"{key}.f32.final" not in gd or floor is None:
        pytest.skip(f"{key} fixtures not generated")
    kw = dict(prompt_embeds=hashed(meta, "ctx"), latents=hashed(meta, "latents_1024"), height=1024, width=1024,
              num_inference_steps=30, guidance_scale=6.0, output_type="latent")
    try:
        m7b.enable_fp8(True, bf16_blocks=list(range(16)))
        lat = FLitePipeline(m7b)(**kw).images.float()
    finally:
        m7b.enable_fp8(False, bf16_blocks=[])
    p = psnr(lat / SCALING + SHIFT, gd[f"{key}.f32.final"])
    print(f"fp8 (bf16 blocks 0-15) 7b 1024^2 30-step CFG-6 final latents: {p:.2f} dB vs reference fp32 (reference's "
          f"own bf16 run: {floor:.2f} dB)")
    assert p >= floor


# ---- the reference's DEFAULT configuration pinned end to end (tests/golden/make_golden_full5.py) --
@pytest.fixture(scope="module")
def gold5():
    from safetensors.torch import load_file

    f = GOLD / "golden_full5.safetensors"
    if not f.exists():
        pytest.skip("golden_full5.safetensors not generated")
    return load_file(str(f)), json.loads((GOLD / "golden_full5_meta.json").read_text())


def _uint8_psnr(img, ref):
    return 10 * math.log10(255.0 ** 2 / max((img.double() - ref.double()).pow(2).mean().item(), 1e-12))


@pytest.mark.parametrize("g", [1.0, 6.0])
def test_10b_1344x896_30_steps_vs_reference(gold5, m10b, g):
    """generate.py:19-22's defaults end to end against the reference itself: 10B (model_v2 layout), 1344x896 (T = 4720:
    the non-square 56 x 84 RoPE grid of model.py:334-400, alpha = 4.2866 from pipeline.py:240-242, 112-row attention
    tails and the 256-row attention route), 30 steps, the hipGraph loop the bench times, then generate.py:77-78's tiled
    VAE decode (2 x 2 overlapping tiles) to uint8. Final latents vs the reference's fp32 trajectory: >= 40 dB at CFG 1
     and at least the reference's own bf16 run; at CFG 6, at least the reference's own bf16 run. The uint8
    image vs oracle/vae_ref.py's tiled decode of the reference latents: >= 40 dB at CFG 1, at CFG 6 at least the
    reference's bf16 image."""
    from f_lite.vae import AutoencoderKL

    gd, meta = gold5
    key = f"10b.1344x896.s30.g{g:g}"
    if f"{key}.f32.final" not in gd:
        pytest.skip(f"{key}.f32.final not generated yet (tests/golden/make_golden_full5.py)")
    floor = meta.get(f"{key}.bf16_vs_f32_psnr")
    if g != 1.0 and floor is None:
        pytest.skip(f"{key}.bf16 (the CFG-6 floor) not generated yet (tests/golden/make_golden_full5.py)")
    assert abs(meta["alpha"] - 4.2866) < 1e-4
    pipe = FLitePipeline(m10b, vae=AutoencoderKL.random(seed=0))
    pipe.enable_vae_tiling()
    kw = dict(prompt_embeds=hashed(meta, "ctx"), latents=hashed(meta, "latents"), height=896, width=1344,
              num_inference_steps=30, guidance_scale=g, use_graph=True)
    lat = pipe(**kw, output_type="latent").images.float()
    p = psnr(lat / SCALING + SHIFT, gd[f"{key}.f32.final"])
    print(f"10b 1344x896 30-step CFG-{g:g} final latents: {p:.2f} dB vs reference fp32 (reference's own bf16 run: "
          f"{'n/a' if floor is None else f'{floor:.2f} dB'})")
    if g == 1.0:
        assert p >= 40.0
    if floor is not None:
        assert p >= floor
    ref = gd.get(f"{key}.f32.image")
    if ref is None:
        pytest.skip(f"{key}.f32.image not decoded yet")
    img = pipe(**kw, output_type="uint8").images.cpu()
    assert img.shape == ref.shape == (1, 896, 1344, 3)
    pi = _uint8_psnr(img, ref)
    ifloor = meta.get(f"{key}.image_bf16_vs_f32_psnr")
    print(f"  uint8 image (HIP loop + HIP tiled VAE) vs oracle tiled VAE on the reference latents: {pi:.2f} dB "
          f"(the reference's own bf16 run: {'n/a' if ifloor is None else f'{ifloor:.2f} dB'})")
    if g == 1.0:
        assert pi >= 40.0
    if ifloor is not None:
        assert pi >= ifloor


def test_fp8_first_blocks_bf16_1344x896_cfg1_vs_reference(gold5, m10b):
    """BASELINE configs[4]'s MXFP8 path at its own size (1344x896) against the reference's fp32 trajectory at CFG 1:
    the quality policy (blocks 0-7 bf16, MXFP8 elsewhere) meets the SURVEY §8d bar of 40 dB; the all-fp8 default is
    printed beside it."""
    gd, meta = gold5
    key = "10b.1344x896.s30.g1"
    if f"{key}.f32.final" not in gd:
        pytest.skip(f"{key}.f32.final not generated yet")
    kw = dict(prompt_embeds=hashed(meta, "ctx"), latents=hashed(meta, "latents"), height=896, width=1344,
              num_inference_steps=30, guidance_scale=1.0, output_type="latent")
    res = {}
    try:
        for label, blocks in (("all fp8", []), ("bf16 blocks 0-7", list(range(8)))):
            m10b.enable_fp8(True, bf16_blocks=blocks)
            lat = FLitePipeline(m10b)(**kw).images.float()
            res[label] = psnr(lat / SCALING + SHIFT, gd[f"{key}.f32.final"])
    finally:
        m10b.enable_fp8(False, bf16_blocks=[])
    print("fp8 10b 1344x896 30-step CFG-1 final latents vs reference fp32: " +
          ", ".join(f"{k} {v:.2f} dB" for k, v in res.items()))
    assert res["bf16 blocks 0-7"] >= 40.0
