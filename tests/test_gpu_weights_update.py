"""GPU: derived weight copies follow IN-PLACE weight updates (load_state_dict copies into the existing storage,
so the parameter pointers do not change; only their version counters do).

The bf16 DiT path reads the bound storage directly; the fp8 path runs on engine-owned MXFP8 copies and the VAE
on engine-owned packed conv weights -- both must be remade (include/flite.h flite_dit_weights_updated /
flite_vae_weights_updated). Bar: after sample -> load_state_dict(new) -> sample, the output is bit-identical to a
model built fresh from the new weights, in bf16 and fp8 modes (including the hipGraph replay and an fp8
off/update/on toggle) and for the VAE in bf16 and fp8 weight storage."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no ROCm device", allow_module_level=True)

from f_lite import DiT, FLitePipeline  # noqa: E402
from f_lite.model import PRESETS  # noqa: E402
from f_lite.vae import AutoencoderKL  # noqa: E402

DEV = "cuda"


def _inputs():
    g = torch.Generator().manual_seed(13)
    lat = torch.randn(1, 16, 16, 16, generator=g).bfloat16().to(DEV)
    pos = torch.randn(1, 24, 128, generator=g).bfloat16().to(DEV)
    return lat, pos


def _sample(m, graph=True):
    lat, pos = _inputs()
    return FLitePipeline(m)(prompt_embeds=pos, latents=lat, height=128, width=128, num_inference_steps=4,
                            guidance_scale=6.0, output_type="latent", use_graph=graph).images.float().cpu()


def _fresh(seed, fp8):
    m = DiT.random(seed=seed, device=DEV, **PRESETS["tiny"])
    if fp8:
        m.enable_fp8(True)
    return m


@pytest.mark.parametrize("fp8", [False, True])
def test_dit_load_state_dict_in_place(fp8):
    m = _fresh(0, fp8)
    before = _sample(m)
    new_sd = DiT.random(seed=1, device=DEV, **PRESETS["tiny"]).state_dict()
    ptrs = [p.data_ptr() for p in m.parameters()]
    m.load_state_dict(new_sd)  # copies into the existing storage
    assert ptrs == [p.data_ptr() for p in m.parameters()]
    after = _sample(m)  # the cached hipGraph replays on the same pointers
    want = _sample(_fresh(1, fp8))
    assert not torch.equal(before, after)
    assert torch.equal(after, want)
    assert torch.equal(_sample(m, graph=False), want)


def test_dit_fp8_toggle_after_update():
    """enable_fp8(False) -> update -> enable_fp8(True) requantises (the copies from before are stale)."""
    m = _fresh(0, True)
    _sample(m)
    m.enable_fp8(False)
    m.load_state_dict(DiT.random(seed=2, device=DEV, **PRESETS["tiny"]).state_dict())
    m.enable_fp8(True)
    assert torch.equal(_sample(m), _sample(_fresh(2, True)))


def test_dit_random_init_in_place_and_rebind_keep_fp8():
    """random_init_ writes through raw pointers (no version bump): tracked by the model; rebinding one weight
    to NEW storage keeps fp8 mode on and requantises before the next run (flite.h flite_dit_enable_fp8)."""
    m = _fresh(0, True)
    _sample(m)
    m.random_init_(seed=4)
    assert torch.equal(_sample(m), _sample(_fresh(4, True)))
    w = m.blocks[1].mlp.down_proj
    w.weight = torch.nn.Parameter(w.weight.detach().clone() * 0.5)  # new storage
    ref = _fresh(4, False)
    with torch.no_grad():
        ref.blocks[1].mlp.down_proj.weight.mul_(0.5)
    ref.enable_fp8(True)
    got = _sample(m)
    assert torch.equal(got, _sample(ref))
    m.enable_fp8(False)
    assert not torch.equal(got, _sample(m))  # it really was the fp8 path


@pytest.mark.parametrize("fp8", [False, True])
def test_vae_load_state_dict_in_place(fp8):
    lat = torch.randn(1, 16, 8, 8, generator=torch.Generator().manual_seed(5)).to(DEV)

    def make(seed):
        v = AutoencoderKL.random(seed=seed)
        if fp8:
            v.enable_layerwise_casting(torch.float8_e4m3fn, torch.bfloat16)
        return v

    v = make(0)
    before = v.decode_to_uint8(lat).cpu()
    v.load_state_dict(AutoencoderKL.random(seed=1).state_dict())
    after = v.decode_to_uint8(lat).cpu()
    want = make(1).decode_to_uint8(lat).cpu()
    assert not torch.equal(before, after)
    assert torch.equal(after, want)


@pytest.mark.parametrize("preset", ["tiny", "tiny_v2"])
def test_lora_merged_forward_matches_oracle(preset):
    """LoRA (pt.py:107-135 / model.py:492-495, merged by f_lite/lora.py) on a model that has already run: the
    in-place merge rebinds the engine (its cross-attention K/V cache included) and the forward matches the fp32
    oracle on W + B @ A unrounded (>= 40 dB), far from the base model's output. Parity against peft itself is
    unpinned (peft is not installed); the adapter math is peft's published base(x) + B(A(x)) * alpha / r, r = alpha."""
    from f_lite.lora import merge_lora_
    from oracle import flite_ref as R

    m = DiT.random(seed=0, device=DEV, **PRESETS[preset])
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 16, 16, 16, generator=g).bfloat16()
    ctx = torch.randn(2, 24, 128, generator=g).bfloat16()
    t = torch.tensor([0.7, 0.7])
    base = m(x.to(DEV), ctx.to(DEV), None, t.to(DEV), output_dtype=torch.float32).cpu()
    lsd = {}
    for name, mod in m.named_modules():
        if isinstance(mod, torch.nn.Linear) and name.rsplit(".", 1)[-1] in ("qkv", "q", "context_kv", "proj"):
            lsd[f"{name}.lora_A.weight"] = torch.randn(8, mod.in_features, generator=g) * 0.05
            lsd[f"{name}.lora_B.weight"] = torch.randn(mod.out_features, 8, generator=g) * 0.05
    assert merge_lora_(m, lsd, target_modules=["qkv", "q", "context_kv", "proj"], rank=8) == len(lsd) // 2
    out = m(x.to(DEV), ctx.to(DEV), None, t.to(DEV), output_dtype=torch.float32).cpu()
    params = R.make_state_dict(R.PRESETS[preset].as_dict(), seed=0)
    for k in list(params):
        mod = k[: -len(".weight")]
        if f"{mod}.lora_A.weight" in lsd:
            params[k] = params[k] + lsd[f"{mod}.lora_B.weight"] @ lsd[f"{mod}.lora_A.weight"]
    ref = R.RefDiT(R.PRESETS[preset], params, dtype=torch.float32)(x.float(), ctx.float(), None, t)
    p, p_base = R.psnr(out, ref), R.psnr(base, ref)
    print(f"{preset} LoRA-merged forward vs fp32 oracle: {p:.2f} dB (base model: {p_base:.2f} dB)")
    assert p >= 40.0 and p_base < p - 10


def test_engine_refuses_stale_context():
    """include/flite.h flite_dit_weights_updated: the context K/V cached by set_context were projected with the old
    weights, so forward fails until the context is set again (the Python wrappers always set it per call)."""
    from f_lite import _native

    m = DiT.random(seed=0, device=DEV, **PRESETS["tiny"])
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 16, 16, 16, generator=g).to(DEV)
    ctx = torch.randn(2 * 24, 128, generator=g).bfloat16().to(DEV)
    m(x, ctx.view(2, 24, 128), None, torch.tensor([0.5, 0.5]).to(DEV))  # binds and prepares the engine
    eng = m.engine()
    out = torch.empty(2, 16, 16, 16, device=DEV)
    eng.set_context(ctx, [0, 24, 48])
    eng.forward(x, out, 0, 1)
    eng.weights_updated(DEV)
    with pytest.raises(_native.FliteError, match="set the context again"):
        eng.forward(x, out, 0, 1)
    eng.set_context(ctx, [0, 24, 48])
    eng.forward(x, out, 0, 1)
