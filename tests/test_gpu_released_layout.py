"""GPU: the RELEASED-checkpoint layout, train_bias_and_rms=False -- what pt.py:31 (load_f_lite_pt) builds for the
published F-Lite weights: no qkv / q / context_kv biases (model.py:465) and a weight-less final RMSNorm
(model.py:474). Bars: >= 40 dB vs the reference's own fp32 outputs (tests/golden/golden_nobias.safetensors, made
by make_golden_nobias.py from the stub-loaded reference) and vs the fp32 oracle at full width; a .pt checkpoint
written the way training saves it (DDP / torch.compile prefixes) loads through load_f_lite_pt and samples
bit-identically to the same weights built directly."""
import dataclasses

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no ROCm device", allow_module_level=True)

from f_lite import DiT, FLitePipeline  # noqa: E402
from f_lite.model import PRESETS  # noqa: E402
from oracle import flite_ref as R  # noqa: E402

DEV = "cuda"


def _nobias(preset):
    return dict(PRESETS[preset], train_bias_and_rms=False)


@pytest.mark.parametrize("preset,mask", [("tiny", False), ("tiny", True), ("tiny_v2", False)])
def test_released_layout_vs_reference(golden, golden_nobias, preset, mask):
    m = DiT.random(seed=0, device=DEV, **_nobias(preset))
    assert m.final_norm.weight is None and m.blocks[0].self_attn.qkv.bias is None
    assert not any(k.endswith(("qkv.bias", "q.bias", "context_kv.bias")) for k in m.state_dict())
    x, ctx, t = golden["in.x"], golden["in.ctx"], golden["in.t"]
    out = m(x.bfloat16().to(DEV), ctx.bfloat16().to(DEV), golden["in.mask"].to(DEV) if mask else None, t.to(DEV),
            output_dtype=torch.float32).cpu()
    ref = golden_nobias[f"dit.{preset}.nobias.f32.{'mask' if mask else 'nomask'}"]
    p = R.psnr(out, ref)
    print(f"{preset} train_bias_and_rms=False{' (ragged mask)' if mask else ''}: {p:.2f} dB vs the reference")
    assert p >= 40.0


def test_released_layout_full_width():
    """10B layout without biases at the reference's default 1344x896 (T = 4720), 512-token context, depth 1."""
    cfg = dict(_nobias("10b"), depth=1)
    m = DiT.random(seed=0, device=DEV, **cfg)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 16, 112, 168, generator=g).bfloat16()
    ctx = torch.randn(2, 512, 4096, generator=g).bfloat16()
    t = torch.tensor([0.75, 0.75]).bfloat16()
    out = m(x.to(DEV), ctx.to(DEV), None, t.to(DEV), output_dtype=torch.float32).cpu()
    ref_cfg = dataclasses.replace(R.PRESETS["10b"], depth=1, train_bias_and_rms=False)
    with torch.no_grad():
        ref = R.RefDiT.random(ref_cfg, dtype=torch.float32)(x.float(), ctx.float(), None, t)
    p = R.psnr(out, ref)
    print(f"10B layout, train_bias_and_rms=False, depth 1, 1344x896: {p:.2f} dB vs the fp32 oracle")
    assert p >= 40.0


def test_pt_checkpoint_roundtrip(tmp_path):
    """training-style .pt (module. / _orig_mod. prefixes) -> load_f_lite_pt (pt.py:15-179 defaults:
    train_bias_and_rms=False, heads = width // 256) -> 4-step CFG sampling == the directly built model's."""
    from f_lite.pt import load_f_lite_pt

    cfg = _nobias("tiny")
    m = DiT.random(seed=3, device=DEV, **cfg)
    sd = {("module._orig_mod." + k): v.detach().cpu().clone() for k, v in m.state_dict().items()}
    torch.save(sd, tmp_path / "f_lite.pt")
    pipe = load_f_lite_pt(tmp_path / "f_lite.pt", torch.device(DEV), dtype="bfloat16", width=512,
                          cross_attn_input_size=128)
    assert pipe.dit_model.config.depth == cfg["depth"] and pipe.dit_model.config.num_heads == 2
    assert not pipe.dit_model.config.train_bias_and_rms
    g = torch.Generator().manual_seed(8)
    lat = torch.randn(1, 16, 16, 16, generator=g).bfloat16().to(DEV)
    pos = torch.randn(1, 24, 128, generator=g).bfloat16().to(DEV)
    kw = dict(prompt_embeds=pos, latents=lat, height=128, width=128, num_inference_steps=4, guidance_scale=6.0,
              output_type="latent")
    got = pipe(**kw).images
    want = FLitePipeline(m)(**kw).images
    assert torch.isfinite(got.float()).all()
    assert torch.equal(got, want)
