"""Generate the golden fixtures from the REFERENCE implementation (run in the build container only).

Imports /root/reference/f_lite/{model,model_v2,pipeline}.py with in-memory stubs for the third-party
packages that are not installed here (diffusers, peft, liger_kernel, flash_attn_interface).
The stubs restate only: config capture, module base classes, and the documented math of LigerRMSNorm
("llama" casting), LigerSwiGLUMLP and flash_attn_varlen_func. Everything else that runs is the
reference's own code. Weights come from oracle.weights (deterministic generator) and are loaded into the
reference module with load_state_dict(strict=True), which also pins our parameter inventory.

Outputs (small, committed): tests/golden/*.safetensors + golden_meta.json. No reference source or
bytecode is written into the repository (sys.dont_write_bytecode).

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import sys

sys.dont_write_bytecode = True

import dataclasses  # noqa: E402
import functools  # noqa: E402
import importlib.util  # noqa: E402
import inspect  # noqa: E402
import json  # noqa: E402
import math  # noqa: E402
import types  # noqa: E402
from pathlib import Path  # noqa: E402

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from safetensors.torch import save_file  # noqa: E402

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
REF = Path("/root/reference/f_lite")
OUT = Path(__file__).resolve().parent

from oracle.weights import make_state_dict  # noqa: E402


def install_stubs():
    # transformers probes flash_attn_interface.__spec__; import it before the stub exists.
    from transformers import Qwen2_5_VLModel, Qwen2_5_VLProcessor  # noqa: F401

    def mod(name):
        m = types.ModuleType(name)
        sys.modules[name] = m
        return m

    # ---- diffusers ----
    d = mod("diffusers")
    cu = mod("diffusers.configuration_utils")

    class ConfigMixin:
        pass

    def register_to_config(init):
        @functools.wraps(init)
        def wrapper(self, *args, **kwargs):
            bound = inspect.signature(init).bind(self, *args, **kwargs)
            bound.apply_defaults()
            cfg = dict(bound.arguments)
            cfg.pop("self")
            init(self, *args, **kwargs)
            object.__setattr__(self, "config", types.SimpleNamespace(**cfg))

        return wrapper

    cu.ConfigMixin = ConfigMixin
    cu.register_to_config = register_to_config
    loaders = mod("diffusers.loaders")

    class FromOriginalModelMixin:
        pass

    class PeftAdapterMixin:
        pass

    loaders.FromOriginalModelMixin = FromOriginalModelMixin
    loaders.PeftAdapterMixin = PeftAdapterMixin
    mod("diffusers.models")
    mu = mod("diffusers.models.modeling_utils")

    class ModelMixin(nn.Module):
        pass

    mu.ModelMixin = ModelMixin
    du = mod("diffusers.utils")

    class BaseOutput:
        pass

    du.BaseOutput = BaseOutput
    au = mod("diffusers.utils.accelerate_utils")
    au.apply_forward_hook = lambda f: f
    tu = mod("diffusers.utils.torch_utils")
    tu.randn_tensor = lambda shape, generator=None, device=None, dtype=None: torch.randn(
        shape, generator=generator, dtype=dtype)

    class AutoencoderKL(nn.Module):
        pass

    class DiffusionPipeline:
        def __init__(self):
            pass

        def register_modules(self, **kw):
            for k, v in kw.items():
                setattr(self, k, v)

        @property
        def _execution_device(self):
            return torch.device("cpu")

        def maybe_free_model_hooks(self):
            pass

    d.AutoencoderKL = AutoencoderKL
    d.DiffusionPipeline = DiffusionPipeline

    # ---- peft ----
    pf = mod("peft")
    pf.get_peft_model_state_dict = lambda m: {}
    pf.set_peft_model_state_dict = lambda m, sd: None

    # ---- liger_kernel (documented math) ----
    mod("liger_kernel")
    lt = mod("liger_kernel.transformers")

    class LigerRMSNorm(nn.Module):
        def __init__(self, hidden_size, eps=1e-6):
            super().__init__()
            self.weight = nn.Parameter(torch.ones(hidden_size))
            self.variance_epsilon = eps

        def forward(self, x):
            xf = x.float()
            r = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.variance_epsilon)
            return self.weight * (xf * r).to(x.dtype)

    class LigerSwiGLUMLP(nn.Module):
        def __init__(self, config):
            super().__init__()
            self.gate_proj = nn.Linear(config.hidden_size, config.intermediate_size, bias=False)
            self.up_proj = nn.Linear(config.hidden_size, config.intermediate_size, bias=False)
            self.down_proj = nn.Linear(config.intermediate_size, config.hidden_size, bias=False)

        def forward(self, x):
            a = self.gate_proj(x)
            b = self.up_proj(x)
            return self.down_proj(F.silu(a.float()).to(b.dtype) * b)

    lt.LigerRMSNorm = LigerRMSNorm
    lt.LigerSwiGLUMLP = LigerSwiGLUMLP

    # ---- flash_attn_interface (documented math) ----
    fa = mod("flash_attn_interface")

    def flash_attn_varlen_func(q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, softmax_scale):
        out = torch.empty_like(q)
        for b in range(len(cu_seqlens_q) - 1):
            qs, qe = int(cu_seqlens_q[b]), int(cu_seqlens_q[b + 1])
            ks, ke = int(cu_seqlens_k[b]), int(cu_seqlens_k[b + 1])
            s = torch.einsum("qhd,khd->hqk", q[qs:qe].float(), k[ks:ke].float()) * softmax_scale
            p = torch.softmax(s, -1)
            out[qs:qe] = torch.einsum("hqk,khd->qhd", p, v[ks:ke].float()).to(q.dtype)
        return out, None

    fa.flash_attn_varlen_func = flash_attn_varlen_func


def load_ref(name):
    spec = importlib.util.spec_from_file_location(f"f_lite.{name}", REF / f"{name}.py")
    m = importlib.util.module_from_spec(spec)
    sys.modules[f"f_lite.{name}"] = m
    spec.loader.exec_module(m)
    return m


TINY = dict(in_channels=16, patch_size=2, hidden_size=512, depth=10, num_heads=2, mlp_ratio=4.0,
            cross_attn_input_size=128, train_bias_and_rms=True, use_rope=True, gradient_checkpoint=False,
            dynamic_softmax_temperature=False, rope_base=10000)
TINY_V2 = dict(TINY, depth=3)


def build(model_mod, cfg, per_block, dtype):
    dit = model_mod.DiT(**cfg)
    sd = make_state_dict(dict(cfg, per_block_adaln=per_block), seed=0)
    missing, unexpected = dit.load_state_dict(sd, strict=True)
    assert not missing and not unexpected
    return dit.to(dtype).eval()


def v2_forward_fixed(dit, model_v2, x, context, context_attn_mask, timesteps):
    """model_v2.DiT.forward (model_v2.py:528-594), repaired: the file repeat_interleaves t_emb per token
    (model_v2.py:555-558) and every DiTBlock repeats it AGAIN (model_v2.py:275-276), and final_modulation gets
    the per-token t_emb (model_v2.py:581-583); both raise. Blocks get the per-sample t_emb (they expand it
    themselves) and the final stage is model.py:578-580."""
    prep = model_v2.prepare_flash_attention_inputs
    context = dit.context_norm(dit.context_proj(context))
    cf, ccu, cmax, _ = prep(context, context_attn_mask)
    b, c, h, w = x.shape
    x = dit.patch_embed(x)
    x = torch.cat([dit.register_tokens.repeat(b, 1, 1), x], 1)
    p = dit.config.patch_size
    cos, sin = dit.rope(x, extend_with_register_tokens=16, height_width=(h // p, w // p))
    cos = cos.repeat(1, b, 1)
    sin = sin.repeat(1, b, 1)
    xf, xcu, xmax, xidx = prep(x)
    t_emb = model_v2.timestep_embedding(timesteps * 1000, dit.config.hidden_size).to(x.device, dtype=x.dtype)
    t_emb = dit.time_embed(t_emb)
    T = 16 + h // p * w // p
    for blk in dit.blocks:
        xf = blk(xf, xcu, xmax, cf, ccu, cmax, t_emb, (cos, sin), T)
    x = model_v2.unprepare_flash_attention_outputs(xf, xidx, b, xmax, dit.config.hidden_size)[:, 16:, :]
    shift, scale = dit.final_modulation(t_emb).chunk(2, dim=1)
    x = dit.final_norm(x)
    x = x * (1 + scale[:, None, :]) + shift[:, None, :]
    x = dit.final_proj(x)
    hp, wp = h // p, w // p
    C = dit.config.in_channels
    return x.reshape(b, hp, wp, p, p, C).permute(0, 5, 1, 3, 2, 4).reshape(b, C, h, w)


class ThreeArg(nn.Module):
    """pipeline.py:271 calls dit_model(x, ctx, t); DiT.forward needs the mask argument."""

    def __init__(self, dit):
        super().__init__()
        self.dit = dit

    def forward(self, x, ctx, t):
        return self.dit(x, ctx, None, t)


class StubVAE:
    def __init__(self, dtype):
        self.config = types.SimpleNamespace(scaling_factor=0.3611, shift_factor=0.1159)
        self.dtype = dtype
        self.seen = None

    def to(self, *a, **k):
        return self

    def requires_grad_(self, *a):
        return self

    def decode(self, z):
        self.seen = z.detach().clone()
        return types.SimpleNamespace(sample=torch.zeros(z.shape[0], 3, z.shape[2] * 8, z.shape[3] * 8, dtype=z.dtype))


class StubEncoder:
    device = torch.device("cpu")

    def requires_grad_(self, *a):
        return self


def run_pipeline(pipeline_mod, dit, latents, pos, neg, steps, guidance, apg, height, width):
    vae = StubVAE(latents.dtype)
    pipe = pipeline_mod.FLitePipeline(ThreeArg(dit), vae, StubEncoder(), None)
    pipe.encode_prompt = lambda **kw: (pos.to(kw.get("dtype")), neg.to(kw.get("dtype")))
    pipeline_mod.randn_tensor = lambda shape, generator=None, device=None, dtype=None: latents.clone().to(dtype)
    pipe.set_progress_bar_config(disable=True)
    apg_cfg = pipeline_mod.APGConfig(enabled=True) if apg else None
    pipe(prompt="x", height=height, width=width, num_inference_steps=steps, guidance_scale=guidance,
         apg_config=apg_cfg)
    # vae.seen = latents / scaling_factor + shift_factor (pipeline.py:304)
    return vae.seen


def main():
    torch.manual_seed(1234)
    install_stubs()
    model = load_ref("model")
    model_v2 = load_ref("model_v2")
    pipeline = load_ref("pipeline")
    T = {}
    meta = {"generator": "oracle.weights seed=0 std=0.02 (norm weights 1)", "configs": {"tiny": TINY,
            "tiny_v2": TINY_V2}, "reference": "/root/reference f_lite/model.py, model_v2.py, pipeline.py"}

    # ---- inputs (generated here, stored) ----
    g = torch.Generator().manual_seed(7)
    x = torch.randn(2, 16, 16, 16, generator=g)
    ctx = torch.randn(2, 24, 128, generator=g)
    mask = torch.ones(2, 24)
    mask[1, 17:] = 0
    ts = torch.tensor([0.75, 0.3])
    T["in.x"] = x
    T["in.ctx"] = ctx
    T["in.mask"] = mask
    T["in.t"] = ts

    with torch.no_grad():
        # ---- per-op vectors of the reference's own helpers ----
        tq = torch.tensor([1.0, 0.75, 0.5, 0.1, 0.9333333], dtype=torch.bfloat16)
        T["op.temb_bf16t.t"] = tq.float()
        T["op.temb_bf16t.out"] = model.timestep_embedding(tq * 1000, 512)
        tf = torch.tensor([1.0, 0.75, 0.5, 0.1, 0.9333333])
        T["op.temb_f32t.t"] = tf
        T["op.temb_f32t.out"] = model.timestep_embedding(tf * 1000, 512)
        rope = model.TwoDimRotary(128, base=10000, h=512, w=512)
        cos, sin = rope(torch.zeros(1, 16 + 12 * 20, 1), height_width=(12, 20), extend_with_register_tokens=16)
        T["op.rope.cos"] = cos[0]
        T["op.rope.sin"] = sin[0]
        rope_bf = rope.to(torch.bfloat16)
        cb, sb = rope_bf(torch.zeros(1), height_width=(12, 20), extend_with_register_tokens=16)
        T["op.rope_bf16.cos"] = cb[0].float()
        T["op.rope_bf16.sin"] = sb[0].float()
        xr = torch.randn(2, 256, 256, generator=g)
        T["op.apply_rope.x"] = xr
        T["op.apply_rope.out"] = model.apply_rotary_emb(xr, cos[:, :256], sin[:, :256])
        xn = torch.randn(7, 512, generator=g) * 3
        T["op.rmsnorm.x"] = xn
        rn = model.RMSNorm(512, trainable=True)
        rn.weight.data = torch.randn(512, generator=g)
        T["op.rmsnorm.w"] = rn.weight.data.clone()
        T["op.rmsnorm.out"] = rn(xn)
        T["op.rmsnorm_noweight.out"] = model.RMSNorm(512)(xn)

        # ---- DiT forward, v1 tiny, fp32 and bf16; with and without ragged context mask ----
        dit32 = build(model, TINY, False, torch.float32)
        T["dit.tiny.f32.nomask"] = dit32(x, ctx, None, ts)
        T["dit.tiny.f32.mask"] = dit32(x, ctx, mask, ts)
        T["dit.tiny.f32.bf16t"] = dit32(x, ctx, None, ts.to(torch.bfloat16))
        dit16 = build(model, TINY, False, torch.bfloat16)
        T["dit.tiny.bf16.nomask"] = dit16(x.bfloat16(), ctx.bfloat16(), None, ts.bfloat16()).float()
        # ---- v2 tiny (per-block adaLN, cross everywhere), fixed final stage ----
        dv2 = build(model_v2, TINY_V2, True, torch.float32)
        T["dit.tiny_v2.f32.nomask"] = v2_forward_fixed(dv2, model_v2, x, ctx, None, ts)

        # ---- schedule tables (pipeline.py:239-257) ----
        sched = {}
        for (hh, ww) in [(256, 256), (1024, 1024), (896, 1344), (128, 128)]:
            for n in (4, 30):
                lh, lw = hh // 8, ww // 8
                alpha = 2 * math.sqrt(lh * lw / (64 * 64))
                rows = []
                for i in range(n, 0, -1):
                    t = i / n
                    tn = (i - 1) / n
                    t = t * alpha / (1 + (alpha - 1) * t)
                    tn = tn * alpha / (1 + (alpha - 1) * tn)
                    rows.append([t, t - tn])
                sched[f"{hh}x{ww}.{n}"] = rows
        meta["schedule"] = sched

        # ---- full pipeline __call__ (tiny v1), 4 steps, 128x128 image (16x16 latent) ----
        lat = torch.randn(1, 16, 16, 16, generator=g)
        pos = torch.randn(1, 24, 128, generator=g)
        neg = torch.zeros_like(pos)
        T["pipe.in.latents"] = lat
        T["pipe.in.pos"] = pos
        T["pipe.f32.cfg6"] = run_pipeline(pipeline, dit32, lat, pos, neg, 4, 6.0, False, 128, 128)
        T["pipe.f32.cfg1"] = run_pipeline(pipeline, dit32, lat, pos, neg, 4, 1.0, False, 128, 128)
        T["pipe.f32.apg"] = run_pipeline(pipeline, dit32, lat, pos, neg, 4, 6.0, True, 128, 128)
        T["pipe.f32.nocfg"] = run_pipeline(pipeline, dit32, lat, pos, neg, 4, 0.5, False, 128, 128)
        T["pipe.bf16.cfg6"] = run_pipeline(pipeline, dit16, lat.bfloat16(), pos.bfloat16(), neg.bfloat16(), 4, 6.0,
                                           False, 128, 128).float()

    T = {k: v.contiguous().float() if v.is_floating_point() else v.contiguous() for k, v in T.items()}
    save_file(T, str(OUT / "golden.safetensors"))
    (OUT / "golden_meta.json").write_text(json.dumps(meta, indent=1))
    print("wrote", len(T), "tensors;", sum(v.numel() for v in T.values()) * 4 / 1e6, "MB")


if __name__ == "__main__":
    main()
