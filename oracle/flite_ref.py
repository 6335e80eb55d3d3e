"""TEST INFRASTRUCTURE ONLY. CPU restatement of the F-Lite DiT forward and sampling loop.

Follows, op by op, the reference at /root/reference (sippycoder/f-lite):
  - DiT.forward                     f_lite/model.py:525-591   (v1 layout: shared adaLN, cross-attn on
                                                              blocks idx < 8 or idx % 4 == 0, model.py:464)
  - DiT.forward (v2 layout)         f_lite/model_v2.py:528-594 (per-block adaLN, cross-attn everywhere) with
                                    the final stage taken from model.py:578-580 (the v2 file
                                    applies final_modulation to the per-token t_emb and cannot run)
  - DiTBlock.forward                f_lite/model.py:270-303
  - Attention.forward               f_lite/model.py:160-213
  - FLitePipeline.__call__ loop     f_lite/pipeline.py:250-297 (+ decode scaling 301-304, post-process 324-327)
and the third-party ops the reference calls, restated from their published semantics:
  - LigerRMSNorm (casting_mode "llama"): fp32 normalise, cast to input dtype, multiply by the weight
  - LigerSwiGLUMLP: down(cast(silu(fp32(gate(x)))) * up(x))
  - flash_attn_varlen_func: per-segment softmax(q k^T * scale) v with fp32 accumulation
The same code runs in fp32 (the parity oracle) or bf16 (the reference's own rounding points).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.nn.functional as F

from .weights import make_state_dict, param_shapes

EPS = 1e-6


def timestep_embedding(t: torch.Tensor, dim: int, max_period: float = 10000) -> torch.Tensor:
    """model.py:20-28"""
    half = dim // 2
    freqs = torch.exp(-math.log(max_period) * torch.arange(start=0, end=half, dtype=torch.float32) / half)
    args = t[:, None].float() * freqs[None]
    return torch.cat([torch.cos(args), torch.sin(args)], dim=-1)


def liger_rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float = EPS) -> torch.Tensor:
    xf = x.float()
    r = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return w * (xf * r).to(x.dtype)


def own_rmsnorm(x: torch.Tensor, w: Optional[torch.Tensor], eps: float = EPS) -> torch.Tensor:
    """model.py:101-108 (all fp32, single cast)."""
    dt = x.dtype
    xf = x.float()
    n = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    if w is not None:
        return (xf * n * w).to(dtype=dt)
    return (xf * n).to(dtype=dt)


def rope_tables(h: int, w: int, dim: int = 128, base: float = 10000.0, n_reg: int = 16, dtype=torch.float32):
    """TwoDimRotary (model.py:334-386) sliced to (h, w) with n_reg leading (cos=1, sin=0) rows.
    In a bf16 model the buffers are cast to bf16 by .to(dtype)."""
    inv_freq = torch.FloatTensor([1.0 / (base ** (i / dim)) for i in range(0, dim, 2)])
    t_h = torch.arange(h, dtype=torch.float32)
    t_w = torch.arange(w, dtype=torch.float32)
    fh = torch.outer(t_h, inv_freq).unsqueeze(1).repeat(1, w, 1)
    fw = torch.outer(t_w, inv_freq).unsqueeze(0).repeat(h, 1, 1)
    f = torch.cat([fh, fw], 2)
    cos = f.cos().to(dtype).reshape(h * w, -1)
    sin = f.sin().to(dtype).reshape(h * w, -1)
    cos = torch.cat([torch.ones(n_reg, cos.shape[1], dtype=dtype), cos], 0)
    sin = torch.cat([torch.zeros(n_reg, sin.shape[1], dtype=dtype), sin], 0)
    return cos, sin


def apply_rotary_emb(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """model.py:403-414 (rotation by -theta on rotate-half pairs, fp32 math)."""
    od = x.dtype
    x = x.float()
    cos = cos.float()
    sin = sin.float()
    d = x.shape[-1] // 2
    x1, x2 = x[..., :d], x[..., d:]
    return torch.cat([x1 * cos + x2 * sin, x1 * (-sin) + x2 * cos], -1).to(od)


# --------------------------------------------------------------------------------------------------
# MXFP8 fake-quant (the fp8 configuration, BASELINE.json configs[4]; no reference counterpart: the reference runs
# bf16 only). Restates include/flite.h / f-lite_amd/csrc/fp8.hip bit for bit: OCP e4m3fn elements, one E8M0 scale
# per 32 consecutive elements of the last dim, e = ceil(log2(amax * (1/448))) from the fp32 bits, clamped to
# [-127, 126]; element = RNE(clamp(x * 2^-e, +-448)).
# --------------------------------------------------------------------------------------------------
def _mx_exp(xb: torch.Tensor) -> torch.Tensor:
    amax = xb.abs().amax(-1, keepdim=True)
    a = (amax * torch.tensor(1.0 / 448.0, dtype=torch.float32)).contiguous()
    bits = a.view(torch.int32)
    e = ((bits >> 23) & 0xFF) - 127 + ((bits & 0x7FFFFF) != 0).to(torch.int32)
    return e.clamp(-127, 126)


def mx_quant(x: torch.Tensor, block: int = 32) -> torch.Tensor:
    """MXFP8 quantise-dequantise along the last dim; returns fp32 (the values the fp8 GEMM multiplies)."""
    shp = x.shape
    xb = x.float().reshape(*shp[:-1], shp[-1] // block, block)
    e = _mx_exp(xb)
    one = torch.ones((), dtype=torch.float32)
    q = (xb * torch.ldexp(one, -e)).clamp(-448.0, 448.0).to(torch.float8_e4m3fn).float()
    return (q * torch.ldexp(one, e)).reshape(shp)


def mx_quant_bytes(x: torch.Tensor, rows_pad: Optional[int] = None):
    """(e4m3 bytes uint8 [rows, K], scales uint8 [K/128, rows_pad, 4]) as flite_quant_fp8_rows writes them."""
    rows, K = x.shape
    xb = x.float().reshape(rows, K // 32, 32)
    e = _mx_exp(xb)
    one = torch.ones((), dtype=torch.float32)
    q = (xb * torch.ldexp(one, -e)).clamp(-448.0, 448.0).to(torch.float8_e4m3fn).view(torch.uint8)
    rp = rows_pad or (rows + 255) // 256 * 256
    sc = torch.zeros(K // 128, rp, 4, dtype=torch.uint8)
    sc[:, :rows, :] = (e[..., 0] + 127).to(torch.uint8).reshape(rows, K // 128, 4).permute(1, 0, 2)
    return q.reshape(rows, K), sc


def attention_varlen(q, k, v, cu_q, cu_k, scale):
    """flash_attn_varlen_func: q [Lq, h, d], k/v [Lk, h, d]; fp32 softmax, output in q.dtype."""
    out = torch.empty_like(q)
    for b in range(len(cu_q) - 1):
        qs, qe = int(cu_q[b]), int(cu_q[b + 1])
        ks, ke = int(cu_k[b]), int(cu_k[b + 1])
        qq = q[qs:qe].float().transpose(0, 1)
        kk = k[ks:ke].float().transpose(0, 1)
        vv = v[ks:ke].float().transpose(0, 1)
        if ke == ks:
            out[qs:qe] = 0
            continue
        s = torch.matmul(qq, kk.transpose(1, 2)) * scale
        p = torch.softmax(s, dim=-1)
        out[qs:qe] = torch.matmul(p, vv).transpose(0, 1).to(q.dtype)
    return out


def prepare_varlen(hidden: torch.Tensor, mask: Optional[torch.Tensor] = None):
    """prepare_flash_attention_inputs (model.py:31-64)."""
    b, l, d = hidden.shape
    if mask is None:
        mask = torch.ones(b, l)
    lens = mask.sum(dim=-1, dtype=torch.int32)
    cu = torch.cat([torch.zeros(1, dtype=torch.int32), lens.cumsum(0, dtype=torch.int32)])
    idx = torch.nonzero(mask.reshape(-1), as_tuple=True)[0]
    return hidden.reshape(-1, d).index_select(0, idx), cu, l, idx


@dataclass
class DiTConfig:
    in_channels: int = 16
    patch_size: int = 2
    hidden_size: int = 3072
    depth: int = 40
    num_heads: int = 12
    mlp_ratio: float = 4.0
    cross_attn_input_size: int = 4096
    train_bias_and_rms: bool = True
    rope_base: float = 10000.0
    per_block_adaln: bool = False  # model_v2.py layout
    use_rope: bool = True  # False: learned positional_embedding (model.py:444,546), no RoPE

    def as_dict(self):
        return dict(self.__dict__)

    def cross(self, i: int) -> bool:
        return True if self.per_block_adaln else (i % 4 == 0 or i < 8)


PRESETS = {
    # SURVEY §8d "Model definitions"
    "7b": DiTConfig(),
    "10b": DiTConfig(per_block_adaln=True),
    # small configs used by the golden fixtures (head_dim 256 like the real model)
    "tiny": DiTConfig(hidden_size=512, depth=10, num_heads=2, cross_attn_input_size=128),
    "tiny_v2": DiTConfig(hidden_size=512, depth=3, num_heads=2, cross_attn_input_size=128, per_block_adaln=True),
}


class RefDiT:
    """Functional restatement of DiT.forward; params is a state dict (fp32 values), cast to `dtype`."""

    # block GEMM weights that the fp8 configuration runs in MXFP8 (f-lite_amd/csrc/dit.cpp: run_block_fp8)
    FP8_WEIGHTS = ("self_attn.qkv", "self_attn.proj", "cross_attn.q", "cross_attn.proj", "mlp.gate_proj",
                   "mlp.up_proj", "mlp.down_proj")

    def __init__(self, cfg: DiTConfig, params: dict, dtype=torch.float32, rope_dtype=None, fp8: bool = False):
        self.cfg = cfg
        self.dtype = dtype
        self.p = {k: v.to(dtype) for k, v in params.items()}
        self.rope_dtype = rope_dtype if rope_dtype is not None else dtype
        # fp8: fake-quantised (MXFP8) block GEMM weights and the activations feeding them
        self.fp8 = fp8
        if fp8:
            for k in list(self.p):
                if k.startswith("blocks.") and k.endswith(".weight") and \
                        any(("." + n + ".") in k for n in self.FP8_WEIGHTS):
                    self.p[k] = mx_quant(self.p[k]).to(dtype)

    def _q8(self, a, round_bf16=False):
        """fp8 mode: the MXFP8 operand an activation becomes (attention outputs are bf16 tensors first)."""
        if not self.fp8:
            return a
        if round_bf16:
            a = a.to(torch.bfloat16)
        return mx_quant(a).to(self.dtype)

    @classmethod
    def random(cls, cfg: DiTConfig, seed: int = 0, dtype=torch.float32, **kw):
        return cls(cfg, make_state_dict(cfg.as_dict(), seed=seed), dtype=dtype, **kw)

    def _lin(self, x, name, bias=True):
        b = self.p.get(name + ".bias") if bias else None
        return F.linear(x, self.p[name + ".weight"], b)

    def block(self, i, x, cu, maxl, ctx, ctx_cu, mod, cos, sin):
        c = self.cfg
        pre = f"blocks.{i}."
        H = c.num_heads
        (shift_sa, scale_sa, gate_sa, shift_ca, scale_ca, gate_ca, shift_mlp, scale_mlp, gate_mlp) = mod
        n = liger_rmsnorm(x, self.p[pre + "norm1.weight"])
        n = self._q8(n * (1 + scale_sa) + shift_sa)
        qkv = self._lin(n, pre + "self_attn.qkv")
        L = qkv.shape[0]
        qkv = qkv.reshape(L, 3, H, -1).permute(1, 2, 0, 3)  # "l (k h d) -> k h l d"
        q, k, v = qkv.unbind(0)
        if cos is not None:  # use_rope (model.py:166-167 applies RoPE only when given)
            q = apply_rotary_emb(q, cos, sin)
            k = apply_rotary_emb(k, cos, sin)
        q = own_rmsnorm(q, None)
        k = own_rmsnorm(k, None)
        q, k, v = (t.transpose(0, 1) for t in (q, k, v))  # "h l d -> l h d"
        hd = q.shape[-1]
        a = self._q8(attention_varlen(q, k, v, cu, cu, hd ** -0.5).reshape(L, -1), round_bf16=True)
        x = x + self._lin(a, pre + "self_attn.proj", bias=False) * gate_sa
        if c.cross(i):
            n = liger_rmsnorm(x, self.p[pre + "norm2.weight"])
            n = self._q8(n * (1 + scale_ca) + shift_ca)
            q = self._lin(n, pre + "cross_attn.q").reshape(L, H, -1)
            kv = self._lin(ctx, pre + "cross_attn.context_kv")
            kv = kv.reshape(kv.shape[0], 2, H, -1).permute(1, 0, 2, 3)  # "l (k h d) -> k l h d"
            kk, vv = kv.unbind(0)
            q = own_rmsnorm(q, None)
            kk = own_rmsnorm(kk, None)
            a = self._q8(attention_varlen(q, kk, vv, cu, ctx_cu, hd ** -0.5).reshape(L, -1), round_bf16=True)
            x = x + self._lin(a, pre + "cross_attn.proj", bias=False) * gate_ca
        n = liger_rmsnorm(x, self.p[pre + "norm3.weight"])
        n = self._q8(n * (1 + scale_mlp) + shift_mlp)
        g = self._lin(n, pre + "mlp.gate_proj", bias=False)
        u = self._lin(n, pre + "mlp.up_proj", bias=False)
        hmid = self._q8(F.silu(g.float()).to(u.dtype) * u)
        x = x + self._lin(hmid, pre + "mlp.down_proj", bias=False) * gate_mlp
        return x

    def t_embed(self, timesteps):
        """model.py:551-552: timestep_embedding(timesteps * 1000) (in the timesteps' dtype), cast, MLP."""
        D = self.cfg.hidden_size
        te = timestep_embedding(timesteps * 1000, D).to(self.dtype)
        h = F.silu(self._lin(te, "time_embed.0"))
        return self._lin(h, "time_embed.2")

    def forward(self, x, context, context_attn_mask, timesteps, return_hidden=False):
        c = self.cfg
        D = c.hidden_size
        p = c.patch_size
        x = x.to(self.dtype)
        context = context.to(self.dtype)
        context = self._lin(context, "context_proj")
        context = liger_rmsnorm(context, self.p["context_norm.weight"])
        ctx_flat, ctx_cu, _, _ = prepare_varlen(context, context_attn_mask)
        b, _, h, w = x.shape
        xe = F.conv2d(x, self.p["patch_embed.patch_proj.weight"], self.p["patch_embed.patch_proj.bias"], stride=p)
        xe = xe.flatten(2).transpose(1, 2)  # "b c h w -> b (h w) c"
        xe = torch.cat([self.p["register_tokens"].repeat(b, 1, 1), xe], 1)
        T = xe.shape[1]
        if c.use_rope:  # model.py:537-544
            cos, sin = rope_tables(h // p, w // p, D // (2 * c.num_heads), c.rope_base, 16, self.rope_dtype)
            cos = cos[None].repeat(1, b, 1)
            sin = sin[None].repeat(1, b, 1)
        else:  # model.py:546
            xe = xe + self.p["positional_embedding"].repeat(b, 1, 1)[:, :T, :]
            cos, sin = None, None
        x_flat, cu, maxl, idx = prepare_varlen(xe)
        t_emb = self.t_embed(timesteps)
        st = F.silu(t_emb)
        if not c.per_block_adaln:
            mod_all = F.linear(st, self.p["adaLN_modulation.1.weight"], self.p["adaLN_modulation.1.bias"])
            mod = mod_all.repeat_interleave(T, dim=0).chunk(9, dim=1)
        for i in range(c.depth):
            if c.per_block_adaln:
                mi = F.linear(st, self.p[f"blocks.{i}.adaLN_modulation.1.weight"],
                              self.p[f"blocks.{i}.adaLN_modulation.1.bias"])
                mod = mi.repeat_interleave(T, dim=0).chunk(9, dim=1)
            x_flat = self.block(i, x_flat, cu, maxl, ctx_flat, ctx_cu, mod, cos, sin)
        xo = x_flat.reshape(b, T, D)[:, 16:, :]
        fm = F.linear(st, self.p["final_modulation.1.weight"], self.p["final_modulation.1.bias"])
        shift, scale = fm.chunk(2, dim=1)
        xo = own_rmsnorm(xo, self.p.get("final_norm.weight"))
        xo = xo * (1 + scale[:, None, :]) + shift[:, None, :]
        xo = self._lin(xo, "final_proj")
        hp, wp = h // p, w // p
        C = c.in_channels
        xo = xo.reshape(b, hp, wp, p, p, C).permute(0, 5, 1, 3, 2, 4).reshape(b, C, h, w)
        return xo

    __call__ = forward


# --------------------------------------------------------------------------------------------------
# Sampling loop (pipeline.py:187-331)
# --------------------------------------------------------------------------------------------------
def schedule(num_steps: int, height: int, width: int, alpha: Optional[float] = None, vae_scale: int = 8):
    """(t, dt) per step, python float64 like the reference (pipeline.py:239-257)."""
    lh, lw = height // vae_scale, width // vae_scale
    if alpha is None:
        alpha = 2 * math.sqrt(lh * lw / (64 * 64))
    out = []
    for i in range(num_steps, 0, -1):
        t = i / num_steps
        tn = (i - 1) / num_steps
        t = t * alpha / (1 + (alpha - 1) * t)
        tn = tn * alpha / (1 + (alpha - 1) * tn)
        out.append((t, t - tn))
    return out


@dataclass
class APG:
    enabled: bool = True
    orthogonal_threshold: float = 0.03


def sample(dit, latents, prompt_embeds, negative_embeds, num_steps=30, guidance_scale=6.0, alpha=None,
           apg: Optional[APG] = None, t_dtype=None, acc_dtype=None, height=None, width=None, trace=None,
           max_steps=None):
    """The denoise loop of FLitePipeline.__call__ (pipeline.py:245-297). Returns the final latents.

    t_dtype: dtype of the timestep tensor (pipeline.py:260 uses the model dtype: bf16 in a bf16 model).
    acc_dtype: dtype of the Euler accumulator (reference: the model dtype).
    max_steps: stop after this many steps of the num_steps schedule (timing samples only).
    """
    B = latents.shape[0]
    lh, lw = latents.shape[-2:]
    height = height or lh * 8
    width = width or lw * 8
    t_dtype = t_dtype or latents.dtype
    acc_dtype = acc_dtype or latents.dtype
    acc = latents.clone().to(acc_dtype)
    lat = acc.clone()
    cfg = guidance_scale >= 1.0
    apg = apg or APG(enabled=False)
    for step, (t, dt) in enumerate(schedule(num_steps, height, width, alpha)):
        if max_steps is not None and step >= max_steps:
            break
        tt = torch.tensor([t] * B, dtype=t_dtype)
        if cfg:
            out = dit(torch.cat([lat] * 2), torch.cat([negative_embeds, prompt_embeds]), None, torch.cat([tt] * 2))
            u, c = out.chunk(2)
            if apg.enabled:
                dy = c
                dd = c - u
                par = (dy * dd).sum() / (dy * dy).sum() * dy
                orth = dd - par
                s = min(1, apg.orthogonal_threshold / orth.std())
                mo = dy + (guidance_scale - 1) * orth * s
            else:
                mo = u + guidance_scale * (c - u)
        else:
            mo = dit(lat, prompt_embeds, None, tt)
        if trace is not None:
            trace.append(mo.detach().clone())
        acc = acc + dt * mo.to(acc_dtype)
        lat = acc.clone().to(latents.dtype) if acc_dtype != latents.dtype else acc.clone()
    return lat


def postprocess(decoded: torch.Tensor) -> torch.Tensor:
    """pipeline.py:324-326 -> uint8 [B, 3, H, W]."""
    images = (decoded / 2 + 0.5).clamp(0, 1)
    return (images * 255).round().clamp(0, 255).to(torch.uint8)


def psnr(a: torch.Tensor, ref: torch.Tensor, peak: Optional[float] = None) -> float:
    a = a.double()
    ref = ref.double()
    mse = (a - ref).pow(2).mean().item()
    peak = peak if peak is not None else ref.abs().max().item()
    if mse == 0:
        return float("inf")
    return 10 * math.log10(peak * peak / mse)
