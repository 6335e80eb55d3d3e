"""DiT with cross attention -- the F-Lite denoiser, MI355X-native.

Drop-in for the reference `f_lite.model.DiT` (/root/reference/f_lite/model.py:417-591): same constructor
keyword arguments and defaults (model.py:419-433), same submodule tree and state-dict keys, a `config`
captured like diffusers' register_to_config, `from_pretrained`/`save_pretrained` for a local diffusers-layout
folder, and a forward that accepts both the 4-argument form `(x, context, context_attn_mask, timesteps)`
(model.py:526, train.py:471) and the 3-argument form `(x, context, timesteps)` the reference pipeline uses
(pipeline.py:271,293).

The modules below only HOLD parameters. `forward` never runs a PyTorch op on them: it binds the parameter
storage to the native engine (libflite_hip.so, include/flite.h) and launches the gfx950 kernels. There is no
CPU path: a model on the CPU raises.
"""
from __future__ import annotations

import json
import math
import os
from pathlib import Path
from types import SimpleNamespace
from typing import Optional

import torch
from torch import nn

from . import _native

N_REGISTERS = 16


class RMSNorm(nn.Module):
    """Parameter holder for LigerRMSNorm (model.py:238,248,260,437) and RMSNorm (model.py:92-112)."""

    def __init__(self, dim, eps=1e-6, trainable=True):
        super().__init__()
        self.eps = eps
        if trainable:
            self.weight = nn.Parameter(torch.ones(dim))
        else:
            self.weight = None


class QKNorm(nn.Module):
    """model.py:115-130 (no parameters: trainable=False)."""

    def __init__(self, dim):
        super().__init__()
        self.query_norm = RMSNorm(dim, trainable=False)
        self.key_norm = RMSNorm(dim, trainable=False)


class Attention(nn.Module):
    """model.py:133-158 (self: qkv + proj; cross: q + context_kv + proj)."""

    def __init__(self, dim, num_heads=8, qkv_bias=False, is_self_attn=True, dynamic_softmax_temperature=False):
        super().__init__()
        assert dim % num_heads == 0
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.scale = self.head_dim ** -0.5
        self.is_self_attn = is_self_attn
        self.dynamic_softmax_temperature = dynamic_softmax_temperature
        if is_self_attn:
            self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        else:
            self.q = nn.Linear(dim, dim, bias=qkv_bias)
            self.context_kv = nn.Linear(dim, dim * 2, bias=qkv_bias)
        self.proj = nn.Linear(dim, dim, bias=False)
        self.qk_norm = QKNorm(self.head_dim)


class SwiGLUMLP(nn.Module):
    """LigerSwiGLUMLP parameter layout (gate_proj / up_proj / down_proj, no biases)."""

    def __init__(self, hidden_size, intermediate_size):
        super().__init__()
        self.gate_proj = nn.Linear(hidden_size, intermediate_size, bias=False)
        self.up_proj = nn.Linear(hidden_size, intermediate_size, bias=False)
        self.down_proj = nn.Linear(intermediate_size, hidden_size, bias=False)


class DiTBlock(nn.Module):
    """model.py:226-267 (per_block_adaln adds the model_v2.py:269-271 adaLN_modulation)."""

    def __init__(self, hidden_size, num_heads, do_cross_attn=False, mlp_ratio=4.0, qkv_bias=True,
                 dynamic_softmax_temperature=False, per_block_adaln=False):
        super().__init__()
        self.hidden_size = hidden_size
        self.norm1 = RMSNorm(hidden_size)
        self.self_attn = Attention(hidden_size, num_heads=num_heads, qkv_bias=qkv_bias, is_self_attn=True,
                                   dynamic_softmax_temperature=dynamic_softmax_temperature)
        if do_cross_attn:
            self.norm2 = RMSNorm(hidden_size)
            self.cross_attn = Attention(hidden_size, num_heads=num_heads, qkv_bias=qkv_bias, is_self_attn=False,
                                        dynamic_softmax_temperature=dynamic_softmax_temperature)
        else:
            self.norm2 = None
            self.cross_attn = None
        self.norm3 = RMSNorm(hidden_size)
        self.mlp = SwiGLUMLP(hidden_size, int(hidden_size * mlp_ratio))
        if per_block_adaln:
            self.adaLN_modulation = nn.Sequential(nn.SiLU(), nn.Linear(hidden_size, 9 * hidden_size, bias=True))
            self.adaLN_modulation[-1].weight.data.zero_()
            self.adaLN_modulation[-1].bias.data.zero_()


class PatchEmbed(nn.Module):
    """model.py:318-331"""

    def __init__(self, patch_size=16, in_channels=3, embed_dim=768):
        super().__init__()
        self.patch_proj = nn.Conv2d(in_channels, embed_dim, kernel_size=patch_size, stride=patch_size)
        self.patch_size = patch_size


_CONFIG_KEYS = ("in_channels", "patch_size", "hidden_size", "depth", "num_heads", "mlp_ratio",
                "cross_attn_input_size", "train_bias_and_rms", "use_rope", "gradient_checkpoint",
                "dynamic_softmax_temperature", "rope_base")


class DiT(nn.Module):
    """F-Lite DiT (model.py:417-591). `per_block_adaln=True` selects the model_v2.py layout (10B)."""

    _per_block_adaln_default = False

    def __init__(self, in_channels=4, patch_size=2, hidden_size=1152, depth=28, num_heads=16, mlp_ratio=4.0,
                 cross_attn_input_size=128, train_bias_and_rms=True, use_rope=True, gradient_checkpoint=False,
                 dynamic_softmax_temperature=False, rope_base=10000, per_block_adaln=None):
        super().__init__()
        if per_block_adaln is None:
            per_block_adaln = self._per_block_adaln_default
        cfg = dict(in_channels=in_channels, patch_size=patch_size, hidden_size=hidden_size, depth=depth,
                   num_heads=num_heads, mlp_ratio=mlp_ratio, cross_attn_input_size=cross_attn_input_size,
                   train_bias_and_rms=train_bias_and_rms, use_rope=use_rope, gradient_checkpoint=gradient_checkpoint,
                   dynamic_softmax_temperature=dynamic_softmax_temperature, rope_base=rope_base)
        self.config = SimpleNamespace(**cfg)
        self.per_block_adaln = bool(per_block_adaln)

        self.context_proj = nn.Linear(cross_attn_input_size, hidden_size)
        self.context_norm = RMSNorm(hidden_size)
        self.patch_embed = PatchEmbed(patch_size, in_channels, hidden_size)
        if not use_rope:
            self.positional_embedding = nn.Parameter(torch.zeros(1, 2048, hidden_size))
        self.register_tokens = nn.Parameter(torch.randn(1, N_REGISTERS, hidden_size))
        self.time_embed = nn.Sequential(nn.Linear(hidden_size, 4 * hidden_size), nn.SiLU(),
                                        nn.Linear(4 * hidden_size, hidden_size))
        if not self.per_block_adaln:
            self.adaLN_modulation = nn.Sequential(nn.SiLU(), nn.Linear(hidden_size, 9 * hidden_size, bias=True))
            self.adaLN_modulation[-1].weight.data.zero_()
            self.adaLN_modulation[-1].bias.data.zero_()
        self.blocks = nn.ModuleList([
            DiTBlock(hidden_size=hidden_size, num_heads=num_heads, mlp_ratio=mlp_ratio,
                     do_cross_attn=True if self.per_block_adaln else (idx % 4 == 0 or idx < 8),  # model.py:464
                     qkv_bias=train_bias_and_rms, dynamic_softmax_temperature=dynamic_softmax_temperature,
                     per_block_adaln=self.per_block_adaln)
            for idx in range(depth)
        ])
        self.final_modulation = nn.Sequential(nn.SiLU(), nn.Linear(hidden_size, 2 * hidden_size, bias=True))
        self.final_norm = RMSNorm(hidden_size, trainable=train_bias_and_rms)
        self.final_proj = nn.Linear(hidden_size, patch_size * patch_size * in_channels)
        nn.init.zeros_(self.final_modulation[-1].weight)
        nn.init.zeros_(self.final_modulation[-1].bias)
        nn.init.zeros_(self.final_proj.weight)
        nn.init.zeros_(self.final_proj.bias)
        self._engine = None
        self._bound = None
        self._fp8 = False
        self._resid16 = None  # residual-stream storage: None = the engine default, else bool (set_residual_dtype)
        self._wgen = 0

    # ------------------------------------------------------------------ construction helpers
    @classmethod
    def empty(cls, device="cuda", dtype=torch.bfloat16, **cfg):
        """Allocate without initialisation (meta construction, then storage on `device`)."""
        with torch.device("meta"):
            m = cls(**cfg)
        m = m.to_empty(device=device)
        return m.to(dtype)

    @classmethod
    def random(cls, seed=0, std=0.02, device="cuda", dtype=torch.bfloat16, **cfg):
        """Seeded synthetic weights on the device (SURVEY §8d init recipe): every matrix/bias/register token
        uniform with std `std`, norm weights 1 -- bit-identical to oracle/weights.py."""
        m = cls.empty(device=device, dtype=dtype, **cfg)
        m.random_init_(seed, std)
        return m

    @torch.no_grad()
    def random_init_(self, seed=0, std=0.02):
        for name, p in self.named_parameters():
            _native.init_param_(p.data, name, seed=seed, std=std, ones=_is_norm_weight(name))
        torch.cuda.synchronize()
        self._wgen += 1  # written through raw pointers: no version bump
        return self

    def weights_updated(self):
        """Declare that parameters were written behind autograd's version counters -- through `p.data` (a
        `p.data.copy_(...)` gets a fresh counter) or through raw device pointers: the engine re-derives its copies
        (MXFP8 weights, the cross-attention K/V cache) before its next run. Writes through the parameters
        themselves (load_state_dict, `p.copy_` under no_grad) are seen without this call."""
        self._wgen += 1
        return self

    @property
    def dtype(self):
        return next(self.parameters()).dtype

    @property
    def device(self):
        return next(self.parameters()).device

    # ------------------------------------------------------------------ diffusers-folder IO
    def config_dict(self):
        """config.json as register_to_config writes it (model.py:418-433): the constructor kwargs only. The
        layout (model.py vs model_v2.py) is not a config key: model_index.json's module names it."""
        d = {k: getattr(self.config, k) for k in _CONFIG_KEYS}
        d["_class_name"] = "DiT"
        return d

    @property
    def module_name(self) -> str:
        """The reference module of this layout, as model_index.json records it (generate.py:65)."""
        return "f_lite.model_v2" if self.per_block_adaln else "f_lite.model"

    def save_pretrained(self, save_directory):
        from safetensors.torch import save_file

        p = Path(save_directory)
        p.mkdir(parents=True, exist_ok=True)
        (p / "config.json").write_text(json.dumps(self.config_dict(), indent=2))
        sd = {k: v.detach().contiguous().cpu() for k, v in self.state_dict().items()}
        save_file(sd, str(p / "diffusion_pytorch_model.safetensors"))

    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path, subfolder=None, torch_dtype=torch.bfloat16,
                        device="cuda", **kwargs):
        """Local diffusers-layout folder: config.json + diffusion_pytorch_model*.safetensors (optionally
        sharded with an index). Hub names cannot be resolved offline."""
        from safetensors.torch import load_file

        p = Path(pretrained_model_name_or_path)
        if subfolder:
            p = p / subfolder
        if not (p / "config.json").exists():
            raise FileNotFoundError(f"{p}/config.json not found (only local diffusers-layout folders are supported)")
        cfg = json.loads((p / "config.json").read_text())
        cfg = {k: v for k, v in cfg.items() if not k.startswith("_") and k in _CONFIG_KEYS + ("per_block_adaln",)}
        files = sorted(p.glob("diffusion_pytorch_model*.safetensors"))
        if not files:
            raise FileNotFoundError(f"no diffusion_pytorch_model*.safetensors in {p}")
        sd = {}
        for f in files:
            sd.update(load_file(str(f)))
        return cls.from_state_dict(clean_state_dict(sd), device=device, torch_dtype=torch_dtype, **cfg)

    # ------------------------------------------------------------------ LoRA (model.py:487-495; f_lite/lora.py)
    def load_lora_weights(self, load_directory, target_modules=None):
        """`<load_directory>/lora_weights.pt` (a peft LoRA state dict, read with weights_only=True) folded into
        the weights: W <- W + B @ A (the adapter's lora_alpha / r = 1 as pt.py:116-121 configures it)."""
        from .lora import merge_lora_

        sd = torch.load(str(Path(load_directory) / "lora_weights.pt"), map_location="cpu", weights_only=True)
        return merge_lora_(self, sd, scaling=1.0, target_modules=target_modules)

    def save_lora_weights(self, save_directory):
        """`<save_directory>/lora_weights.pt`: the adapters merged by load_lora_weights / load_f_lite_pt, latest per
        module (what get_peft_model_state_dict returns for peft's one adapter, model.py:487-490)."""
        from .lora import merged_state_dict

        sd = merged_state_dict(self)
        if not sd:
            raise RuntimeError("no LoRA adapter has been loaded into this model")
        torch.save(sd, f"{save_directory}/lora_weights.pt")

    @classmethod
    def from_state_dict(cls, sd, device="cuda", torch_dtype=torch.bfloat16, **cfg):
        """Build on `device` in `torch_dtype` and load `sd` strictly. A per-block-adaLN state dict given to the
        model.py class (or the reverse) is refused with the class to use instead."""
        m = cls.empty(device=device, dtype=torch_dtype, **cfg)
        v2_keys = any(k.startswith("blocks.") and ".adaLN_modulation." in k for k in sd)
        if v2_keys != m.per_block_adaln:
            want = "f_lite.model_v2.DiT" if v2_keys else "f_lite.model.DiT"
            raise ValueError(f"state dict is the {'model_v2' if v2_keys else 'model'}.py layout: load it with {want} "
                             "(model_index.json dit_model module)")
        m.load_state_dict(sd, strict=True)
        return m

    # ------------------------------------------------------------------ native engine
    def _native_config(self):
        c = self.config
        cfg = _native.DitConfig()
        cfg.in_channels = c.in_channels
        cfg.patch_size = c.patch_size
        cfg.hidden_size = c.hidden_size
        cfg.depth = c.depth
        cfg.num_heads = c.num_heads
        cfg.mlp_hidden = int(c.hidden_size * c.mlp_ratio)
        cfg.cross_attn_input_size = c.cross_attn_input_size
        cfg.train_bias_and_rms = int(bool(c.train_bias_and_rms))
        cfg.per_block_adaln = int(self.per_block_adaln)
        cfg.n_register_tokens = N_REGISTERS
        cfg.rope_base = float(c.rope_base)
        cfg.bf16_timestep_quant = int(self.dtype == torch.bfloat16)
        cfg.bf16_rope_tables = int(self.dtype == torch.bfloat16)
        cfg.use_rope = int(bool(c.use_rope))
        return cfg

    def engine(self) -> _native.DitEngine:
        """The native engine with every parameter bound (re-binds when parameter storage moved)."""
        params = list(self.named_parameters())
        if not params[0][1].is_cuda:
            raise _native.FliteError("DiT parameters are on the CPU: the F-Lite path runs only on a ROCm device "
                                     "(move the model with .to('cuda', torch.bfloat16)); there is no CPU fallback")
        if self.dtype != torch.bfloat16:
            raise _native.FliteError("the native DiT path computes with bf16 parameters; call .to(torch.bfloat16)")
        # storage (pointers) and contents: an in-place update (load_state_dict's copy_, random_init_) bumps the
        # version, and the engine's derived copies (fp8 weights) are remade from the new values
        ptrs = tuple((n, p.data_ptr()) for n, p in params)
        vers = (self._wgen,) + tuple(p._version for _, p in params)
        if self._engine is None:
            self._engine = _native.DitEngine(self._native_config())
            self._bound = None
            if self._resid16 is not None:
                self._engine.set_residual_bf16(self._resid16)
        if self._bound is None or self._bound[0] != ptrs:
            for n, p in params:
                self._engine.bind(n, p.data)  # new storage: the engine requantises before its next run
        elif self._bound[1] != vers:
            self._engine.weights_updated(self.device)
        self._bound = (ptrs, vers)
        return self._engine

    def set_residual_dtype(self, dtype=torch.bfloat16):
        """Storage of the blocks' residual stream x (model.py:289,297,301): torch.bfloat16 (the default since round 6:
        the reference's own storage, each update still one fp32 fma rounded once) or torch.float32 (every update and
        the stream in fp32: 1.5-3 dB closer to the reference's fp32 run, 1.5 % slower). include/flite.h
        flite_dit_set_residual_bf16."""
        if dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("residual dtype must be torch.float32 or torch.bfloat16")
        self._resid16 = dtype == torch.bfloat16
        if self._engine is not None:
            self._engine.set_residual_bf16(self._resid16)
        return self

    def enable_fp8(self, enabled: bool = True, bf16_blocks=(), gemm_classes=None, block_classes=None):
        """BASELINE.json configs[4]: run every block GEMM (qkv, proj, cross q / proj, SwiGLU gate-up, down) on
        MXFP8 weights and activations (OCP e4m3, E8M0 scale per 32 K elements) on the gfx950 block-scaled MFMA.
        The bf16 parameters stay the source of truth; the engine quantises them once. Precision policies (DESIGN §5
        prices each): `bf16_blocks`, block indices that keep their bf16 GEMMs (e.g. (0, depth - 1)); `gemm_classes`,
        the GEMM classes that run MXFP8 in the other blocks (names of _native.FP8_CLASSES, e.g. ("gate_up",), or an
        int mask; None = all); `block_classes`, one class set per block (each as `gemm_classes`; 0 = that block bf16),
        which overrides `gemm_classes` (include/flite.h flite_dit_set_fp8_block_classes). No reference counterpart
        (the reference runs bf16 only)."""
        self._fp8 = bool(enabled)
        eng = self.engine()
        eng.set_fp8_bf16_blocks(bf16_blocks)
        eng.set_fp8_gemm_classes(_native.fp8_class_mask(gemm_classes))
        if block_classes is not None and len(block_classes) != self.config.depth:
            raise ValueError(f"block_classes: one class set per block ({self.config.depth}), got {len(block_classes)}")
        eng.set_fp8_block_classes([] if block_classes is None else
                                  [c if isinstance(c, int) and not isinstance(c, bool) else _native.fp8_class_mask(c)
                                   for c in block_classes])
        eng.enable_fp8(self._fp8, self.device)
        return self

    # ------------------------------------------------------------------ forward
    @torch.no_grad()
    def forward(self, x, context, *args, context_attn_mask=None, timesteps=None, output_dtype=None):
        """DiT.forward (model.py:525-591). Accepts (x, ctx, t) and (x, ctx, mask, t)."""
        if len(args) == 1:
            timesteps = args[0]
        elif len(args) == 2:
            context_attn_mask, timesteps = args
        elif len(args) > 2:
            raise TypeError("forward(x, context[, context_attn_mask], timesteps)")
        if timesteps is None:
            raise TypeError("DiT.forward() missing the timesteps argument")
        eng = self.engine()
        dev = self.device
        _native.require_gpu(x, "x", contiguous=False)
        b, c, h, w = x.shape
        p = self.config.patch_size
        if c != self.config.in_channels:
            raise ValueError(f"x has {c} channels, model expects {self.config.in_channels}")
        if h % p or w % p:
            raise ValueError(f"latent size {h}x{w} must be a multiple of patch_size {p}")
        if context.dim() != 3 or context.shape[0] != b or context.shape[2] != self.config.cross_attn_input_size:
            raise ValueError(f"context must be [B={b}, L, {self.config.cross_attn_input_size}], got "
                             f"{tuple(context.shape)}")
        ctx = context.to(device=dev, dtype=torch.bfloat16).contiguous()
        L = ctx.shape[1]
        flat = ctx.view(b * L, -1)
        if context_attn_mask is None:  # all context tokens valid (model.py:46-47)
            cu = [i * L for i in range(b + 1)]
            packed = flat
        else:  # prepare_flash_attention_inputs (model.py:31-64): keep valid tokens in order, per-seq counts
            m = context_attn_mask.reshape(b, L).detach().to("cpu") != 0
            lens = m.sum(1).tolist()
            cu = [0]
            for n_ in lens:
                cu.append(cu[-1] + int(n_))
            idx = torch.nonzero(m.reshape(-1), as_tuple=True)[0].to(torch.int32).to(dev)
            packed = _native.gather_rows(flat, idx) if idx.numel() else flat[:0]
        eng.prepare(b, h, w, max(b * L, 1), max(b, 1))
        eng.set_context(packed, cu)
        ts = timesteps
        if not torch.is_tensor(ts):
            ts = torch.tensor(ts)
        ts = ts.reshape(-1)
        if ts.numel() == 1 and b > 1:
            ts = ts.expand(b)
        quant = ts.dtype == torch.bfloat16  # timesteps * 1000 evaluated in bf16 (model.py:551)
        t32 = ts.to(device=dev, dtype=torch.float32).contiguous()
        eng.set_timesteps(t32, quant)
        out_dtype = output_dtype or self.dtype
        out = torch.empty(b, c, h, w, device=dev, dtype=out_dtype)
        xin = x.contiguous()
        if xin.dtype not in (torch.float32, torch.bfloat16):
            xin = xin.float()
        eng.forward(xin, out, 0, 1)
        return out


def clean_state_dict(sd):
    """Strip the DDP / torch.compile key prefixes, as load_f_lite_pt does (pt.py:98-101)."""
    return {k.replace("module.", "").replace("_orig_mod.", ""): v for k, v in sd.items()}


def _is_norm_weight(name: str) -> bool:
    return name.endswith(("norm1.weight", "norm2.weight", "norm3.weight")) or name in (
        "context_norm.weight", "final_norm.weight")


# Model presets (SURVEY §8d "Model definitions"): F-Lite 7B = model.py layout with the train.py:685-698
# defaults; "10B" = model_v2.py layout (per-block adaLN, cross-attention in all 40 blocks), 12 heads (pt.py:89).
PRESETS = {
    "7b": dict(in_channels=16, patch_size=2, hidden_size=3072, depth=40, num_heads=12, mlp_ratio=4.0,
               cross_attn_input_size=4096, train_bias_and_rms=True, per_block_adaln=False),
    "10b": dict(in_channels=16, patch_size=2, hidden_size=3072, depth=40, num_heads=12, mlp_ratio=4.0,
                cross_attn_input_size=4096, train_bias_and_rms=True, per_block_adaln=True),
    "tiny": dict(in_channels=16, patch_size=2, hidden_size=512, depth=10, num_heads=2, mlp_ratio=4.0,
                 cross_attn_input_size=128, train_bias_and_rms=True, per_block_adaln=False),
    "tiny_v2": dict(in_channels=16, patch_size=2, hidden_size=512, depth=3, num_heads=2, mlp_ratio=4.0,
                    cross_attn_input_size=128, train_bias_and_rms=True, per_block_adaln=True),
}
