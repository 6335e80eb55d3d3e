"""Flux VAE decoder (diffusers AutoencoderKL, FLUX.1 config) on the MI355X-native path.

The reference calls `self.vae.decode(latents.to(vae_dtype)).sample` (pipeline.py:307) on a diffusers
AutoencoderKL (not vendored; FLUX.1-schnell VAE per pt.py:143), after `latents / scaling_factor +
shift_factor` (pipeline.py:301-304), and post-processes to uint8 (pipeline.py:324-326). This module holds the
decoder parameters under the diffusers state-dict keys (`decoder.*`) and runs the whole decode + uint8
conversion natively (libflite_hip.so: flite_vae_*): implicit-GEMM MFMA 3x3 convolutions with the nearest-2x
upsample folded into the addressing, fused residual adds, GroupNorm(+SiLU) kernels and the mid-block
attention as MFMA GEMMs around a row softmax.
"""
from __future__ import annotations

import ctypes
import json
import math
from pathlib import Path
from types import SimpleNamespace

import torch
from torch import nn

from . import _native

FLUX_VAE_CONFIG = dict(in_channels=3, out_channels=3, latent_channels=16, block_out_channels=(128, 256, 512, 512),
                       layers_per_block=2, norm_num_groups=32, scaling_factor=0.3611, shift_factor=0.1159,
                       sample_size=1024, use_quant_conv=False, use_post_quant_conv=False,
                       mid_block_add_attention=True)


class ResnetBlock2D(nn.Module):
    def __init__(self, cin, cout, groups=32):
        super().__init__()
        self.norm1 = nn.GroupNorm(groups, cin, eps=1e-6)
        self.conv1 = nn.Conv2d(cin, cout, 3, padding=1)
        self.norm2 = nn.GroupNorm(groups, cout, eps=1e-6)
        self.conv2 = nn.Conv2d(cout, cout, 3, padding=1)
        if cin != cout:
            self.conv_shortcut = nn.Conv2d(cin, cout, 1)


class AttnBlock(nn.Module):
    def __init__(self, c, groups=32):
        super().__init__()
        self.group_norm = nn.GroupNorm(groups, c, eps=1e-6)
        self.to_q = nn.Linear(c, c)
        self.to_k = nn.Linear(c, c)
        self.to_v = nn.Linear(c, c)
        self.to_out = nn.ModuleList([nn.Linear(c, c), nn.Dropout(0.0)])


class MidBlock(nn.Module):
    def __init__(self, c, groups=32, attn=True):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(c, c, groups), ResnetBlock2D(c, c, groups)])
        self.attentions = nn.ModuleList([AttnBlock(c, groups)] if attn else [])


class Upsample2D(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv = nn.Conv2d(c, c, 3, padding=1)


class UpBlock(nn.Module):
    def __init__(self, cin, cout, n, upsample, groups=32):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(cin if i == 0 else cout, cout, groups) for i in range(n)])
        if upsample:
            self.upsamplers = nn.ModuleList([Upsample2D(cout)])


class Decoder(nn.Module):
    def __init__(self, latent_channels=16, block_out_channels=(128, 256, 512, 512), layers_per_block=2,
                 norm_num_groups=32, mid_attention=True):
        super().__init__()
        rev = list(reversed(block_out_channels))
        self.conv_in = nn.Conv2d(latent_channels, rev[0], 3, padding=1)
        self.mid_block = MidBlock(rev[0], norm_num_groups, mid_attention)
        blocks = []
        prev = rev[0]
        for i, c in enumerate(rev):
            blocks.append(UpBlock(prev, c, layers_per_block + 1, i < len(rev) - 1, norm_num_groups))
            prev = c
        self.up_blocks = nn.ModuleList(blocks)
        self.conv_norm_out = nn.GroupNorm(norm_num_groups, block_out_channels[0], eps=1e-6)
        self.conv_act = nn.SiLU()
        self.conv_out = nn.Conv2d(block_out_channels[0], 3, 3, padding=1)


def vae_param_init(name: str, shape) -> tuple:
    """(std, kind) of the synthetic VAE initialisation: GroupNorm weight 1 / bias 0, conv/linear weights
    uniform with std 1/sqrt(fan_in) (keeps activations O(1) through 30+ layers), biases std 0.02."""
    if ".norm" in name or "group_norm" in name or "conv_norm_out" in name:
        return (0.0, "ones") if name.endswith(".weight") else (0.0, "zeros")
    if name.endswith(".bias"):
        return (0.02, "hash")
    fan_in = int(math.prod(shape[1:]))
    return (1.0 / math.sqrt(fan_in), "hash")


def decoder_flops(H: int, W: int, cfg: dict = FLUX_VAE_CONFIG) -> float:
    """Algorithmic FLOPs (2/MAC) of one decode to an H x W image (convs, 1x1 shortcuts, attention)."""
    rev = list(reversed(cfg["block_out_channels"]))
    n = len(rev)
    h, w = H >> (n - 1), W >> (n - 1)
    L = cfg["latent_channels"]
    f = 2 * 9 * L * rev[0] * h * w
    c = rev[0]
    hw = h * w
    f += 2 * 2 * (2 * 9 * c * c * hw)  # mid resnets
    f += 4 * 2 * hw * c * c + 2 * 2 * hw * hw * c  # q,k,v,out + QK^T + PV
    prev = c
    for i, co in enumerate(rev):
        for j in range(cfg["layers_per_block"] + 1):
            ci = prev if j == 0 else co
            f += 2 * 9 * ci * co * hw + 2 * 9 * co * co * hw
            if ci != co:
                f += 2 * ci * co * hw
        prev = co
        if i < n - 1:
            hw *= 4
            f += 2 * 9 * co * co * hw
    f += 2 * 9 * rev[-1] * 3 * hw
    return float(f)


class AutoencoderKL(nn.Module):
    """Decoder half of diffusers AutoencoderKL with the FLUX.1 VAE config (decode path only)."""

    def __init__(self, **cfg):
        super().__init__()
        c = dict(FLUX_VAE_CONFIG)
        c.update(cfg)
        self.config = SimpleNamespace(**c)
        self.decoder = Decoder(c["latent_channels"], tuple(c["block_out_channels"]), c["layers_per_block"],
                               c["norm_num_groups"], c["mid_block_add_attention"])
        self._engine = None
        self._bound = None
        self._prepared = None
        self._wgen = 0  # bumped by writers that bypass the parameters' version counters
        # diffusers AutoencoderKL tiling state (enable_tiling / disable_tiling): tiles of sample_size pixels =
        # sample_size / 2**(levels-1) latents, overlap factor 0.25
        self.use_tiling = False
        self.use_slicing = False
        self.tile_sample_min_size = int(c["sample_size"])
        self.tile_latent_min_size = int(c["sample_size"]) >> (len(c["block_out_channels"]) - 1)
        self.tile_overlap_factor = 0.25
        self.fp8_weights = False  # enable_layerwise_casting(torch.float8_e4m3fn)

    def enable_tiling(self, use_tiling: bool = True):
        """diffusers AutoencoderKL.enable_tiling (the reference calls it at generate.py:78)."""
        self.use_tiling = use_tiling

    def disable_tiling(self):
        self.enable_tiling(False)

    def enable_slicing(self):
        """diffusers AutoencoderKL.enable_slicing (generate.py:77): the native decoder already decodes one image
        at a time."""
        self.use_slicing = True

    def disable_slicing(self):
        self.use_slicing = False

    def enable_layerwise_casting(self, storage_dtype=torch.float8_e4m3fn, compute_dtype=torch.bfloat16, **_):
        """diffusers ModelMixin.enable_layerwise_casting for the decoder (the "fp8 VAE" of SURVEY 8f rank 4): the
        3x3 conv weights are stored in fp8 and up-cast to bf16 right before each conv. Stored as MXFP8 (e4m3 with
        one power-of-two scale per 32 input-channel values of a tap) rather than a per-tensor cast (random-init
        Flux VAE: 34.7 dB from the bf16-weight decode, 50.4 dB from the oracle on the same quantised weights). Norm, attention and bias parameters stay bf16, as diffusers
        skips them by default."""
        if storage_dtype not in (torch.float8_e4m3fn, torch.bfloat16):
            raise _native.FliteError(f"layerwise casting: storage dtype {storage_dtype} is not supported")
        if compute_dtype != torch.bfloat16:
            raise _native.FliteError("layerwise casting: the native decoder computes in bf16")
        self.fp8_weights = storage_dtype == torch.float8_e4m3fn
        self._prepared = None

    def disable_layerwise_casting(self):
        self.enable_layerwise_casting(torch.bfloat16)

    @classmethod
    def empty(cls, device="cuda", dtype=torch.bfloat16, **cfg):
        with torch.device("meta"):
            m = cls(**cfg)
        return m.to_empty(device=device).to(dtype)

    @classmethod
    def random(cls, seed=0, device="cuda", dtype=torch.bfloat16, **cfg):
        m = cls.empty(device=device, dtype=dtype, **cfg)
        with torch.no_grad():
            for name, p in m.named_parameters():
                std, kind = vae_param_init(name, tuple(p.shape))
                if kind == "ones":
                    _native.init_param_(p.data, name, ones=True)
                else:
                    _native.init_param_(p.data, "vae." + name, seed=seed, std=std)
        torch.cuda.synchronize()
        return m

    @classmethod
    def from_pretrained(cls, path, torch_dtype=torch.bfloat16, device="cuda", subfolder=None):
        from safetensors.torch import load_file

        p = Path(path) / subfolder if subfolder else Path(path)
        cfg = json.loads((p / "config.json").read_text())
        keep = {k: v for k, v in cfg.items() if k in FLUX_VAE_CONFIG}
        m = cls.empty(device=device, dtype=torch_dtype, **keep)
        sd = {}
        for f in sorted(p.glob("diffusion_pytorch_model*.safetensors")):
            sd.update(load_file(str(f)))
        dec = {k: v for k, v in sd.items() if k.startswith("decoder.")}  # encoder weights are not needed
        m.load_state_dict(dec, strict=True)
        return m

    def save_pretrained(self, path):
        from safetensors.torch import save_file

        p = Path(path)
        p.mkdir(parents=True, exist_ok=True)
        cfg = {k: (list(v) if isinstance(v, tuple) else v) for k, v in vars(self.config).items()}
        cfg["_class_name"] = "AutoencoderKL"
        (p / "config.json").write_text(json.dumps(cfg, indent=2))
        save_file({k: v.detach().contiguous().cpu() for k, v in self.state_dict().items()},
                  str(p / "diffusion_pytorch_model.safetensors"))

    def weights_updated(self):
        """Declare that parameters were written behind autograd's version counters (through `p.data` or raw device
        pointers): the engine re-packs its conv weights before the next decode."""
        self._wgen += 1
        return self

    @property
    def dtype(self):
        return next(self.parameters()).dtype

    def engine(self):
        params = list(self.named_parameters())
        if not params[0][1].is_cuda or self.dtype != torch.bfloat16:
            raise _native.FliteError("the native VAE decoder needs bf16 parameters on a ROCm device")
        # storage and contents: an in-place update (load_state_dict's copy_) bumps the parameters' versions, and
        # the engine re-packs its conv weights from the new values
        ptrs = tuple((n, p.data_ptr()) for n, p in params)
        vers = (self._wgen,) + tuple(p._version for _, p in params)
        if self._engine is None:
            self._engine = _native.VaeEngine(self.config)
            self._bound = None
        if self._bound is None or self._bound[0] != ptrs:
            for n, p in params:
                self._engine.bind(n, p.data)
            self._prepared = None
        elif self._bound[1] != vers:
            self._engine.weights_updated()
        self._bound = (ptrs, vers)
        if self._prepared is None:
            self._engine.enable_fp8_weights(self.fp8_weights)
        return self._engine

    @torch.no_grad()
    def decode_to_uint8(self, latents: torch.Tensor, scaling_factor=None, shift_factor=None) -> torch.Tensor:
        """latents (fp32 [B, 16, h, w], the sampler output) -> uint8 [B, 8h, 8w, 3] on the device."""
        eng = self.engine()
        scaling = self.config.scaling_factor if scaling_factor is None else scaling_factor
        shift = self.config.shift_factor if shift_factor is None else shift_factor
        z = latents.float().contiguous()
        B, C, h, w = z.shape
        n = len(self.config.block_out_channels) - 1
        img = torch.empty(B, h << n, w << n, 3, device=z.device, dtype=torch.uint8)
        tl = self.tile_latent_min_size
        if self.use_tiling and (h > tl or w > tl):  # AutoencoderKL._decode's tiling condition
            key = ("tiled", h, w, tl, self.tile_sample_min_size, self.tile_overlap_factor)
            if self._prepared != key:
                eng.prepare_tiled(h, w, tl, self.tile_sample_min_size, self.tile_overlap_factor)
                self._prepared = key
            eng.decode_tiled_uint8(z, img, scaling, shift)
            return img
        if self._prepared != (h, w):
            eng.prepare(h, w)
            self._prepared = (h, w)
        eng.decode_uint8(z, img, scaling, shift)
        return img
