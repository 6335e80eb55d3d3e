"""TEST INFRASTRUCTURE ONLY. CPU restatement of the Flux VAE decoder (diffusers AutoencoderKL.decode).

diffusers is not installed in this image and is not vendored in the reference (requirements.txt:1, unpinned);
the reference calls it at pipeline.py:301-307. This restates the published diffusers Decoder for the FLUX.1 VAE
config (latent_channels 16, block_out_channels (128, 256, 512, 512), layers_per_block 2, GroupNorm(32, eps 1e-6),
SiLU, UNetMidBlock2D with one single-head attention, UpDecoderBlock2D with nearest-2x Upsample2D + conv):

    conv_in -> mid(resnet, attn, resnet) -> 4 x up_block(3 resnets [+ upsample]) -> GN -> SiLU -> conv_out
    ResnetBlock2D: h = conv1(silu(norm1(x))); h = conv2(silu(norm2(h))); out = shortcut(x) + h
    Attention:     h = group_norm(x); softmax(q k^T / sqrt(C)) v -> to_out[0]; out = h + x

PARITY UNPINNED against diffusers itself (no diffusers source or Flux VAE weights in the container): this
restatement is the oracle for the HIP VAE kernels, on weights from the shared deterministic generator.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .weights import hash_uniform

FLUX = dict(latent_channels=16, block_out_channels=(128, 256, 512, 512), layers_per_block=2, norm_num_groups=32,
            scaling_factor=0.3611, shift_factor=0.1159)


def vae_param_shapes(cfg=FLUX):
    rev = list(reversed(cfg["block_out_channels"]))
    s = {}

    def conv(n, co, ci, k):
        s[n + ".weight"] = (co, ci, k, k)
        s[n + ".bias"] = (co,)

    def gn(n, c):
        s[n + ".weight"] = (c,)
        s[n + ".bias"] = (c,)

    def resnet(pre, ci, co):
        gn(pre + ".norm1", ci)
        conv(pre + ".conv1", co, ci, 3)
        gn(pre + ".norm2", co)
        conv(pre + ".conv2", co, co, 3)
        if ci != co:
            conv(pre + ".conv_shortcut", co, ci, 1)

    conv("decoder.conv_in", rev[0], cfg["latent_channels"], 3)
    resnet("decoder.mid_block.resnets.0", rev[0], rev[0])
    a = "decoder.mid_block.attentions.0"
    gn(a + ".group_norm", rev[0])
    for n in ("to_q", "to_k", "to_v", "to_out.0"):
        s[f"{a}.{n}.weight"] = (rev[0], rev[0])
        s[f"{a}.{n}.bias"] = (rev[0],)
    resnet("decoder.mid_block.resnets.1", rev[0], rev[0])
    prev = rev[0]
    for i, c in enumerate(rev):
        for j in range(cfg["layers_per_block"] + 1):
            resnet(f"decoder.up_blocks.{i}.resnets.{j}", prev if j == 0 else c, c)
        prev = c
        if i < len(rev) - 1:
            conv(f"decoder.up_blocks.{i}.upsamplers.0.conv", c, c, 3)
    gn("decoder.conv_norm_out", rev[-1])
    conv("decoder.conv_out", 3, rev[-1], 3)
    return s


def make_vae_state_dict(cfg=FLUX, seed=0):
    """Same values as f_lite.vae.AutoencoderKL.random (bf16-rounded, returned in fp32)."""
    out = {}
    for name, shape in vae_param_shapes(cfg).items():
        if ".norm" in name or "group_norm" in name or "conv_norm_out" in name:
            out[name] = torch.ones(shape) if name.endswith(".weight") else torch.zeros(shape)
            continue
        std = 0.02 if name.endswith(".bias") else 1.0 / math.sqrt(math.prod(shape[1:]))
        v = torch.from_numpy(hash_uniform("vae." + name, math.prod(shape), std, seed)).reshape(shape)
        out[name] = v.to(torch.bfloat16).float()
    return out


class RefVAEDecoder:
    def __init__(self, params, cfg=FLUX, dtype=torch.float32):
        self.p = {k: v.to(dtype) for k, v in params.items()}
        self.cfg = cfg
        self.dtype = dtype

    def _conv(self, x, n, pad=1):
        return F.conv2d(x, self.p[n + ".weight"], self.p[n + ".bias"], padding=pad)

    def _gn(self, x, n):
        return F.group_norm(x, self.cfg["norm_num_groups"], self.p[n + ".weight"], self.p[n + ".bias"], eps=1e-6)

    def _resnet(self, x, pre):
        h = self._conv(F.silu(self._gn(x, pre + ".norm1")), pre + ".conv1")
        h = self._conv(F.silu(self._gn(h, pre + ".norm2")), pre + ".conv2")
        if pre + ".conv_shortcut.weight" in self.p:
            x = self._conv(x, pre + ".conv_shortcut", pad=0)
        return x + h

    def _attn(self, x, pre):
        B, C, H, W = x.shape
        h = self._gn(x, pre + ".group_norm").reshape(B, C, H * W).transpose(1, 2)
        q = F.linear(h, self.p[pre + ".to_q.weight"], self.p[pre + ".to_q.bias"])
        k = F.linear(h, self.p[pre + ".to_k.weight"], self.p[pre + ".to_k.bias"])
        v = F.linear(h, self.p[pre + ".to_v.weight"], self.p[pre + ".to_v.bias"])
        a = torch.softmax(q @ k.transpose(1, 2) / math.sqrt(C), dim=-1) @ v
        o = F.linear(a, self.p[pre + ".to_out.0.weight"], self.p[pre + ".to_out.0.bias"])
        return o.transpose(1, 2).reshape(B, C, H, W) + x

    def decode(self, z):
        """z: latents already scaled (z / scaling_factor + shift_factor), [B, 16, h, w] -> image [B, 3, 8h, 8w]."""
        x = self._conv(z.to(self.dtype), "decoder.conv_in")
        x = self._resnet(x, "decoder.mid_block.resnets.0")
        x = self._attn(x, "decoder.mid_block.attentions.0")
        x = self._resnet(x, "decoder.mid_block.resnets.1")
        n = len(self.cfg["block_out_channels"])
        for i in range(n):
            for j in range(self.cfg["layers_per_block"] + 1):
                x = self._resnet(x, f"decoder.up_blocks.{i}.resnets.{j}")
            if i < n - 1:
                x = F.interpolate(x, scale_factor=2.0, mode="nearest")
                x = self._conv(x, f"decoder.up_blocks.{i}.upsamplers.0.conv")
        x = F.silu(self._gn(x, "decoder.conv_norm_out"))
        return self._conv(x, "decoder.conv_out")


def decode_to_uint8(dec: RefVAEDecoder, latents, scaling=FLUX["scaling_factor"], shift=FLUX["shift_factor"]):
    """pipeline.py:304-326: latents / scaling + shift -> decode -> uint8 [B, H, W, 3]."""
    img = dec.decode(latents / scaling + shift)
    img = (img / 2 + 0.5).clamp(0, 1)
    img = (img * 255).round().clamp(0, 255).to(torch.uint8)
    return img.permute(0, 2, 3, 1).contiguous()


def _blend_v(a, b, blend_extent):
    """diffusers AutoencoderKL.blend_v: b's first rows ramp from a's last rows, in place."""
    e = min(a.shape[2], b.shape[2], blend_extent)
    for y in range(e):
        b[:, :, y, :] = a[:, :, -e + y, :] * (1 - y / e) + b[:, :, y, :] * (y / e)
    return b


def _blend_h(a, b, blend_extent):
    """diffusers AutoencoderKL.blend_h: b's first columns ramp from a's last columns, in place."""
    e = min(a.shape[3], b.shape[3], blend_extent)
    for x in range(e):
        b[:, :, :, x] = a[:, :, :, -e + x] * (1 - x / e) + b[:, :, :, x] * (x / e)
    return b


def tiled_decode(dec, z, tile_latent=128, tile_sample=1024, overlap=0.25):
    """diffusers AutoencoderKL.tiled_decode (diffusers is third-party and not vendored; requirements.txt:1 leaves
    it unpinned), which the reference turns on with pipe.vae.enable_tiling() (generate.py:77-78,
    pipeline.py:90-93) and AutoencoderKL.decode takes once a latent side exceeds tile_latent. Restated from its
    published algorithm: latent tiles every int(tile_latent * (1 - overlap)), each decoded on its own; every tile
    blended in place with its (already blended) upper, then left neighbour over int(tile_sample * overlap)
    pixels; crops of tile_sample - that extent concatenated. `dec` maps scaled latents [B, C, h, w] to images
    [B, 3, 8h, 8w]. Parity unpinned against diffusers itself; blending in the decoder's dtype (fp32 here)."""
    overlap_size = int(tile_latent * (1 - overlap))
    blend_extent = int(tile_sample * overlap)
    row_limit = tile_sample - blend_extent
    rows = []
    for i in range(0, z.shape[2], overlap_size):
        row = []
        for j in range(0, z.shape[3], overlap_size):
            row.append(dec.decode(z[:, :, i:i + tile_latent, j:j + tile_latent]))
        rows.append(row)
    result_rows = []
    for i, row in enumerate(rows):
        result_row = []
        for j, tile in enumerate(row):
            if i > 0:
                tile = _blend_v(rows[i - 1][j], tile, blend_extent)
            if j > 0:
                tile = _blend_h(row[j - 1], tile, blend_extent)
            result_row.append(tile[:, :, :row_limit, :row_limit])
        result_rows.append(torch.cat(result_row, dim=3))
    return torch.cat(result_rows, dim=2)


def tiled_decode_to_uint8(dec, latents, tile_latent=128, tile_sample=1024, overlap=0.25,
                          scaling=FLUX["scaling_factor"], shift=FLUX["shift_factor"]):
    """pipeline.py:304-326 with the tiled decode above."""
    img = tiled_decode(dec, latents / scaling + shift, tile_latent, tile_sample, overlap)
    img = (img / 2 + 0.5).clamp(0, 1)
    img = (img * 255).round().clamp(0, 255).to(torch.uint8)
    return img.permute(0, 2, 3, 1).contiguous()
