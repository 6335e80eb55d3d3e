"""Decode time of the native Flux VAE with bf16 vs MXFP8-stored conv weights (1024^2: 128x128 latents), plus the
weight-storage bytes of each mode. Usage: python f-lite_amd/tools/vae_fp8_time.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from f_lite.vae import AutoencoderKL  # noqa: E402


def timed(vae, lat, n=10):
    vae.decode_to_uint8(lat)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        vae.decode_to_uint8(lat)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


vae = AutoencoderKL.random(seed=0)
conv = sum(p.numel() for n, p in vae.named_parameters() if p.dim() == 4 and p.shape[-1] == 3)
lat = torch.randn(1, 16, 128, 128, device="cuda")
t16 = timed(vae, lat)
vae.enable_layerwise_casting(torch.float8_e4m3fn)
t8 = timed(vae, lat)
print(f"3x3 conv weights {conv / 1e6:.1f} M: bf16 {conv * 2 / 2**20:.1f} MiB, MXFP8 {conv * 33 / 32 / 2**20:.1f} MiB")
print(f"decode 1024^2: bf16 weights {t16:.2f} ms, fp8 weights {t8:.2f} ms ({100 * (t8 / t16 - 1):+.1f} %)")
