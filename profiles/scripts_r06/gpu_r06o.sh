#!/bin/bash
# round 6, call o: 10B 1344x896 30-step CFG-6 product path vs the reference's fp32 trajectory (the bf16 floor is still
# generating): latents and tiled-VAE image PSNR, printed
set -o pipefail
mkdir -p gpurun_out/r06o
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u - > gpurun_out/r06o/cfg6_1344.log 2>&1 <<'PY' || { tail -20 gpurun_out/r06o/cfg6_1344.log; exit 1; }
import json, math, sys
sys.path[:0] = ["f-lite_amd", "."]
import torch
from safetensors.torch import load_file
from f_lite import DiT, FLitePipeline, _native
from f_lite.model import PRESETS
from f_lite.vae import AutoencoderKL
gd = load_file("tests/golden/golden_full5.safetensors"); meta = json.load(open("tests/golden/golden_full5_meta.json"))
def hashed(k):
    name, shape = meta["inputs"][k]
    return _native.init_param_(torch.empty(*shape, device="cuda", dtype=torch.bfloat16), name, seed=0, std=1.0)
def psnr(a, ref):
    a, ref = a.double().cpu(), ref.double().cpu()
    return 10 * math.log10(ref.abs().max().item() ** 2 / (a - ref).pow(2).mean().item())
m = DiT.random(seed=0, device="cuda", **PRESETS["10b"])
pipe = FLitePipeline(m, vae=AutoencoderKL.random(seed=0)); pipe.enable_vae_tiling()
kw = dict(prompt_embeds=hashed("ctx"), latents=hashed("latents"), height=896, width=1344, num_inference_steps=30,
          guidance_scale=6.0, use_graph=True)
for resid in (torch.bfloat16, torch.float32):
    m.set_residual_dtype(resid)
    lat = pipe(**kw, output_type="latent").images.float()
    p = psnr(lat / 0.3611 + 0.1159, gd["10b.1344x896.s30.g6.f32.final"])
    img = pipe(**kw, output_type="uint8").images.cpu().double(); ref = gd["10b.1344x896.s30.g6.f32.image"].double()
    pi = 10 * math.log10(255.0 ** 2 / (img - ref).pow(2).mean().item())
    print(f"10b 1344x896 30-step CFG-6, {resid} residual: latents {p:.2f} dB, uint8 image {pi:.2f} dB vs the reference fp32 run", flush=True)
PY
cat gpurun_out/r06o/cfg6_1344.log | grep "dB"
