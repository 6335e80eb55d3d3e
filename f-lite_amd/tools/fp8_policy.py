"""fp8 precision policies: which blocks keep bf16 GEMMs and which GEMM classes run
MXFP8, against image quality and speed.

BASELINE configs[4] workload: 10B (model_v2 layout), 1344x896, 30 CFG-6 steps, tiled VAE decode to uint8. For each
policy: the uint8 image's PSNR against the bf16 image (same seed, peak 255), the final latents' PSNR against the bf16
latents, and images/s over `--images` graph-replayed images after a warm-up. One JSON line per policy.

    python f-lite_amd/tools/fp8_policy.py [--images 3] [--policies "none;0,39;0,1,38,39"]
        [--class-policies "gate_up;gate_up,down;qkv,proj,cross_q,cross_proj"]

--policies: block lists kept bf16 (every GEMM class fp8 in the others); --class-policies: GEMM-class sets run MXFP8
in every block (_native.FP8_CLASSES names; the other classes run their bf16 GEMMs). Either list may be "" to skip it.
"""
import argparse
import json
import math
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "f-lite_amd"), str(ROOT)]

import torch  # noqa: E402

from f_lite import DiT, FLitePipeline, _native  # noqa: E402
from f_lite.model import PRESETS  # noqa: E402
from f_lite.vae import AutoencoderKL  # noqa: E402


def psnr(a, b, peak=None):
    mse = (a.double() - b.double()).pow(2).mean().item()
    peak = b.double().abs().max().item() if peak is None else peak
    return float("inf") if mse == 0 else 10 * math.log10(peak * peak / mse)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=3)
    ap.add_argument("--height", type=int, default=896)
    ap.add_argument("--width", type=int, default=1344)
    ap.add_argument("--policies", default="none;0;39;0,39;0,1,38,39;0,1,2,3;36,37,38,39;0,1,2,3,36,37,38,39")
    ap.add_argument("--class-policies", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    m = DiT.random(seed=0, device=dev, **PRESETS["10b"])
    pipe = FLitePipeline(m, vae=AutoencoderKL.random(seed=0, device=dev))
    pipe.enable_vae_tiling()
    ctx = torch.empty(1, 512, 4096, device=dev, dtype=torch.bfloat16)
    _native.init_param_(ctx, "synthetic.t5_context", seed=1, std=1.0)
    lh, lw = args.height // 8, args.width // 8

    def lat(i):
        t = torch.empty(1, 16, lh, lw, device=dev, dtype=torch.bfloat16)
        return _native.init_param_(t, f"synthetic.latents.{i}", seed=2, std=1.0)

    kw = dict(prompt_embeds=ctx, height=args.height, width=args.width, num_inference_steps=30, guidance_scale=6.0)

    def measure():
        img = pipe(**kw, latents=lat(0), output_type="uint8").images.cpu()
        lat_out = pipe(**kw, latents=lat(0), output_type="latent").images.float().cpu()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.images):
            pipe(**kw, latents=lat(1 + i), output_type="uint8")
        torch.cuda.synchronize()
        return img, lat_out, args.images / (time.perf_counter() - t0)

    ref_img, ref_lat, ref_ips = measure()
    print(json.dumps({"policy": "bf16", "images_per_s": round(ref_ips, 4)}), flush=True)
    runs = [(pol, None) for pol in args.policies.split(";") if args.policies.strip()]
    runs += [("none", cp) for cp in args.class_policies.split(";") if args.class_policies.strip()]
    for pol, classes in runs:
        blocks = [] if pol.strip() in ("", "none") else [int(b) for b in pol.split(",")]
        m.enable_fp8(True, bf16_blocks=blocks, gemm_classes=classes)
        img, lat_out, ips = measure()
        print(json.dumps({"policy": "fp8", "bf16_blocks": blocks, "fp8_classes": classes or "all",
                          "images_per_s": round(ips, 4), "speedup_vs_bf16": round(ips / ref_ips, 4),
                          "image_psnr_vs_bf16_db": round(psnr(img.float(), ref_img.float(), 255.0), 2),
                          "latent_psnr_vs_bf16_db": round(psnr(lat_out, ref_lat), 2)}), flush=True)
    m.enable_fp8(False)


if __name__ == "__main__":
    main()
