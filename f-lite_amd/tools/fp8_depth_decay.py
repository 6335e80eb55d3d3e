"""How the MXFP8 configuration's distance grows with depth (VERDICT r02 "What's weak" 1), at the configs[4]
shape: 10B layout, 1344x896 (T = 4720), 512-token context, CFG batch 2, t = 0.75.

For depth in (1, 2, 4, 8): GPU bf16 path, GPU fp8 path, fp32 oracle, fake-quant (MXFP8) oracle -> the four
distances; at depth 40: GPU fp8 vs GPU bf16 (the round-2 24.98 dB figure); then one 30-step CFG-6 image each in
bf16 and fp8 through the whole pipeline (tiled VAE decode, uint8) and their PSNR.

    python f-lite_amd/tools/fp8_depth_decay.py [--out gpurun_out/fp8_depth_decay.json] [--depths 1,2,4,8]
"""
import argparse
import dataclasses
import json
import math
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "f-lite_amd")]

import torch  # noqa: E402

from f_lite import DiT, FLitePipeline  # noqa: E402
from f_lite.model import PRESETS  # noqa: E402
from f_lite.vae import AutoencoderKL  # noqa: E402
from oracle import flite_ref as R  # noqa: E402

DEV = "cuda"


def psnr(a, ref, peak=None):
    a, ref = a.double().cpu(), ref.double().cpu()
    mse = (a - ref).pow(2).mean().item()
    peak = ref.abs().max().item() if peak is None else peak
    return float("inf") if mse == 0 else 10 * math.log10(peak * peak / mse)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/fp8_depth_decay.json")
    ap.add_argument("--depths", default="1,2,4,8")
    ap.add_argument("--no-images", action="store_true")
    args = ap.parse_args()
    torch.set_num_threads(16)
    t0 = time.time()
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 16, 112, 168, generator=g).bfloat16()
    ctx = torch.randn(2, 512, 4096, generator=g).bfloat16()
    t = torch.tensor([0.75, 0.75]).bfloat16()
    res = {"shape": "10B layout, 1344x896 (T=4720), ctx 512, CFG batch 2, t=0.75", "depth": {}}

    def fwd(m):
        return m(x.to(DEV), ctx.to(DEV), None, t.to(DEV), output_dtype=torch.float32).cpu()

    for d in [int(v) for v in args.depths.split(",")]:
        m = DiT.random(seed=0, device=DEV, **dict(PRESETS["10b"], depth=d))
        bf = fwd(m)
        m.enable_fp8(True)
        f8 = fwd(m)
        del m
        torch.cuda.empty_cache()
        rc = dataclasses.replace(R.PRESETS["10b"], depth=d)
        with torch.no_grad():
            f32 = R.RefDiT.random(rc, dtype=torch.float32)(x.float(), ctx.float(), None, t)
            fq = R.RefDiT.random(rc, dtype=torch.float32, fp8=True)(x.float(), ctx.float(), None, t)
        r = {"fp8_vs_fakequant": psnr(f8, fq), "fp8_vs_fp32": psnr(f8, f32), "fakequant_vs_fp32": psnr(fq, f32),
             "bf16_vs_fp32": psnr(bf, f32), "fp8_vs_bf16": psnr(f8, bf)}
        res["depth"][d] = r
        print(f"[{time.time() - t0:6.0f}s] depth {d}: " + ", ".join(f"{k} {v:.2f} dB" for k, v in r.items()),
              flush=True)

    m = DiT.random(seed=0, device=DEV, **PRESETS["10b"])
    bf = fwd(m)
    m.enable_fp8(True)
    f8 = fwd(m)
    res["depth40_fp8_vs_bf16"] = psnr(f8, bf)
    print(f"[{time.time() - t0:6.0f}s] depth 40: fp8 vs bf16 path {res['depth40_fp8_vs_bf16']:.2f} dB", flush=True)

    if not args.no_images:
        vae = AutoencoderKL.random(seed=0)
        pipe = FLitePipeline(m, vae=vae)
        pipe.enable_vae_tiling()
        pos = torch.empty(1, 512, 4096, device=DEV, dtype=torch.bfloat16)
        from f_lite import _native

        _native.init_param_(pos, "synthetic.t5_context", seed=1, std=1.0)
        lat = torch.empty(1, 16, 112, 168, device=DEV, dtype=torch.bfloat16)
        _native.init_param_(lat, "synthetic.latents.0", seed=2, std=1.0)
        out = {}
        for mode in ("fp8", "bf16"):
            m.enable_fp8(mode == "fp8")
            kw = dict(prompt_embeds=pos, latents=lat, height=896, width=1344, num_inference_steps=30,
                      guidance_scale=6.0)
            out[mode] = (pipe(**kw, output_type="latent").images.float().cpu(),
                         pipe(**kw, output_type="uint8").images.cpu())
            print(f"[{time.time() - t0:6.0f}s] 30-step {mode} image done", flush=True)
        res["image30_latent_psnr"] = psnr(out["fp8"][0], out["bf16"][0])
        res["image30_uint8_psnr"] = psnr(out["fp8"][1].float(), out["bf16"][1].float(), peak=255.0)
        print(f"30-step 1344x896 CFG 6: fp8 vs bf16 final latents {res['image30_latent_psnr']:.2f} dB, uint8 image "
              f"{res['image30_uint8_psnr']:.2f} dB", flush=True)
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
