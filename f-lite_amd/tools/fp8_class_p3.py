"""fp8 GEMM-class policies against the REFERENCE (not against our bf16 path): the 30-step 256^2 loop's final latents
vs the stub-loaded reference's fp32 trajectory (tests/golden/golden_full3, as test_gpu_fp8.py's P3 test), at CFG 1
and CFG 6, for 7B and 10B. DESIGN §5's Pareto table prices the same policies' speed at 1344x896, CFG 6.

    python f-lite_amd/tools/fp8_class_p3.py [--models 7b,10b] [--policies "all;gate_up,qkv;down;none"]

Policy "none" is the bf16 path; a policy "all@0,1,38,39" keeps those blocks bf16 with every class fp8 in the rest.
One line per (model, CFG, policy).
"""
import argparse
import json
import math
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "f-lite_amd"), str(ROOT)]

import torch  # noqa: E402
from safetensors.torch import load_file  # noqa: E402

from f_lite import DiT, FLitePipeline  # noqa: E402
from f_lite import _native as nat  # noqa: E402
from f_lite.model import PRESETS  # noqa: E402


def psnr(a, b):
    mse = (a.double() - b.double()).pow(2).mean().item()
    peak = b.double().abs().max().item()
    return float("inf") if mse == 0 else 10 * math.log10(peak * peak / mse)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="7b,10b")
    ap.add_argument("--policies", default="none;all;gate_up,qkv;gate_up,down;gate_up;qkv,proj,cross_q,cross_proj;down")
    args = ap.parse_args()
    gdir = ROOT / "tests" / "golden"
    gd = load_file(str(gdir / "golden_full3.safetensors"))
    meta = json.loads((gdir / "golden_full3_meta.json").read_text())
    dev = torch.device("cuda", 0)
    for name in args.models.split(","):
        m = DiT.random(seed=0, device=dev, **PRESETS[name])
        ctx = torch.empty(*meta["inputs"]["ctx"][1], device=dev, dtype=torch.bfloat16)
        nat.init_param_(ctx, meta["inputs"]["ctx"][0], seed=0, std=1.0)
        lat = torch.empty(*meta["inputs"]["latents_256"][1], device=dev, dtype=torch.bfloat16)
        nat.init_param_(lat, meta["inputs"]["latents_256"][0], seed=0, std=1.0)
        for pol in args.policies.split(";"):
            classes, _, blocks = pol.partition("@")
            keep16 = [int(b) for b in blocks.split(",") if b.strip()]
            if classes == "none":
                m.enable_fp8(False)
            else:
                m.enable_fp8(True, bf16_blocks=keep16, gemm_classes=None if classes == "all" else classes.split(","))
            for g in (1.0, 6.0):
                key = f"{name}.256.s30.g{g:g}"
                out = FLitePipeline(m)(prompt_embeds=ctx, latents=lat.clone(), height=256, width=256,
                                       num_inference_steps=30, guidance_scale=g,
                                       output_type="latent").images.float().cpu()
                p = psnr(out / 0.3611 + 0.1159, gd[f"{key}.f32.final"])
                print(json.dumps({"model": name, "cfg": g, "policy": pol, "psnr_vs_ref_fp32": round(p, 2),
                                  "ref_bf16_vs_ref_fp32": round(meta[f"{key}.bf16_vs_f32_psnr"], 2)}), flush=True)
        m.enable_fp8(False)
        del m
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
