"""Per-block MXFP8 class policies against the REFERENCE at the metric's size: the 30-step
1024^2 CFG-1 loop's final latents vs the stub-loaded reference's fp32 trajectory (tests/golden/golden_full4, as
test_gpu_full_depth.py::test_fp8_first_blocks_bf16_1024_cfg1_vs_reference), 10B and 7B. Policies use
_native.fp8_block_masks syntax (blocks a policy does not name run every class MXFP8); "bf16" is the bf16 path.

    python f-lite_amd/tools/fp8_block_policy.py [--models 10b,7b] [--policies "0-7:none|0-3:none;4-7:down|..."]

One JSON line per (model, policy) with the PSNR and the policy's MXFP8 share of the block GEMM FLOPs.
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

DEFAULT = "bf16|0-7:none|0-3:none;4-7:down|0-3:none;4-7:gate_up+down|0-3:none;4-7:gate_up+down+qkv|0-1:none;2-7:down|" \
          "0-7:down|0-7:gate_up+down|0-3:down;4-7:gate_up+down|0-5:none|0-2:none;3-7:gate_up+down|"


def psnr(a, b):
    mse = (a.double() - b.double()).pow(2).mean().item()
    peak = b.double().abs().max().item()
    return float("inf") if mse == 0 else 10 * math.log10(peak * peak / mse)


def fp8_share(masks, cfg, T=4112):
    """MXFP8 share of the block GEMM FLOPs (SURVEY §8d per-block terms; cross blocks per layout)."""
    D, F = cfg["hidden_size"], int(cfg["hidden_size"] * cfg["mlp_ratio"])
    tot = f8 = 0.0
    for i, m in enumerate(masks):
        cross = cfg["per_block_adaln"] or i % 4 == 0 or i < 8
        terms = {1: 3 * D * D, 2: D * D, 16: 2 * D * F, 32: F * D}
        if cross:
            terms.update({4: D * D, 8: D * D})
        for bit, f in terms.items():
            tot += f
            f8 += f if m & bit else 0.0
    return f8 / tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="10b,7b")
    ap.add_argument("--policies", default=DEFAULT, help="'|'-separated policies ('bf16' = the bf16 path)")
    ap.add_argument("--cfg", type=float, default=1.0, help="guidance (golden_full4 holds 1 and 6)")
    args = ap.parse_args()
    gdir = ROOT / "tests" / "golden"
    gd = load_file(str(gdir / "golden_full4.safetensors"))
    meta = json.loads((gdir / "golden_full4_meta.json").read_text())
    dev = torch.device("cuda", 0)
    for name in args.models.split(","):
        cfg = PRESETS[name]
        m = DiT.random(seed=0, device=dev, **cfg)
        ctx = torch.empty(*meta["inputs"]["ctx"][1], device=dev, dtype=torch.bfloat16)
        nat.init_param_(ctx, meta["inputs"]["ctx"][0], seed=0, std=1.0)
        lat = torch.empty(*meta["inputs"]["latents_1024"][1], device=dev, dtype=torch.bfloat16)
        nat.init_param_(lat, meta["inputs"]["latents_1024"][0], seed=0, std=1.0)
        key = f"{name}.1024.s30.g{args.cfg:g}"
        for pol in args.policies.split("|"):
            if pol == "bf16":
                m.enable_fp8(False)
                masks = [0] * cfg["depth"]
            else:
                masks = nat.fp8_block_masks("" if pol == "all" else pol, cfg["depth"])
                m.enable_fp8(True, block_classes=masks)
            out = FLitePipeline(m)(prompt_embeds=ctx, latents=lat.clone(), height=1024, width=1024,
                                   num_inference_steps=30, guidance_scale=args.cfg,
                                   output_type="latent").images.float().cpu()
            p = psnr(out / 0.3611 + 0.1159, gd[f"{key}.f32.final"])
            print(json.dumps({"model": name, "policy": pol or "all", "cfg": args.cfg, "psnr_vs_ref_fp32": round(p, 2),
                              "fp8_flop_share": round(fp8_share(masks, cfg), 4),
                              "ref_bf16_vs_ref_fp32": round(meta.get(f"{key}.bf16_vs_f32_psnr", float("nan")), 2)}),
                  flush=True)
        m.enable_fp8(False)
        del m
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
