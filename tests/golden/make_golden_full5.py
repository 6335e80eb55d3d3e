"""The reference's DEFAULT configuration pinned end to end (VERDICT r05 "next 1"; SURVEY §8c fixture set iv).

generate.py:19-22 defaults every user runs: width 1344, height 896, 30 steps, CFG 6 (BASELINE configs[2] / [4]),
here on the 10B (model_v2) layout. T = 16 + 56 * 84 = 4720 tokens per sample, a non-square 56 x 84 RoPE grid
(model.py:334-400), alpha = 2 * sqrt(112 * 168 / 4096) = 4.2866 (pipeline.py:240-242), and the 112 x 168 latent
that generate.py:77-78's VAE tiling splits into 2 x 2 overlapping tiles.

Run in the build container only (needs /root/reference; ~8 h of CPU, ~40 GB of RAM; resumable):

    python tests/golden/make_golden_full5.py [--threads 6] [--only KEY ...] [--no-image]

Same stub-loading, block streaming and on-disk per-call cache as make_golden_full4.py (the reference's own
DiT.forward, DiTBlock.forward and FLitePipeline.__call__; the 10B-v2 top level is make_golden.v2_forward_fixed,
SURVEY §0.3); the CFG-1 cond-half shortcut is the one stated in make_golden_full4.py's header.

Fixtures (tests/golden/golden_full5.safetensors) + golden_full5_meta.json:
  10b.1344x896.s30.g1.f32.final    CFG 1, the reference's fp32 arithmetic: final latents / scaling + shift
  10b.1344x896.s30.g6.f32.final    CFG 6 (generate.py's default guidance), fp32
  10b.1344x896.s30.g6.bf16.final   CFG 6 in the reference's bf16 arithmetic (its own floor vs fp32)
  10b.1344x896.s30.g1.bf16.final   CFG 1, bf16 (the CFG-1 floor)
  {key}.image                      uint8 [1, 896, 1344, 3]: oracle/vae_ref.py's restated diffusers tiled decode
                                   (128-latent tiles, overlap 0.25, seed-0 generator weights) on that final + the
                                   pipeline.py:324-326 post-process; the bf16 images give the image-space floor.
"""
from __future__ import annotations

import sys

sys.dont_write_bytecode = True

import argparse  # noqa: E402
import json  # noqa: E402
import math  # noqa: E402
import time  # noqa: E402
from pathlib import Path  # noqa: E402

import torch  # noqa: E402
from safetensors.torch import load_file, save_file  # noqa: E402

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(REPO))
import make_golden as MG  # noqa: E402
import make_golden_full as MGF  # noqa: E402
from make_golden_full2 import V2Adapter  # noqa: E402
from make_golden_full4 import CachedCall  # noqa: E402

STEPS = 30
H, W = 896, 1344
LAT_NAME = "golden.latents.1344x896"  # [1, 16, 112, 168]
LAT_SHAPE = (1, 16, H // 8, W // 8)
OUT = HERE / "golden_full5.safetensors"
META = HERE / "golden_full5_meta.json"
CACHE = REPO / ".golden_cache" / "full5"
# (key, guidance, dtype, cond_only) in priority order: the >= 40 dB bar, the CFG-6 pair, then the CFG-1 floor
TRAJ = [("10b.1344x896.s30.g1.f32", 1.0, torch.float32, True),
        ("10b.1344x896.s30.g6.f32", 6.0, torch.float32, False),
        ("10b.1344x896.s30.g6.bf16", 6.0, torch.bfloat16, False),
        ("10b.1344x896.s30.g1.bf16", 1.0, torch.bfloat16, True)]


def vae_oracle_image_tiled(z):
    """oracle/vae_ref.py tiled decode of z (= latents / scaling + shift, what reaches vae.decode; the tiling
    generate.py:77-78 enables) + pipeline.py:324-326."""
    from oracle.vae_ref import RefVAEDecoder, make_vae_state_dict, tiled_decode

    dec = RefVAEDecoder(make_vae_state_dict(seed=0))
    img = tiled_decode(dec, z.float())
    img = (img / 2 + 0.5).clamp(0, 1)
    return (img * 255).round().clamp(0, 255).to(torch.uint8).permute(0, 2, 3, 1).contiguous()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=6)
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--no-image", action="store_true")
    args = ap.parse_args()
    torch.manual_seed(1234)
    torch.set_num_threads(args.threads)
    t_start = time.time()

    def log(msg):
        print(f"[{time.time() - t_start:7.1f}s] {msg}", flush=True)

    T = load_file(str(OUT)) if OUT.exists() else {}
    meta = json.loads(META.read_text()) if META.exists() else {}
    meta.update({"generator": "oracle.weights seed=0 std=0.02 (norm weights 1); inputs hash_uniform seed 0 std 1 "
                              "(bf16-rounded) under the names below",
                 "inputs": {"ctx": [MGF.CTX_NAME, [1, 512, 4096]], "latents": [LAT_NAME, list(LAT_SHAPE)]},
                 "reference": "/root/reference f_lite/model_v2.py (10b), pipeline.py (blocks streamed)",
                 "steps": STEPS, "size": [H, W], "model": "10b (model_v2 layout)",
                 "alpha": 2 * math.sqrt((H // 8) * (W // 8) / 4096),
                 "cfg1": "cond half only, see make_golden_full4.py header",
                 "vae_image": "oracle/vae_ref.py tiled_decode (tile 128 latent / 1024 px, overlap 0.25), seed-0 "
                              "weights, on each trajectory's final latents, uint8 NHWC"})

    def save():
        meta["shapes"] = {k: list(v.shape) for k, v in T.items()}
        save_file({k: v.contiguous() for k, v in T.items()}, str(OUT))
        META.write_text(json.dumps(meta, indent=1))
        log(f"wrote {len(T)} tensors to {OUT.name}")

    def images():
        if args.no_image:
            return
        for key, _, _, _ in TRAJ:
            if f"{key}.final" in T and f"{key}.image" not in T:
                log(f"{key}: oracle VAE tiled decode")
                T[f"{key}.image"] = vae_oracle_image_tiled(T[f"{key}.final"])
                save()
        for key, _, dt, _ in TRAJ:  # the reference's own bf16 floor in image space
            base = key.rsplit(".", 1)[0]
            if dt == torch.bfloat16 and f"{key}.image" in T and f"{base}.f32.image" in T:
                a, b = T[f"{key}.image"].double(), T[f"{base}.f32.image"].double()
                meta[f"{base}.image_bf16_vs_f32_psnr"] = 10 * math.log10(255.0 ** 2 / max((a - b).pow(2).mean().item(),
                                                                                        1e-12))
                log(f"  {base} reference bf16 vs fp32 image: {meta[f'{base}.image_bf16_vs_f32_psnr']:.2f} dB")
        save()

    images()
    todo = [tr for tr in TRAJ if (args.only is None or tr[0] in args.only) and f"{tr[0]}.final" not in T]
    if todo:
        MG.install_stubs()
        model_v2 = MG.load_ref("model_v2")
        pipeline = MG.load_ref("pipeline")
        pos = MGF.hashed(MGF.CTX_NAME, (1, 512, 4096))
        neg = torch.zeros_like(pos)
        lat = MGF.hashed(LAT_NAME, LAT_SHAPE)
        with torch.no_grad():
            log("10b: generating weights")
            dit, set_dtype = MGF.stream_dit(model_v2, MGF.CFG_7B, True, log)
            fwd = V2Adapter(dit, model_v2)
            for key, g, dt, cond_only in todo:
                log(f"{key}: trajectory")
                set_dtype(dt)
                call = CachedCall(fwd, CACHE / key, cond_only, log)
                T[f"{key}.final"] = MGF.run_pipe(pipeline, call, lat.to(dt), pos.to(dt), neg.to(dt), STEPS, g,
                                                 H, W).float()
                base = key.rsplit(".", 1)[0]
                if f"{base}.f32.final" in T and f"{base}.bf16.final" in T:
                    meta[f"{base}.bf16_vs_f32_psnr"] = MGF.psnr(T[f"{base}.bf16.final"], T[f"{base}.f32.final"])
                    log(f"  {base} reference bf16 vs fp32 final latents: {meta[f'{base}.bf16_vs_f32_psnr']:.2f} dB")
                save()
                images()


if __name__ == "__main__":
    main()
