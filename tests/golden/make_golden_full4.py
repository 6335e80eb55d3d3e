"""The METRIC configuration pinned end to end (VERDICT r03 "next 1"; SURVEY §8c fixture set iv, §8d P3).

Run in the build container only (needs /root/reference; ~6-8 h of CPU, ~40 GB of RAM; resumable):

    python tests/golden/make_golden_full4.py [--threads 6] [--only KEY ...] [--no-image]

Same stub-loading and block streaming as make_golden_full.py (the reference's own DiT.forward, DiTBlock.forward
and FLitePipeline.__call__; the 10B-v2 top level is make_golden.v2_forward_fixed), at the metric's
own size: 10B (model_v2 layout), 1024^2 (T = 4112), 30 steps, alpha from pipeline.py:241-242.

Resumable: every DiT call's output is cached on disk (.golden_cache/full4/<traj>/<call>.pt, keyed by a checksum of
the call's input, so a resumed pipeline replays the finished steps and recomputes from the first missing one).

Fixtures (tests/golden/golden_full4.safetensors) + golden_full4_meta.json:
  10b.1024.s30.g6.f32.final    30-step CFG-6 trajectory in the reference's fp32 arithmetic: final latents / scaling
                               + shift (pipeline.py:304), i.e. exactly what reaches vae.decode
  10b.1024.s30.g6.bf16.final   the same run in the reference's bf16 arithmetic (its own floor vs fp32)
  10b.1024.s30.g1.f32.final    CFG 1 (pipeline.py:248: guidance >= 1 still runs the CFG batch), fp32
  7b.1024.s30.g1.f32.final     BASELINE configs[1]'s model (7B, model.py layout) at CFG 1, fp32 (when time allows)
  7b.1024.s30.g6.f32.final     7B at CFG 6 (configs[1] itself), fp32 (when time allows)
  10b.1024.s30.g1.bf16.final   CFG 1, bf16 (when time allows)
  7b.1024.s30.g6.bf16.final    configs[1] in the reference's bf16 arithmetic: the configs[1] floor (round 5)
  {key}.image                  uint8 [1, 1024, 1024, 3]: oracle/vae_ref.py (the restated Flux decoder, seed-0
                               generator weights) on that trajectory's final latents + pipeline.py:324-326; the
                               bf16 runs' images give the reference's own image-space floor (meta *.image_bf16_vs_f32).
                               Made right after each trajectory (and first, for finals that lack one).

CFG 1 shortcut (stated): at guidance 1 pipeline.py:290 forms uncond + 1 * (cond - uncond). The wrapper below runs
the reference DiT on the cond half only and hands the pipeline [cond, cond], so the combination returns cond
exactly; the reference's own batch-2 call returns cond up to one fp32 rounding of (uncond + (cond - uncond)),
~1e-7 relative, 100+ dB below the 40 dB bar. The uncond rows never influence the cond rows in the reference
(varlen attention per sequence, row-wise norms), so the cond half is the same computation. It halves the CPU cost.
"""
from __future__ import annotations

import sys

sys.dont_write_bytecode = True

import argparse  # noqa: E402
import hashlib  # noqa: E402
import json  # noqa: E402
import math  # noqa: E402
import time  # noqa: E402
from pathlib import Path  # noqa: E402

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
from safetensors.torch import load_file, save_file  # noqa: E402

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(REPO))
import make_golden as MG  # noqa: E402
import make_golden_full as MGF  # noqa: E402
from make_golden_full2 import V2Adapter  # noqa: E402

STEPS = 30
OUT = HERE / "golden_full4.safetensors"
META = HERE / "golden_full4_meta.json"
CACHE = REPO / ".golden_cache" / "full4"
# (key, guidance, dtype, cond_only), in priority order: the >= 40 dB bar first, then the CFG-6 pair, then 7B
# (model.py layout, BASELINE configs[1]) and the CFG-1 floor; the model is the key's first field
TRAJ = [("10b.1024.s30.g1.f32", 1.0, torch.float32, True),
        ("10b.1024.s30.g6.f32", 6.0, torch.float32, False),
        ("10b.1024.s30.g6.bf16", 6.0, torch.bfloat16, False),
        ("7b.1024.s30.g1.f32", 1.0, torch.float32, True),
        ("7b.1024.s30.g6.f32", 6.0, torch.float32, False),
        ("10b.1024.s30.g1.bf16", 1.0, torch.bfloat16, True),
        ("7b.1024.s30.g6.bf16", 6.0, torch.bfloat16, False)]


def _digest(*ts):
    h = hashlib.sha1()
    for t in ts:
        h.update(t.detach().contiguous().float().numpy().tobytes())
    return h.hexdigest()


class CachedCall(nn.Module):
    """DiT.forward-shaped call with an on-disk cache per call index (input checksum verified on replay)."""

    def __init__(self, fwd, cache_dir, cond_only, log):
        super().__init__()
        self.fwd = fwd
        self.dir = cache_dir
        self.dir.mkdir(parents=True, exist_ok=True)
        self.cond_only = cond_only
        self.k = 0
        self.log = log

    def forward(self, x, ctx, mask, t):
        key = _digest(x, ctx, t)
        f = self.dir / f"{self.k:03d}.pt"
        self.k += 1
        if f.exists():
            rec = torch.load(f, weights_only=True)
            if rec["key"] == key:
                return rec["out"].to(x.dtype)
            self.log(f"    cache {f.name}: input changed, recomputing")
        t0 = time.time()
        if self.cond_only:
            assert x.shape[0] == 2
            oc = self.fwd(x[1:], ctx[1:], mask, t[1:])
            out = torch.cat([oc, oc])
        else:
            out = self.fwd(x, ctx, mask, t)
        torch.save({"key": key, "out": out.detach().clone()}, f)
        self.log(f"    call {self.k - 1} ({'cond only' if self.cond_only else 'CFG batch'}, t={float(t[0]):.4f}, "
                 f"{x.dtype}): {time.time() - t0:.0f} s")
        return out


def vae_oracle_image(z):
    """oracle/vae_ref.py decode of z (= latents / scaling + shift, what reaches vae.decode) + pipeline.py:324-326."""
    from oracle.vae_ref import RefVAEDecoder, make_vae_state_dict

    img = RefVAEDecoder(make_vae_state_dict(seed=0)).decode(z.float())
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
                 "inputs": {"ctx": [MGF.CTX_NAME, [1, 512, 4096]],
                            "latents_1024": [MGF.LAT1024_NAME, [1, 16, 128, 128]]},
                 "reference": "/root/reference f_lite/model.py (7b), model_v2.py (10b), pipeline.py (blocks streamed)",
                 "steps": STEPS, "size": [1024, 1024], "model": "key prefix: 10b (model_v2 layout), 7b (model.py)",
                 "cfg1": "cond half only, see make_golden_full4.py header",
                 "vae_image": "oracle/vae_ref.py seed-0 weights on each trajectory's final latents, uint8 NHWC"})

    def save():
        meta["shapes"] = {k: list(v.shape) for k, v in T.items()}
        save_file({k: v.contiguous() for k, v in T.items()}, str(OUT))
        META.write_text(json.dumps(meta, indent=1))
        log(f"wrote {len(T)} tensors to {OUT.name}")

    def images():
        if args.no_image:
            return
        for key, _, dt, _ in TRAJ:
            if f"{key}.final" in T and f"{key}.image" not in T:
                log(f"{key}: oracle VAE decode")
                T[f"{key}.image"] = vae_oracle_image(T[f"{key}.final"])
                save()
        for key, _, dt, _ in TRAJ:  # the reference's own bf16 floor in image space (P3 image metric)
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
        mods = {"7b": (MG.load_ref("model"), False), "10b": (MG.load_ref("model_v2"), True)}
        model_v2 = mods["10b"][0]
        pipeline = MG.load_ref("pipeline")
        pos = MGF.hashed(MGF.CTX_NAME, (1, 512, 4096))
        neg = torch.zeros_like(pos)
        lat = MGF.hashed(MGF.LAT1024_NAME, (1, 16, 128, 128))
        loaded, fwd, set_dtype = None, None, None
        with torch.no_grad():
            for key, g, dt, cond_only in todo:
                name = key.split(".")[0]
                if name != loaded:  # one model's streamed weights at a time (~40 GB)
                    fwd = set_dtype = dit = None
                    log(f"{name}: generating weights")
                    mod, per_block = mods[name]
                    dit, set_dtype = MGF.stream_dit(mod, MGF.CFG_7B, per_block, log)
                    fwd = V2Adapter(dit, model_v2) if per_block else dit
                    loaded = name
                log(f"{key}: trajectory")
                set_dtype(dt)
                call = CachedCall(fwd, CACHE / key, cond_only, log)
                T[f"{key}.final"] = MGF.run_pipe(pipeline, call, lat.to(dt), pos.to(dt), neg.to(dt), STEPS, g,
                                                 1024, 1024).float()
                base = key.rsplit(".", 1)[0]
                if f"{base}.f32.final" in T and f"{base}.bf16.final" in T:
                    meta[f"{base}.bf16_vs_f32_psnr"] = MGF.psnr(T[f"{base}.bf16.final"], T[f"{base}.f32.final"])
                    log(f"  {base} reference bf16 vs fp32 final latents: {meta[f'{base}.bf16_vs_f32_psnr']:.2f} dB")
                save()
                images()


if __name__ == "__main__":
    main()
