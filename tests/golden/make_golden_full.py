"""Full-size golden fixtures (SURVEY §8c fixture set iii) from the REFERENCE, at full 40-block depth.

Run in the build container only (it needs /root/reference; about 20 min of CPU and ~30 GB of RAM):

    python tests/golden/make_golden_full.py

The reference modules are stub-loaded exactly as in make_golden.py (same stubs for the absent third-party
packages). To fit a 7B / 10B model in fp32 next to its activations, the blocks are STREAMED: the reference
DiT is built with depth=0 (context_proj, patch_embed, rope, time_embed, adaLN, final stage) and its
`blocks` list is filled with proxies; proxy i copies block i's weights (kept once, in bf16 -- every generator
value is bf16-representable, so the copy into an fp32 block is exact) into ONE shared reference DiTBlock and
calls it. DiT.forward (model.py:525-591), DiTBlock.forward (model.py:270-303 / model_v2.py:274-309) and the
pipeline loop (pipeline.py:187-331) are the reference's own code; only the 10B-v2 top level uses
make_golden.v2_forward_fixed (the v2 file cannot run as published).

Inputs are regenerated, not stored: weights from oracle.weights (seed 0, std 0.02, norm weights 1), the
context and latents from the same hash generator under the names below (seed 0, std 1), bf16-rounded, so the
GPU tests rebuild them bit-identically with flite_init_param.

Timesteps: the fp32 runs feed the DiT bf16 timesteps (the t_tensor a bf16 pipeline creates at
pipeline.py:260, quantised again by timesteps * 1000 at model.py:551), as the GPU path does -- SURVEY §0.5.

Fixtures (tests/golden/golden_full.safetensors, ~4 MB) + golden_full_meta.json:
  7b.256.f32.final       7B, 256x256, 4 steps, CFG 6: final latents / scaling + shift (pipeline.py:304), fp32
  7b.256.bf16.final      the same in the reference's bf16 arithmetic (its own rounding floor vs fp32)
  7b.256.step{k}.x / .t / .out   the 4 teacher-forcing points of the fp32 run: the CFG-batched DiT input
                         [2,16,32,32], its timestep and the raw [uncond, cond] output (fp32)
  7b.1024.out            one CFG-batched 7B forward at 1024x1024 (T = 4112), fp32, [2,16,128,128]
  10b.1024.out           the same for the 10B model_v2 layout
"""
from __future__ import annotations

import sys

sys.dont_write_bytecode = True

import json  # noqa: E402
import math  # noqa: E402
import time  # noqa: E402
from pathlib import Path  # noqa: E402

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
from safetensors.torch import save_file  # noqa: E402

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
import make_golden as MG  # noqa: E402

from oracle.weights import hash_uniform, make_param, param_shapes  # noqa: E402

CFG_7B = dict(in_channels=16, patch_size=2, hidden_size=3072, depth=40, num_heads=12, mlp_ratio=4.0,
              cross_attn_input_size=4096, train_bias_and_rms=True, use_rope=True, gradient_checkpoint=False,
              dynamic_softmax_temperature=False, rope_base=10000)
CTX_NAME = "golden.ctx"            # [1, 512, 4096]
LAT256_NAME = "golden.latents.256"  # [1, 16, 32, 32]
LAT1024_NAME = "golden.latents.1024"  # [1, 16, 128, 128]
T_1024 = 0.75                      # timestep of the 1024^2 forward (bf16: 0.75 exactly)


def hashed(name, shape, std=1.0):
    n = math.prod(shape)
    return torch.from_numpy(hash_uniform(name, n, std, 0)).reshape(shape).to(torch.bfloat16).float()


class StreamBlock(nn.Module):
    """Proxy for reference block i: load its bf16 weights into the shared reference DiTBlock and call it."""

    def __init__(self, idx, weights, shared):
        super().__init__()
        self.idx = idx
        self._w = weights  # plain dict attributes: not parameters of the proxy
        self._shared = shared

    def forward(self, *args):
        blk = self._shared["block"]
        with torch.no_grad():
            for n, p in blk.named_parameters():
                p.copy_(self._w[n])
        return blk(*args)


def stream_dit(model_mod, cfg, per_block, log):
    """Reference DiT with streamed blocks; returns (dit, set_dtype) where set_dtype(dt) casts it and builds the
    shared blocks in dtype dt."""
    shapes = param_shapes(dict(cfg, per_block_adaln=per_block))
    top_cfg = dict(cfg, depth=0)
    dit = model_mod.DiT(**top_cfg)
    top = {k: make_param(k, v) for k, v in shapes.items() if not k.startswith("blocks.")}
    missing, unexpected = dit.load_state_dict(top, strict=True)
    assert not missing and not unexpected
    D = cfg["hidden_size"]
    blocks = []
    shared_by_kind = {}
    t0 = time.time()
    for i in range(cfg["depth"]):
        pre = f"blocks.{i}."
        cross = True if per_block else (i % 4 == 0 or i < 8)
        w = {k[len(pre):]: make_param(k, v).to(torch.bfloat16) for k, v in shapes.items() if k.startswith(pre)}
        shared = shared_by_kind.setdefault(cross, {})
        blocks.append(StreamBlock(i, w, shared))
        if i % 8 == 0:
            log(f"  weights of block {i} generated ({time.time() - t0:.0f} s)")
    dit.blocks = nn.ModuleList(blocks)
    # inventory check: every block's generated names are exactly a reference DiTBlock's state dict
    for cross in shared_by_kind:
        ref_blk = model_mod.DiTBlock(hidden_size=D, num_heads=cfg["num_heads"], mlp_ratio=cfg["mlp_ratio"],
                                     do_cross_attn=cross, qkv_bias=cfg["train_bias_and_rms"])
        i = next(b.idx for b in blocks if (True if per_block else (b.idx % 4 == 0 or b.idx < 8)) == cross)
        names = set(blocks[i]._w)
        assert names == set(ref_blk.state_dict().keys()), (cross, names ^ set(ref_blk.state_dict().keys()))

    def set_dtype(dt):
        dit.to(dt)
        for cross, shared in shared_by_kind.items():
            shared["block"] = model_mod.DiTBlock(hidden_size=D, num_heads=cfg["num_heads"],
                                                 mlp_ratio=cfg["mlp_ratio"], do_cross_attn=cross,
                                                 qkv_bias=cfg["train_bias_and_rms"]).to(dt).eval()
        return dit

    return dit, set_dtype


class RecordingThreeArg(nn.Module):
    """pipeline.py:271's 3-argument call -> DiT.forward(x, ctx, None, t); feeds bf16 timesteps
    (the bf16 pipeline's t_tensor) and records every call's input, timestep and raw output."""

    def __init__(self, dit, record):
        super().__init__()
        self.dit = dit
        self.record = record

    def forward(self, x, ctx, t):
        out = self.dit(x, ctx, None, t.to(torch.bfloat16))
        if self.record is not None:
            self.record.append((x.detach().float().clone(), t.detach().float().clone(), out.detach().float().clone()))
        return out


def run_pipe(pipeline_mod, dit, latents, pos, neg, steps, guidance, height, width, record=None):
    vae = MG.StubVAE(latents.dtype)
    pipe = pipeline_mod.FLitePipeline(RecordingThreeArg(dit, record), vae, MG.StubEncoder(), None)
    pipe.encode_prompt = lambda **kw: (pos.to(kw.get("dtype")), neg.to(kw.get("dtype")))
    pipeline_mod.randn_tensor = lambda shape, generator=None, device=None, dtype=None: latents.clone().to(dtype)
    pipe.set_progress_bar_config(disable=True)
    pipe(prompt="x", height=height, width=width, num_inference_steps=steps, guidance_scale=guidance)
    return vae.seen


def psnr(a, ref):
    mse = (a.double() - ref.double()).pow(2).mean().item()
    peak = ref.double().abs().max().item()
    return float("inf") if mse == 0 else 10 * math.log10(peak * peak / mse)


def main():
    torch.manual_seed(1234)
    torch.set_num_threads(8)
    t_start = time.time()

    def log(msg):
        print(f"[{time.time() - t_start:7.1f}s] {msg}", flush=True)

    MG.install_stubs()
    model = MG.load_ref("model")
    model_v2 = MG.load_ref("model_v2")
    pipeline = MG.load_ref("pipeline")
    T = {}
    meta = {"generator": "oracle.weights seed=0 std=0.02 (norm weights 1); inputs hash_uniform seed 0 std 1 "
                         "(bf16-rounded) under the names below",
            "inputs": {"ctx": [CTX_NAME, [1, 512, 4096]], "latents_256": [LAT256_NAME, [1, 16, 32, 32]],
                       "latents_1024": [LAT1024_NAME, [1, 16, 128, 128]]},
            "reference": "/root/reference f_lite/model.py, model_v2.py, pipeline.py (blocks streamed, see header)",
            "timesteps": "bf16 (pipeline.py:260 in a bf16 model) fed to an fp32 model"}
    pos = hashed(CTX_NAME, (1, 512, 4096))
    neg = torch.zeros_like(pos)

    with torch.no_grad():
        # ---------------- 7B (model.py layout) ----------------
        log("7B: generating weights")
        dit, set_dtype = stream_dit(model, CFG_7B, False, log)
        set_dtype(torch.float32)
        lat = hashed(LAT256_NAME, (1, 16, 32, 32))
        rec = []
        log("7B 256^2 4-step fp32 trajectory")
        T["7b.256.f32.final"] = run_pipe(pipeline, dit, lat, pos, neg, 4, 6.0, 256, 256, rec)
        for k, (x, t, out) in enumerate(rec):
            T[f"7b.256.step{k}.x"] = x
            T[f"7b.256.step{k}.t"] = t
            T[f"7b.256.step{k}.out"] = out
        log("7B 1024^2 one CFG-batched forward, fp32")
        lat1024 = hashed(LAT1024_NAME, (1, 16, 128, 128))
        x2 = torch.cat([lat1024] * 2)
        ctx2 = torch.cat([neg, pos])
        t2 = torch.tensor([T_1024] * 2, dtype=torch.bfloat16)
        T["7b.1024.out"] = dit(x2, ctx2, None, t2).float()
        log("7B 256^2 4-step bf16 trajectory (reference rounding)")
        set_dtype(torch.bfloat16)
        T["7b.256.bf16.final"] = run_pipe(pipeline, dit, lat.bfloat16(), pos.bfloat16(), neg.bfloat16(), 4, 6.0,
                                          256, 256).float()
        meta["7b.256.bf16_vs_f32_psnr"] = psnr(T["7b.256.bf16.final"], T["7b.256.f32.final"])
        log(f"  reference bf16 vs fp32 final latents: {meta['7b.256.bf16_vs_f32_psnr']:.2f} dB")
        del dit, set_dtype

        # ---------------- 10B (model_v2.py layout, repaired final stage) ----------------
        log("10B: generating weights")
        cfg10 = dict(CFG_7B)
        dv2, set_dtype = stream_dit(model_v2, cfg10, True, log)
        set_dtype(torch.float32)
        log("10B 1024^2 one CFG-batched forward, fp32")
        T["10b.1024.out"] = MG.v2_forward_fixed(dv2, model_v2, x2, ctx2, None, t2).float()
        del dv2, set_dtype

    meta["t_1024"] = T_1024
    meta["shapes"] = {k: list(v.shape) for k, v in T.items()}
    T = {k: v.contiguous().float() for k, v in T.items()}
    save_file(T, str(HERE / "golden_full.safetensors"))
    (HERE / "golden_full_meta.json").write_text(json.dumps(meta, indent=1))
    log(f"wrote {len(T)} tensors, {sum(v.numel() for v in T.values()) * 4 / 1e6:.1f} MB")


if __name__ == "__main__":
    main()
