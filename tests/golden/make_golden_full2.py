"""Full-size P2 / P3 fixtures at 1024^2 (SURVEY §8c fixture set iv, §8d "re-measure P2 at T = 4112").

Run in the build container only (needs /root/reference; about 1.5 h of CPU on 8 cores, ~40 GB of RAM):

    python tests/golden/make_golden_full2.py

Same stub-loading and block streaming as make_golden_full.py (the reference's own DiT.forward, DiTBlock.forward
and FLitePipeline.__call__; the 10B-v2 top level is make_golden.v2_forward_fixed).

Fixtures (tests/golden/golden_full2.safetensors) + golden_full2_meta.json, for M in {7b, 10b}:
  {M}.1024.tf{t}.out     P2 teacher-forced single step at t in {1.0, 0.5, 0.1}: the CFG-batched [uncond, cond]
                         raw DiT output (fp32, [2,16,128,128]) on the input
                             x_t = bf16( t * noise + (1 - t) * x0 )    (fp32 arithmetic, then one bf16 rounding)
                         with noise = hashed(latents_1024) and x0 = hashed(x0_1024); the GPU test rebuilds x_t
                         with the same two torch ops on the CPU.
  {M}.1024.f32.final     P3 free-running 4-step CFG-6 trajectory at 1024^2 (alpha = 4): final latents /
                         scaling + shift (pipeline.py:304), fp32 reference arithmetic
  {M}.1024.bf16.final    the same run in the reference's bf16 arithmetic (its own floor vs fp32)
"""
from __future__ import annotations

import sys

sys.dont_write_bytecode = True

import json  # noqa: E402
import time  # noqa: E402
from pathlib import Path  # noqa: E402

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
from safetensors.torch import save_file  # noqa: E402

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
import make_golden as MG  # noqa: E402
import make_golden_full as MGF  # noqa: E402

X0_NAME = "golden.x0.1024"  # [1, 16, 128, 128]
TF_TIMES = (1.0, 0.5, 0.1)
STEPS = 4


def teacher_input(noise, x0, t):
    """x_t = bf16(t * noise + (1 - t) * x0), fp32 arithmetic (the GPU test repeats these exact ops)."""
    return (noise * t + x0 * (1.0 - t)).to(torch.bfloat16).float()


class V2Adapter(nn.Module):
    """DiT.forward-shaped (x, ctx, mask, t) call into the repaired v2 top level."""

    def __init__(self, dit, model_v2):
        super().__init__()
        self.dit = dit
        self._m = model_v2

    def forward(self, x, ctx, mask, t):
        return MG.v2_forward_fixed(self.dit, self._m, x, ctx, mask, t)


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
            "inputs": {"ctx": [MGF.CTX_NAME, [1, 512, 4096]], "latents_1024": [MGF.LAT1024_NAME, [1, 16, 128, 128]],
                       "x0_1024": [X0_NAME, [1, 16, 128, 128]]},
            "teacher_input": "x_t = bf16(t * noise + (1 - t) * x0) in fp32 arithmetic; noise = latents_1024",
            "reference": "/root/reference f_lite/model.py, model_v2.py, pipeline.py (blocks streamed)",
            "timesteps": "bf16 (pipeline.py:260 in a bf16 model) fed to an fp32 model",
            "tf_times": list(TF_TIMES), "steps": STEPS, "guidance": 6.0}
    pos = MGF.hashed(MGF.CTX_NAME, (1, 512, 4096))
    neg = torch.zeros_like(pos)
    ctx2 = torch.cat([neg, pos])
    noise = MGF.hashed(MGF.LAT1024_NAME, (1, 16, 128, 128))
    x0 = MGF.hashed(X0_NAME, (1, 16, 128, 128))

    with torch.no_grad():
        for name, mod, per_block in (("7b", model, False), ("10b", model_v2, True)):
            log(f"{name}: generating weights")
            dit, set_dtype = MGF.stream_dit(mod, MGF.CFG_7B, per_block, log)
            set_dtype(torch.float32)
            fwd = V2Adapter(dit, model_v2) if per_block else dit
            for t in TF_TIMES:
                log(f"{name} 1024^2 teacher-forced forward at t={t}")
                x = teacher_input(noise, x0, t)
                t2 = torch.tensor([t] * 2, dtype=torch.bfloat16)
                T[f"{name}.1024.tf{t}.out"] = fwd(torch.cat([x, x]), ctx2, None, t2).float()
            log(f"{name} 1024^2 {STEPS}-step CFG-6 trajectory, fp32")
            T[f"{name}.1024.f32.final"] = MGF.run_pipe(pipeline, fwd, noise, pos, neg, STEPS, 6.0, 1024, 1024).float()
            log(f"{name} 1024^2 {STEPS}-step CFG-6 trajectory, bf16 (reference rounding)")
            set_dtype(torch.bfloat16)
            T[f"{name}.1024.bf16.final"] = MGF.run_pipe(pipeline, fwd, noise.bfloat16(), pos.bfloat16(),
                                                        neg.bfloat16(), STEPS, 6.0, 1024, 1024).float()
            meta[f"{name}.1024.bf16_vs_f32_psnr"] = MGF.psnr(T[f"{name}.1024.bf16.final"],
                                                             T[f"{name}.1024.f32.final"])
            log(f"  {name} reference bf16 vs fp32 final latents: {meta[f'{name}.1024.bf16_vs_f32_psnr']:.2f} dB")
            del dit, set_dtype, fwd
            # checkpoint what we have, so a late failure keeps the 7B half
            meta["shapes"] = {k: list(v.shape) for k, v in T.items()}
            save_file({k: v.contiguous().float() for k, v in T.items()}, str(HERE / "golden_full2.safetensors"))
            (HERE / "golden_full2_meta.json").write_text(json.dumps(meta, indent=1))
            log(f"wrote {len(T)} tensors")


if __name__ == "__main__":
    main()
