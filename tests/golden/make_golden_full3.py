"""Full-depth P3 fixtures at the metric's 30 steps (SURVEY §8d parity protocol P3: "report final-latent PSNR vs the
fp32 oracle at CFG 6 next to the reference's own floor, and at CFG 1, where the >= 40 dB bar applies").

Run in the build container only (needs /root/reference; about 2-3 h of CPU on 8 cores, ~35 GB of RAM):

    python tests/golden/make_golden_full3.py

Same stub-loading and block streaming as make_golden_full.py (the reference's own DiT.forward, DiTBlock.forward
and FLitePipeline.__call__; the 10B-v2 top level is make_golden.v2_forward_fixed), at 256^2 so the
30-step trajectories finish on the CPU.

Fixtures (tests/golden/golden_full3.safetensors) + golden_full3_meta.json, for M in {7b, 10b}, G in {6, 1}:
  {M}.256.s30.g{G}.f32.final    30-step trajectory, CFG G, fp32 reference arithmetic: final latents / scaling +
                                shift (pipeline.py:304)
  {M}.256.s30.g{G}.bf16.final   the same run in the reference's bf16 arithmetic (its own floor vs fp32)
Inputs: the prompt context and 256^2 latents of make_golden_full.py (golden.ctx, golden.latents.256).
"""
from __future__ import annotations

import sys

sys.dont_write_bytecode = True

import json  # noqa: E402
import time  # noqa: E402
from pathlib import Path  # noqa: E402

import torch  # noqa: E402
from safetensors.torch import save_file  # noqa: E402

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
import make_golden as MG  # noqa: E402
import make_golden_full as MGF  # noqa: E402
from make_golden_full2 import V2Adapter  # noqa: E402

STEPS = 30
GUIDANCE = (6.0, 1.0)


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
            "inputs": {"ctx": [MGF.CTX_NAME, [1, 512, 4096]], "latents_256": [MGF.LAT256_NAME, [1, 16, 32, 32]]},
            "reference": "/root/reference f_lite/model.py, model_v2.py, pipeline.py (blocks streamed)",
            "steps": STEPS, "guidance": list(GUIDANCE), "size": [256, 256]}
    pos = MGF.hashed(MGF.CTX_NAME, (1, 512, 4096))
    neg = torch.zeros_like(pos)
    lat = MGF.hashed(MGF.LAT256_NAME, (1, 16, 32, 32))

    with torch.no_grad():
        for name, mod, per_block in (("7b", model, False), ("10b", model_v2, True)):
            log(f"{name}: generating weights")
            dit, set_dtype = MGF.stream_dit(mod, MGF.CFG_7B, per_block, log)
            fwd = V2Adapter(dit, model_v2) if per_block else dit
            for g in GUIDANCE:
                key = f"{name}.256.s{STEPS}.g{g:g}"
                log(f"{key}: fp32 trajectory")
                set_dtype(torch.float32)
                T[f"{key}.f32.final"] = MGF.run_pipe(pipeline, fwd, lat, pos, neg, STEPS, g, 256, 256).float()
                log(f"{key}: bf16 trajectory (reference rounding)")
                set_dtype(torch.bfloat16)
                T[f"{key}.bf16.final"] = MGF.run_pipe(pipeline, fwd, lat.bfloat16(), pos.bfloat16(), neg.bfloat16(),
                                                      STEPS, g, 256, 256).float()
                meta[f"{key}.bf16_vs_f32_psnr"] = MGF.psnr(T[f"{key}.bf16.final"], T[f"{key}.f32.final"])
                log(f"  {key} reference bf16 vs fp32 final latents: {meta[f'{key}.bf16_vs_f32_psnr']:.2f} dB")
                # checkpoint after every trajectory pair, so a late failure keeps what is done
                meta["shapes"] = {k: list(v.shape) for k, v in T.items()}
                save_file({k: v.contiguous().float() for k, v in T.items()}, str(HERE / "golden_full3.safetensors"))
                (HERE / "golden_full3_meta.json").write_text(json.dumps(meta, indent=1))
                log(f"wrote {len(T)} tensors")
            del dit, set_dtype, fwd


if __name__ == "__main__":
    main()
