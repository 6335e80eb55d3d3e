"""Per-rank compute of the CFG-parallel latency mode (distributed.cfg_parallel_sample), measured on one GPU.

A 2-GPU run is not available on the single-GPU box, so this times what one rank of the pair does: 30 DiT
forwards of ONE branch (batch 1, M = T rows per GEMM) plus the flite_cfg_euler update, eagerly, for the 10B
model at 1024^2. Beside it, the batched CFG loop (batch 2, M = 2T) runs eagerly and as a hipGraph. The
all-gather of the branch outputs (1 MiB fp32 per step) is not included. The 2-GPU latency of the denoise loop
is then roughly the branch time plus 30 exchanges.

    python f-lite_amd/tools/cfgpar_branch_time.py [--model 10b] [--height 1024 --width 1024] [--reps 2]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from f_lite import DiT  # noqa: E402
from f_lite import _native as nat  # noqa: E402
from f_lite.model import PRESETS  # noqa: E402
from f_lite.pipeline import flow_schedule  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="10b")
    ap.add_argument("--height", type=int, default=1024)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = dict(PRESETS[args.model])
    m = DiT.random(seed=0, device=dev, **cfg)
    eng = m.engine()
    L = 512
    ctx = nat.init_param_(torch.empty(1, L, cfg["cross_attn_input_size"], device=dev, dtype=torch.bfloat16),
                          "synthetic.t5_context", seed=1, std=1.0)
    lh, lw = args.height // 8, args.width // 8
    lat = nat.init_param_(torch.empty(1, 16, lh, lw, device=dev, dtype=torch.bfloat16), "synthetic.latents.0",
                          seed=2, std=1.0)
    sched = flow_schedule(args.steps, lh, lw)
    t_list = [t for t, _ in sched]
    dt_list = [dt for _, dt in sched]

    # batched CFG loop (what bench.py runs): batch 2 = [uncond; cond]
    eng.prepare(2, lh, lw, 2 * L, args.steps)
    eng.set_context(torch.cat([torch.zeros_like(ctx), ctx]).reshape(2 * L, -1).contiguous(), [0, L, 2 * L])
    acc = lat.float().contiguous()

    def batched(graph):
        return lambda: eng.sample(acc.clone(), 1, t_list, dt_list, 6.0, True, use_graph=graph)

    t_batched_eager = timed(batched(False), args.reps)
    t_batched_graph = timed(batched(True), args.reps)

    # one CFG-parallel rank: batch 1, its branch's context, the same timesteps
    eng.prepare(1, lh, lw, L, args.steps)
    eng.set_context(ctx.reshape(L, -1).contiguous(), [0, L])
    eng.set_timesteps(torch.tensor(t_list, dtype=torch.float32, device=dev), True)
    out = torch.empty_like(acc)

    def branch():
        a = acc.clone()
        for i, dt in enumerate(dt_list):
            eng.forward(a, out, i, 0)
            nat.cfg_euler_(a, out, out, 6.0, dt)  # the peer's output would arrive here
        return a

    t_branch = timed(branch, args.reps)
    print(json.dumps({
        "workload": f"{args.model} {args.width}x{args.height}, {args.steps} steps, DiT loop only (no VAE)",
        "batched_cfg_loop_eager_s": round(t_batched_eager, 4),
        "batched_cfg_loop_graph_s": round(t_batched_graph, 4),
        "cfg_parallel_one_rank_eager_s": round(t_branch, 4),
        "branch_vs_batched_eager": round(t_branch / t_batched_eager, 4),
        "note": "one rank of the CFG-parallel pair; the per-step all-gather (1 MiB fp32) is not included",
    }))


if __name__ == "__main__":
    main()
