"""Standalone timing of the attention shapes of the DiT on the 256-row kernel (attention_q256.hip) and the 128-row
kernel (attention.hip), same inputs, alternating, HIP events on the launch stream.

    python f-lite_amd/tools/q256_bench.py [--reps 50] [--rounds 3]
    (FLITE_Q256_PLAN / FLITE_Q256_MIN_KEYS in the environment steer the 256-row plan, one setting per process)

Shapes: self-attention of the metric workload (2 x 4112 tokens, 12 heads, hd 256), the 1344x896 length (4720), and
the cond-only cross-attention under the uniform-context collapse (1 x 4112 queries over 512 keys). Prints one line
per (shape, kernel): mean us per launch and TF/s (4 * Lq * Lk * hd * H * B FLOP).
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "f-lite_amd"), str(ROOT)]

import torch  # noqa: E402

from f_lite import _native as nat  # noqa: E402



def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shapes", default="self,self1344,cross", help="comma list of: self, self1344, cross, round")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    D = 256
    known = {"self": ("self 1024^2", [4112, 4112], [4112, 4112], 12),
             "self1344": ("self 1344x896", [4720, 4720], [4720, 4720], 12),
             "cross": ("cross cond-only", [4112], [512], 12),
             "round": ("one round 2x4096 H8", [4096, 4096], [4096, 4096], 8),
             "self512": ("self 512^2", [1040, 1040], [1040, 1040], 12),
             "self1536": ("self 1536^2", [9232, 9232], [9232, 9232], 12),
             "self7b": ("self 7B 1024^2", [4112, 4112], [4112, 4112], 12)}  # 256 q256 tiles = 1 round, no tail
    shapes = [known[s] for s in args.shapes.split(",")]
    g = torch.Generator(device=dev).manual_seed(3)

    def unit(x):
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-6)

    cases = []
    for name, lq, lk, H in shapes:
        cu_q = torch.tensor([0] + list(torch.tensor(lq).cumsum(0)), dtype=torch.int32, device=dev)
        cu_k = torch.tensor([0] + list(torch.tensor(lk).cumsum(0)), dtype=torch.int32, device=dev)
        q = unit(torch.randn(sum(lq), H, D, device=dev, generator=g)).bfloat16()
        k = unit(torch.randn(sum(lk), H, D, device=dev, generator=g)).bfloat16()
        v = torch.randn(sum(lk), H, D, device=dev, generator=g).bfloat16()
        ws = nat.attn_workspace(dev, len(lq), H, max(lq), max(lk))
        flops = 4.0 * sum(a * b for a, b in zip(lq, lk)) * D * H
        cases.append((name, (q, k, v, cu_q, cu_k, max(lq), D ** -0.5), ws, max(lk), flops))
    res = {}
    for r in range(args.rounds):
        for name, a, ws, mk, flops in cases:
            for kern, mode in (("q128", 0), ("q256", 1), ("auto", 2)):
                nat.attn_set_q256(mode)
                kw = dict(max_score=16.5, workspace=ws, max_k=mk)
                out = nat.attn_varlen(*a, **kw)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    nat.attn_varlen(*a, out=out, **kw)
                e1.record()
                torch.cuda.synchronize()
                res.setdefault((name, kern), []).append(e0.elapsed_time(e1) * 1000.0 / args.reps)
    for (name, kern), ts in res.items():
        flops = next(c[4] for c in cases if c[0] == name)
        best = min(ts)
        print(f"{name:18s} {kern}: {best:8.1f} us (rounds {', '.join(f'{t:.1f}' for t in ts)})  "
              f"{flops / best * 1e-6:7.1f} TF/s  frac {flops / best * 1e6 / 2.5166e15:.3f}", flush=True)


if __name__ == "__main__":
    main()
