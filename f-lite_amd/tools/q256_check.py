"""Diagnostic: the 256-row attention kernel (attention_q256.hip) against a GPU fp32 reference, error per segment.

    python f-lite_amd/tools/q256_check.py [--lens 4112,4112] [--heads 12]
    FLITE_Q256_PLAN="<split tiles>,<tail chunks>" forces the split plan (env of the process).

Prints the plan-independent error of every (sequence, head, 256-row q-tile) and of the tail rows, for the q256 path
(max_k given) and the 128-row kernel (max_k = 0), relative to torch fp32 softmax(q k^T / 16) v on the GPU.
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "f-lite_amd"), str(ROOT)]

import torch  # noqa: E402

from f_lite import _native as nat  # noqa: E402

nat.attn_set_q256(True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lens", default="4112,4112")
    ap.add_argument("--heads", type=int, default=12)
    args = ap.parse_args()
    lens = [int(x) for x in args.lens.split(",")]
    H, D, B = args.heads, 256, len(lens)
    dev = torch.device("cuda", 0)
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32)
    g = torch.Generator(device=dev).manual_seed(5)

    def unit(x):
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-6)

    q = unit(torch.randn(int(cu[-1]), H, D, device=dev, generator=g)).bfloat16()
    k = unit(torch.randn(int(cu[-1]), H, D, device=dev, generator=g)).bfloat16()
    v = torch.randn(int(cu[-1]), H, D, device=dev, generator=g).bfloat16()
    ws = nat.attn_workspace(dev, B, H, max(lens), max(lens))
    a = (q, k, v, cu.to(dev), cu.to(dev), max(lens), D ** -0.5)
    new = nat.attn_varlen(*a, max_score=16.5, workspace=ws, max_k=max(lens)).float()
    cnt = int(ws[:4096].view(torch.int32).abs().sum().item())
    old = nat.attn_varlen(*a, max_score=16.5, workspace=ws).float()
    ref = torch.empty_like(new)
    for b in range(B):
        s0, s1 = int(cu[b]), int(cu[b + 1])
        for h in range(H):
            qq, kk, vv = q[s0:s1, h].float(), k[s0:s1, h].float(), v[s0:s1, h].float()
            ref[s0:s1, h] = torch.softmax(qq @ kk.T / 16.0, -1) @ vv
    print(f"counters after the q256 launch: {cnt} (0 = reset)")
    # rows of query block 1 vs block 0 of each wave in the first tile of (0, 0) (variant builds that feed block 1 the
    # block-0 queries must give equal rows)
    t = new[:256, 0].view(4, 2, 32, D)
    print("qb1 - qb0 max |diff| per wave:", [float((t[w, 1] - t[w, 0]).abs().max()) for w in range(4)])
    for row in (0, 33, 40, 63, 97):  # per 32-column block: relative error and the least-squares scale out/ref
        o, r_ = new[row, 0], ref[row, 0]
        blk = [(round(float((o[c:c + 32] - r_[c:c + 32]).norm() / r_[c:c + 32].norm()), 3),
                round(float((o[c:c + 32] * r_[c:c + 32]).sum() / (r_[c:c + 32] ** 2).sum()), 3)) for c in range(0, 256, 32)]
        print(f"row {row}: per d-tile (rel err, scale): {blk}")
    for name, out in (("q256", new), ("q128", old)):
        bad = []
        for b in range(B):
            s0, L = int(cu[b]), lens[b]
            for h in range(H):
                for t0 in range(0, L, 256):
                    t1 = min(L, t0 + 256)
                    d = (out[s0 + t0:s0 + t1, h] - ref[s0 + t0:s0 + t1, h]).norm() / ref[s0 + t0:s0 + t1, h].norm()
                    if d > 1e-2:
                        rows = (out[s0 + t0:s0 + t1, h] - ref[s0 + t0:s0 + t1, h]).norm(dim=-1) / \
                            ref[s0 + t0:s0 + t1, h].norm(dim=-1)
                        br = (rows > 1e-2).nonzero().flatten().tolist()
                        bad.append((b, h, t0, round(float(d), 4), br[:6], len(br)))
        tot = ((out - ref).norm() / ref.norm()).item()
        print(f"{name}: rel {tot:.3e}; bad tiles {len(bad)}: {bad[:24]}")


if __name__ == "__main__":
    main()
