"""Attention on tiny cases against a torch fp32 softmax reference: per-row / per-column error maps (diagnostic; used
to localise the warp-specialised variant's d-tile corruption, profiles/r05i)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from f_lite import _native as nat  # noqa: E402


def run(lq, lk, H=1, seed=0):
    torch.manual_seed(seed)
    D = 256
    q = torch.nn.functional.normalize(torch.randn(lq, H, D, device="cuda"), dim=-1).mul(16).bfloat16()
    k = torch.nn.functional.normalize(torch.randn(lk, H, D, device="cuda"), dim=-1).mul(16).bfloat16()
    v = torch.randn(lk, H, D, device="cuda").bfloat16()
    cu_q = torch.tensor([0, lq], dtype=torch.int32, device="cuda")
    cu_k = torch.tensor([0, lk], dtype=torch.int32, device="cuda")
    o = nat.attn_varlen(q, k, v, cu_q, cu_k, lq, D ** -0.5, max_score=16.5, max_k=lk)
    torch.cuda.synchronize()
    ref = torch.softmax(torch.einsum("qhd,khd->hqk", q.float(), k.float()) * D ** -0.5, -1)
    ref = torch.einsum("hqk,khd->qhd", ref, v.float())
    return o.float(), ref


for lq, lk in ((64, 1), (64, 64), (128, 64), (128, 128), (200, 300)):
    o, ref = run(lq, lk)
    err = (o - ref).abs().max().item()
    rel = ((o - ref).norm() / ref.norm()).item()
    print(f"lq {lq} lk {lk}: max abs {err:.3e} rel {rel:.3e}", flush=True)
    if lk == 1:
        print("  row0 o[:8]", o[0, 0, :8].tolist())
        print("  ref[:8]   ", ref[0, 0, :8].tolist())
        ratio = (o[:, 0, :] / ref[:, 0, :]).median().item()
        print("  median ratio", ratio)
    bad = ((o - ref).abs().amax(dim=(1, 2)) > 0.05).nonzero().flatten().tolist()
    print("  bad rows", bad[:20], len(bad))
    badd = ((o - ref).abs().amax(dim=(0, 1)) > 0.05).nonzero().flatten().tolist()
    print("  bad cols", badd[:40], len(badd))
