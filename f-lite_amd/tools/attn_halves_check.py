"""Key halves in the 128-row attention kernel: accuracy and timing. Measured in round 5 and not kept: apply
`profiles/r05p/attn_key_halves.patch` and rebuild first; without it FLITE_ATTN_HALVES does nothing.

    FLITE_ATTN_HALVES=<n> python f-lite_amd/tools/attn_halves_check.py check   # n q-tiles halved (forced), every case
    python f-lite_amd/tools/attn_halves_check.py time                          # the launcher's own plan
    FLITE_ATTN_HALVES=<n> python f-lite_amd/tools/attn_halves_check.py time    # a forced count (sweep)

check: tools/attn_equal.py's cases with a workspace sized by flite_attn_workspace_bytes_for, vs a torch fp32
reference (rel-L2, as attn_m16_check.py) and vs the same launch without halves (FLITE_ATTN_HALVES=0 in a second
process: `dump` / `compare` like attn_equal.py). time: the cond-only cross-attention of the collapsed 1024^2 loop
(1 sequence x 12 heads, 4112 queries, 512 keys), the CFG-pair cross-attention (2 sequences) and the self-attention.
"""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parent))
import torch
from attn_equal import CASES
from attn_m16_check import reference
from f_lite import _native as nat

dev = "cuda"
D = 256


def outputs():
    outs, rels = [], []
    for lens_q, lens_k, H, split in CASES:
        lens_k = lens_q if lens_k is None else lens_k
        cu_q = torch.tensor([0] + list(torch.tensor(lens_q).cumsum(0)), dtype=torch.int32)
        cu_k = torch.tensor([0] + list(torch.tensor(lens_k).cumsum(0)), dtype=torch.int32)
        g = torch.Generator(device=dev).manual_seed(sum(lens_q) + H)
        q = torch.nn.functional.normalize(torch.randn(int(cu_q[-1]), H, D, device=dev, generator=g), dim=-1)
        k = torch.nn.functional.normalize(torch.randn(max(int(cu_k[-1]), 1), H, D, device=dev, generator=g), dim=-1)
        v = torch.randn(max(int(cu_k[-1]), 1), H, D, device=dev, generator=g).bfloat16()
        q, k = (q * 16).bfloat16(), (k * 16).bfloat16()
        ws = nat.attn_workspace(dev, len(lens_q), H, max(lens_q), max(lens_k)) if split else None
        o = nat.attn_varlen(q, k, v, cu_q.to(dev), cu_k.to(dev), max(lens_q), D ** -0.5, max_score=16.5, workspace=ws,
                            max_k=max(lens_k))
        ref = reference(q, k, v, lens_q, lens_k, D ** -0.5)
        rels.append(((o.float() - ref).norm() / ref.norm().clamp_min(1e-30)).item())
        outs.append(o.cpu())
    return outs, rels


def check(path=None):
    outs, rels = outputs()
    for (lens_q, lens_k, H, split), r, o in zip(CASES, rels, outs):
        print(f"case {lens_q} {lens_k} H={H} split={split}: rel-L2 vs fp32 {r:.3e}  finite "
              f"{bool(torch.isfinite(o.float()).all())}", flush=True)
    print(f"halves forced: {os.environ.get('FLITE_ATTN_HALVES', 'plan')}; worst rel-L2 {max(rels):.3e}", flush=True)
    if path:
        torch.save(outs, path)


def compare(a, b):
    A, B = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    for i, (x, y) in enumerate(zip(A, B)):
        eq = torch.equal(x.view(torch.int16), y.view(torch.int16))
        diff = (x.float() - y.float()).abs().max().item()
        print(f"case {i} {CASES[i][:3]}: {'identical' if eq else 'differs'} (max abs diff {diff:.3e})", flush=True)


def timing(B, T, Lk, H=12, iters=50):
    q = torch.nn.functional.normalize(torch.randn(B * T, H, D, device=dev), dim=-1).mul(16).bfloat16()
    k = torch.nn.functional.normalize(torch.randn(B * Lk, H, D, device=dev), dim=-1).mul(16).bfloat16()
    v = torch.randn(B * Lk, H, D, device=dev).bfloat16()
    cu_q = torch.arange(B + 1, dtype=torch.int32, device=dev) * T
    cu_k = torch.arange(B + 1, dtype=torch.int32, device=dev) * Lk
    out = torch.empty_like(q)
    ws = nat.attn_workspace(dev, B, H, T, Lk)
    for _ in range(5):
        nat.attn_varlen(q, k, v, cu_q, cu_k, T, D ** -0.5, out=out, max_score=16.5, workspace=ws, max_k=Lk)
    torch.cuda.synchronize()
    res = []
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            nat.attn_varlen(q, k, v, cu_q, cu_k, T, D ** -0.5, out=out, max_score=16.5, workspace=ws, max_k=Lk)
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) / iters * 1000)
    fl = 4.0 * B * H * T * Lk * D
    print(f"time B={B} T={T} Lk={Lk} halves={os.environ.get('FLITE_ATTN_HALVES', 'plan')}: " +
          " / ".join(f"{r:.1f}" for r in res) + f" us  ({fl / min(res) / 1e6:.0f} TF/s best)", flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "check":
        check(sys.argv[2] if len(sys.argv) > 2 else None)
    elif sys.argv[1] == "compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        timing(1, 4112, 512)
        timing(2, 4112, 512)
        if "--self" in sys.argv:
            timing(2, 4112, 4112, iters=20)
