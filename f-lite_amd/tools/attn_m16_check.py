"""Error of the bounded attention kernel against a torch fp32 reference, and its time at the DiT shapes.

Run once per kernel (the choice is process-wide, read at the first launch):
    python f-lite_amd/tools/attn_m16_check.py            # 32x32x16 kernel (attention.hip)
    FLITE_ATTN_M16=1 python f-lite_amd/tools/attn_m16_check.py   # 16x16x32 kernel (attention_m16.hip)
The 16x16x32 kernel is not in the product: `git apply profiles/r05l/attn_m16.patch` and rebuild to bring it back
(FLITE_ATTN_M16=2: its variant with attention.hip's V image). Without the patch the variable does nothing.
Cases: tools/attn_equal.py's (DiT self/cross shapes with and without the tail split, ragged, single-tile), then the
timing of the 1024^2 self-attention (T = 4112, split tail), cross-attention (512 keys) and the 1344x896 shape.
`--loop-like`: the self-attention timed per launch alone, after a qkv-sized GEMM, with the loop's strided rows, and
both (DESIGN §3 "16x16x32 MFMA form").
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parent))
import torch
from attn_equal import CASES
from f_lite import _native as nat

dev = "cuda"
D = 256


def reference(q, k, v, lens_q, lens_k, scale):
    out = torch.zeros(q.shape, dtype=torch.float32, device=dev)
    oq = ok = 0
    for lq, lk in zip(lens_q, lens_k):
        if lk > 0:
            qs = q[oq:oq + lq].float().transpose(0, 1)
            ks = k[ok:ok + lk].float().transpose(0, 1)
            vs = v[ok:ok + lk].float().transpose(0, 1)
            p = torch.softmax(qs @ ks.transpose(1, 2) * scale, dim=-1)
            out[oq:oq + lq] = (p @ vs).transpose(0, 1)
        oq += lq
        ok += lk
    return out


def check():
    worst = 0.0
    for lens_q, lens_k, H, split in CASES:
        lens_k = lens_q if lens_k is None else lens_k
        cu_q = torch.tensor([0] + list(torch.tensor(lens_q).cumsum(0)), dtype=torch.int32)
        cu_k = torch.tensor([0] + list(torch.tensor(lens_k).cumsum(0)), dtype=torch.int32)
        g = torch.Generator(device=dev).manual_seed(sum(lens_q) + H)
        q = torch.nn.functional.normalize(torch.randn(int(cu_q[-1]), H, D, device=dev, generator=g), dim=-1)
        k = torch.nn.functional.normalize(torch.randn(max(int(cu_k[-1]), 1), H, D, device=dev, generator=g), dim=-1)
        v = torch.randn(max(int(cu_k[-1]), 1), H, D, device=dev, generator=g).bfloat16()
        q, k = (q * 16).bfloat16(), (k * 16).bfloat16()
        ws = nat.attn_workspace(dev, len(lens_q), H) if split else None
        o = nat.attn_varlen(q, k, v, cu_q.to(dev), cu_k.to(dev), max(lens_q), D ** -0.5, max_score=16.5, workspace=ws,
                            max_k=max(lens_k))
        ref = reference(q, k, v, lens_q, lens_k, D ** -0.5)
        err = (o.float() - ref).abs()
        rel = (err.norm() / ref.norm().clamp_min(1e-30)).item()
        print(f"case {lens_q} {lens_k} H={H} split={split}: max abs {err.max().item():.3e}  rel-L2 {rel:.3e}  "
              f"finite {bool(torch.isfinite(o.float()).all())}", flush=True)
        worst = max(worst, rel)
    print(f"worst rel-L2 {worst:.3e}", flush=True)


def timing(T, Lk, iters=50, H=12, qkv_rows=False, gemm=False):
    """qkv_rows: q, k, v as head views of one [L, 3 * H * 256] buffer (the qkv GEMM's output rows, as in the DiT
    loop); gemm: a [2T, 3072] x [3072, 9216] bf16 matmul before every launch (the loop's qkv GEMM), attention
    timed alone by events around each launch."""
    B = 2
    qn = torch.nn.functional.normalize(torch.randn(B * T, H, D, device=dev), dim=-1).mul(16).bfloat16()
    kn = torch.nn.functional.normalize(torch.randn(B * Lk, H, D, device=dev), dim=-1).mul(16).bfloat16()
    vn = torch.randn(B * Lk, H, D, device=dev).bfloat16()
    if qkv_rows and T == Lk:
        buf = torch.cat([qn.flatten(1), kn.flatten(1), vn.flatten(1)], dim=1)  # [L, 3 H D]
        q, k, v = (buf[:, i * H * D:(i + 1) * H * D].view(B * T, H, D) for i in range(3))
    else:
        q, k, v = qn, kn, vn
    cu_q = torch.tensor([0, T, 2 * T], dtype=torch.int32, device=dev)
    cu_k = torch.tensor([0, Lk, 2 * Lk], dtype=torch.int32, device=dev)
    out = torch.empty_like(qn)
    ws = nat.attn_workspace(dev, B, H)
    ga = torch.randn(B * T, 3072, device=dev).bfloat16() if gemm else None
    gb = torch.randn(3072, 9216, device=dev).bfloat16() if gemm else None
    for _ in range(5):
        nat.attn_varlen(q, k, v, cu_q, cu_k, T, D ** -0.5, out=out, max_score=16.5, workspace=ws, max_k=Lk)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for s, e in ev:
        if gemm:
            torch.mm(ga, gb)
        s.record()
        nat.attn_varlen(q, k, v, cu_q, cu_k, T, D ** -0.5, out=out, max_score=16.5, workspace=ws, max_k=Lk)
        e.record()
    torch.cuda.synchronize()
    ms = sorted(s.elapsed_time(e) for s, e in ev)[iters // 2]
    fl = 4.0 * B * H * T * Lk * D
    print(f"time T={T} Lk={Lk} qkv_rows={qkv_rows} gemm={gemm}: median {ms * 1000:.1f} us  {fl / ms / 1e9:.0f} TF/s",
          flush=True)


if __name__ == "__main__":
    import os

    print("kernel:", "16x16x32 (attention_m16.hip)" if os.environ.get("FLITE_ATTN_M16") == "1" else
          "32x32x16 (attention.hip)", flush=True)
    if "--loop-like" in sys.argv:  # which in-loop condition moves the kernel: strided rows, a GEMM in front, both
        for _ in range(2):
            for rows, gm in ((False, False), (True, False), (False, True), (True, True)):
                timing(4112, 4112, iters=30, qkv_rows=rows, gemm=gm)
        sys.exit(0)
    if "--time-only" not in sys.argv:
        check()
    if "--no-time" in sys.argv:
        sys.exit(0)
    for _ in range(2):
        timing(4112, 4112)
        timing(4096, 4112)
        timing(4112, 512)
        timing(4720, 4720, iters=30)
