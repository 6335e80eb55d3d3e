"""Standalone launches of every major DiT kernel at the bench shapes, for rocprofv3 counter passes.

    rocprofv3 --pmc <counters> --output-format csv -d <dir> -- python3 f-lite_amd/tools/pmc_kernels.py

rocprofv3 7.2 crashes in --pmc passes over the full engine (Measurement), so each kernel class of
one 10B / 1024^2 CFG-batched DiT block (M = 2 x 4112 = 8224 rows, D = 3072, F = 12288, 12 heads of 256, a
512-token context) is launched here with the engine's shapes, epilogues, workspaces and launch choices, on
inputs of the engine's statistics (q/k RMS-normalised before attention, so the bounded-score softmax applies).

Classes are separated in the trace by a marker: before class k, a fill_ of a [k + 1]-element int32 tensor
(its own kernel). tools/pmc_reduce.py cuts the dispatch sequence at the markers.
"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from f_lite import _native as nat  # noqa: E402

CLASSES = ["qkv", "rope_qknorm", "attn_self", "proj", "rmsnorm_mod", "cross_q", "attn_cross", "attn_cross_c", "gateup",
           "down"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=6)
    ap.add_argument("--only", default=None, help="comma list of classes")
    ap.add_argument("--residual", default="bf16", choices=["bf16", "fp32"],
                    help="residual-stream storage of the proj / down epilogues and the norm input (round 6: bf16)")
    args = ap.parse_args()
    dev = "cuda"
    T, B, D, F, H, HD, LC = 4112, 2, 3072, 12288, 12, 256, 512
    M = B * T
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*shape, std=1.0):
        return (torch.randn(*shape, device=dev, generator=g) * std).bfloat16()

    x = torch.randn(M, D, device=dev, generator=g) * 4  # the residual stream
    if args.residual == "bf16":
        x = x.bfloat16()
    epi_resid = nat.EPI_RESID_BF16 if args.residual == "bf16" else nat.EPI_RESID_F32
    nbuf = rnd(M, D)
    w_qkv, b_qkv = rnd(3 * D, D, std=0.02), rnd(3 * D, std=0.02)
    w_proj = rnd(D, D, std=0.02)
    w_q, b_q = rnd(D, D, std=0.02), rnd(D, std=0.02)
    w_gate, w_up, w_down = rnd(F, D, std=0.02), rnd(F, D, std=0.02), rnd(D, F, std=0.02)
    qkv = torch.empty(M, 3 * D, device=dev, dtype=torch.bfloat16)
    q_cross = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    obuf = rnd(M, D)
    hbuf = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    kv = rnd(B * LC, 2 * D)
    nat.rope_qknorm_(kv, H, 0)  # cross K normalised once (step-invariant cache)
    gate = torch.randn(B, D, device=dev, generator=g) * 0.1
    shift = torch.randn(B, D, device=dev, generator=g) * 0.1
    scale = torch.randn(B, D, device=dev, generator=g) * 0.1
    wnorm = torch.ones(D, device=dev, dtype=torch.bfloat16)
    cos, sin = nat.rope_tables(64, 64, device=dev)
    cu = torch.tensor([0, T, 2 * T], dtype=torch.int32, device=dev)
    cu_c = torch.tensor([0, LC, 2 * LC], dtype=torch.int32, device=dev)
    gws = nat.gemm_workspace(dev)
    aws = nat.attn_workspace(dev, B, H)
    resid_kw = dict(gate=gate, gate_seg_stride=D, rows_per_seg=T)
    # q/k in the qkv buffer normalised once so attention sees QK-normed operands
    nat.gemm(nbuf, w_qkv, b_qkv, out=qkv)
    nat.rope_qknorm_(qkv, 2 * H, 2 * H, cos, sin, T)
    qkv_att = qkv.clone()
    q3 = qkv_att.view(M, 3, H, HD)

    def run(name):
        if name == "qkv":
            nat.gemm(nbuf, w_qkv, b_qkv, out=qkv, workspace=gws)
        elif name == "rope_qknorm":
            nat.rope_qknorm_(qkv, 2 * H, 2 * H, cos, sin, T)
        elif name == "attn_self":
            nat.attn_varlen(q3[:, 0], q3[:, 1], q3[:, 2], cu, cu, T, HD ** -0.5, out=obuf.view(M, H, HD),
                            max_score=16.5, workspace=aws, max_k=T)
        elif name == "proj":
            nat.gemm(obuf, w_proj, out=x, epilogue=epi_resid, workspace=gws, **resid_kw)
        elif name == "rmsnorm_mod":
            nat.rmsnorm_modulate(x, wnorm, shift, scale, seg_rows=T, out=nbuf)
        elif name == "cross_q":
            nat.gemm(nbuf, w_q, b_q, out=q_cross, workspace=gws)
        elif name == "attn_cross":
            kv3 = kv.view(B * LC, 2, H, HD)
            nat.attn_varlen(q3[:, 0], kv3[:, 0], kv3[:, 1], cu, cu_c, T, HD ** -0.5, out=obuf.view(M, H, HD),
                            max_score=16.5, workspace=aws, max_k=LC)
        elif name == "attn_cross_c":  # the uniform-context collapse's launch: the cond sequence's rows only
            kv3 = kv.view(B * LC, 2, H, HD)
            nat.attn_varlen(q3[T:, 0], kv3[LC:, 0], kv3[LC:, 1], cu[:2], cu_c[:2], T, HD ** -0.5,
                            out=obuf[T:].view(T, H, HD), max_score=16.5, workspace=aws, max_k=LC)
        elif name == "gateup":
            nat.gemm(nbuf, w_gate, out=hbuf, epilogue=nat.EPI_SWIGLU_BF16, w2=w_up, workspace=gws)
        elif name == "down":
            nat.gemm(hbuf, w_down, out=x, epilogue=epi_resid, workspace=gws, **resid_kw)

    classes = args.only.split(",") if args.only else CLASSES
    torch.cuda.synchronize()
    for k, name in enumerate(classes):
        marker = torch.empty(k + 1, dtype=torch.int32, device=dev)
        marker.fill_(k)
        torch.cuda.synchronize()
        for _ in range(args.launches):
            run(name)
        torch.cuda.synchronize()
    print(json.dumps({"classes": classes, "launches": args.launches}))


if __name__ == "__main__":
    main()
