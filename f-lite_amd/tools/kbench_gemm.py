"""Micro-benchmark + correctness check of flite_gemm_bf16 at the DiT shapes (run on the GPU box)."""
import sys, time
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
from f_lite import _native as nat

torch.manual_seed(0)
dev = "cuda"

def check(M, N, K, epi=nat.EPI_STORE_BF16, bias=True):
    a = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
    b = (torch.randn(N, device=dev) * 0.1).bfloat16() if bias else None
    ref = a.float() @ w.float().t()
    if b is not None: ref += b.float()
    if epi == nat.EPI_STORE_BF16:
        out = nat.gemm(a, w, b)
    elif epi == nat.EPI_STORE_F32:
        out = nat.gemm(a, w, b, epilogue=epi)
    err = (out.float() - ref).norm() / ref.norm()
    print(f"check M={M} N={N} K={K} epi={epi}: rel_l2={err.item():.3e}", flush=True)
    return err.item()

def check_swiglu(M, F, K):
    a = torch.randn(M, K, device=dev).bfloat16()
    wg = (torch.randn(F, K, device=dev) * 0.05).bfloat16()
    wu = (torch.randn(F, K, device=dev) * 0.05).bfloat16()
    g = a.float() @ wg.float().t(); u = a.float() @ wu.float().t()
    ref = torch.nn.functional.silu(g) * u
    out = nat.gemm(a, wg, epilogue=nat.EPI_SWIGLU_BF16, w2=wu)
    err = (out.float() - ref).norm() / ref.norm()
    print(f"swiglu M={M} F={F} K={K}: rel_l2={err.item():.3e}", flush=True)

def check_resid(M, N, K, T):
    a = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
    b = (torch.randn(N, device=dev) * 0.1).bfloat16()
    nseg = (M + T - 1) // T
    gate = torch.randn(nseg, N, device=dev)
    x0 = torch.randn(M, N, device=dev)
    ref = x0.clone()
    y = a.float() @ w.float().t() + b.float()
    for s in range(nseg):
        ref[s*T:(s+1)*T] += y[s*T:(s+1)*T] * gate[s]
    x = x0.clone()
    nat.gemm(a, w, b, out=x, epilogue=nat.EPI_RESID_F32, gate=gate, gate_seg_stride=N, rows_per_seg=T)
    err = (x - ref).norm() / ref.norm()
    print(f"resid M={M} N={N} K={K} T={T}: rel_l2={err.item():.3e}", flush=True)

WS = None


def bench(M, N, K, iters=20, epi=nat.EPI_STORE_BF16, rounds=5):
    """DP (no workspace) vs stream-K (workspace) interleaved in one process; median ms per launch."""
    global WS
    if WS is None:
        WS = nat.gemm_workspace(dev)
    a = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
    w2 = (torch.randn(N, K, device=dev) * 0.05).bfloat16() if epi == nat.EPI_SWIGLU_BF16 else None
    resid = epi == nat.EPI_RESID_F32
    out = torch.zeros(M, N, device=dev, dtype=torch.float32 if resid else torch.bfloat16)
    gate = torch.randn(2, N, device=dev) if resid else None
    kw = dict(gate=gate, gate_seg_stride=N, rows_per_seg=(M + 1) // 2) if resid else {}
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    res = {"dp": [], "sk": []}
    for _ in range(rounds):
        for mode in ("dp", "sk"):
            ws = WS if mode == "sk" else None
            for _ in range(2):
                nat.gemm(a, w, out=out, epilogue=epi, w2=w2, workspace=ws, **kw)
            torch.cuda.synchronize()
            s.record()
            for _ in range(iters):
                nat.gemm(a, w, out=out, epilogue=epi, w2=w2, workspace=ws, **kw)
            e.record(); torch.cuda.synchronize()
            res[mode].append(s.elapsed_time(e) / iters)
    Nf = 2 * N if epi == nat.EPI_SWIGLU_BF16 else N
    fl = 2 * M * Nf * K
    med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    wt = torch.randn(Nf, K, device=dev).bfloat16()
    for _ in range(3): torch.mm(a, wt.t())
    torch.cuda.synchronize(); s.record()
    for _ in range(iters): torch.mm(a, wt.t())
    e.record(); torch.cuda.synchronize()
    ms_t = s.elapsed_time(e) / iters
    print(f"bench M={M} N={Nf} K={K} epi={epi}: dp {med['dp']:.3f} ms {fl/med['dp']/1e9:.0f} TF/s | "
          f"sk {med['sk']:.3f} ms {fl/med['sk']/1e9:.0f} TF/s | torch.mm {ms_t:.3f} ms {fl/ms_t/1e9:.0f} TF/s",
          flush=True)

if __name__ == "__main__":
    check(256, 256, 64)
    check(300, 200, 128)
    check(8224, 3072, 3072)
    check(30, 27648, 3072, epi=nat.EPI_STORE_F32)
    check_swiglu(1000, 1024, 512)
    check_resid(1000, 768, 256, 300)
    bench(8224, 9216, 3072)
    bench(8224, 3072, 3072)
    bench(8224, 12288, 3072, epi=nat.EPI_SWIGLU_BF16)
    bench(8224, 3072, 12288)
    bench(8224, 3072, 3072, epi=nat.EPI_RESID_F32)
    bench(8224, 3072, 12288, epi=nat.EPI_RESID_F32)
    bench(8192, 8192, 8192, iters=10)
    bench(8224, 1536, 3072, epi=nat.EPI_SWIGLU_BF16)
