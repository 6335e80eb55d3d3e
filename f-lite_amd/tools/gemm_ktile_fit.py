"""Per-tile fixed cost of the data-parallel bf16 GEMM (run on the GPU box).

Times the gate/up (SwiGLU) and proj (gated residual) shapes of the 10B / 1024^2 workload at several K with M and
N fixed, so the tile count and the rounds per CU stay the same, and fits time = a + b * (K / 64): b is the cost
of one 64-deep k-tile per round of tiles, a the per-round fixed cost (workgroup launch, setup, the first two
k-tiles' DMA latency, epilogue and teardown). a / time is what a persistent kernel that overlaps the next tile's
prologue with the current epilogue could at most recover.
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
import torch
from f_lite import _native as nat

dev = "cuda"
torch.manual_seed(0)


def time_launch(fn, iters=20, rounds=5):
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    best = []
    for _ in range(rounds):
        fn()
        torch.cuda.synchronize()
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        best.append(s.elapsed_time(e) / iters)
    return float(np.median(best))


def fit(name, make, Ks):
    ts = []
    for K in Ks:
        fn = make(K)
        t = time_launch(fn)
        ts.append(t)
        print(f"{name} K={K}: {t * 1e3:.1f} us", flush=True)
    nk = np.array(Ks) / 64.0
    b, a = np.polyfit(nk, np.array(ts), 1)
    print(f"{name}: per-k-tile {b * 1e3:.3f} us/launch, intercept {a * 1e3:.1f} us/launch "
          f"({100 * a / ts[Ks.index(3072)]:.1f} % of K=3072)", flush=True)


M, D, F = 8224, 3072, 12288
# K <= 3072: at K = 4096 the gate/up operands (268 MB) overflow the 256 MiB Infinity Cache and the line bends
Ks = [1024, 2048, 3072]


def make_swiglu(K):
    a = torch.randn(M, K, device=dev).bfloat16()
    wg = (torch.randn(F, K, device=dev) * 0.05).bfloat16()
    wu = (torch.randn(F, K, device=dev) * 0.05).bfloat16()
    out = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    return lambda: nat.gemm(a, wg, out=out, epilogue=nat.EPI_SWIGLU_BF16, w2=wu)


def make_resid(K):
    a = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(D, K, device=dev) * 0.05).bfloat16()
    x = torch.zeros(M, D, device=dev)
    gate = torch.randn(2, D, device=dev)
    return lambda: nat.gemm(a, w, out=x, epilogue=nat.EPI_RESID_F32, gate=gate, gate_seg_stride=D,
                            rows_per_seg=M // 2)


def make_store(K):
    a = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(D, K, device=dev) * 0.05).bfloat16()
    out = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    return lambda: nat.gemm(a, w, out=out)


fit("swiglu", make_swiglu, Ks)
fit("resid", make_resid, Ks)
fit("store", make_store, Ks)
