"""Epilogue cost on the DiT residual GEMM shapes: the same GEMM with the bf16 store, the fp32 store and the gated
fp32 residual read-modify-write (with and without the gate rows), interleaved rounds, median per launch."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402
from f_lite import _native as nat  # noqa: E402

dev = "cuda"
torch.manual_seed(0)
ws = nat.gemm_workspace(dev)
for M, N, K in [(8224, 3072, 3072), (8224, 3072, 12288)]:
    a = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
    b = (torch.randn(N, device=dev) * 0.1).bfloat16()
    gate = torch.randn(2, N, device=dev)
    x = torch.randn(M, N, device=dev)
    ob = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    of = torch.empty(M, N, device=dev)
    T = M // 2
    fns = {
        "store_bf16": lambda: nat.gemm(a, w, b, out=ob, workspace=ws),
        "store_f32": lambda: nat.gemm(a, w, b, out=of, epilogue=nat.EPI_STORE_F32, workspace=ws),
        "resid_gate": lambda: nat.gemm(a, w, b, out=x, epilogue=nat.EPI_RESID_F32, gate=gate, gate_seg_stride=N,
                                       rows_per_seg=T, workspace=ws),
        "resid_nogate": lambda: nat.gemm(a, w, b, out=x, epilogue=nat.EPI_RESID_F32, workspace=ws),
    }
    times = {k: [] for k in fns}
    for f in fns.values():
        f()
    for rnd in range(8):
        items = list(fns.items())
        for name, f in (items if rnd % 2 == 0 else items[::-1]):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                f()
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / 10 * 1e3)
    print(f"M={M} N={N} K={K}: " + "  ".join(f"{k} {sorted(v)[len(v) // 2]:.1f} us" for k, v in times.items()),
          flush=True)
