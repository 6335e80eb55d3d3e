"""fp8 GEMM epilogue cost at the 1344x896 residual shapes (M = 2 x 4720): bf16 store vs gated fp32 residual."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402
from f_lite import _native as nat  # noqa: E402

dev = "cuda"
torch.manual_seed(0)
for M, N, K in [(9440, 3072, 3072), (9440, 3072, 12288)]:
    a8, asc = nat.quant_fp8_rows(torch.randn(M, K, device=dev).bfloat16())
    w8, wsc = nat.quant_fp8_rows((torch.randn(N, K, device=dev) * 0.05).bfloat16())
    b = (torch.randn(N, device=dev) * 0.1).bfloat16()
    gate = torch.randn(2, N, device=dev)
    x = torch.randn(M, N, device=dev)
    ob = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    T = M // 2
    fns = {
        "store_bf16": lambda: nat.gemm_fp8(a8, asc, w8, wsc, b, out=ob),
        "resid_gate": lambda: nat.gemm_fp8(a8, asc, w8, wsc, b, out=x, epilogue=nat.EPI8_RESID_F32, gate=gate,
                                           gate_seg_stride=N, rows_per_seg=T),
        "resid_shared_gate": lambda: nat.gemm_fp8(a8, asc, w8, wsc, b, out=x, epilogue=nat.EPI8_RESID_F32,
                                                  gate=gate, gate_seg_stride=0, rows_per_seg=T),
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
    print(f"fp8 M={M} N={N} K={K}: " + "  ".join(f"{k} {sorted(v)[len(v) // 2]:.1f} us" for k, v in times.items()),
          flush=True)
