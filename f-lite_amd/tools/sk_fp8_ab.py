"""fp8 GEMM at the 1344x896 shapes (M = 2 x 4720): data-parallel vs stream-K (workspace; FLITE_FP8_SK_ALWAYS=1
forces the split where the cost model declines it). Median us per launch, interleaved rounds."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402
from f_lite import _native as nat  # noqa: E402

dev = "cuda"
torch.manual_seed(0)
ws = nat.gemm_workspace(dev)
for name, M, N, K, epi in [("qkv", 9440, 9216, 3072, "store"), ("proj", 9440, 3072, 3072, "resid"),
                           ("down", 9440, 3072, 12288, "resid"), ("gateup", 9440, 24576, 3072, "swiglu")]:
    a8, asc = nat.quant_fp8_rows(torch.randn(M, K, device=dev).bfloat16())
    if epi == "swiglu":
        w8, wsc = nat.quant_fp8_gateup((torch.randn(N // 2, K, device=dev) * 0.02).bfloat16(),
                                       (torch.randn(N // 2, K, device=dev) * 0.02).bfloat16())
        kw = dict(epilogue=nat.EPI8_SWIGLU_FP8)
    else:
        w8, wsc = nat.quant_fp8_rows((torch.randn(N, K, device=dev) * 0.02).bfloat16())
        kw = {}
        if epi == "resid":
            x = torch.zeros(M, N, device=dev)
            kw = dict(out=x, epilogue=nat.EPI8_RESID_F32, gate=torch.ones(2, N, device=dev), gate_seg_stride=N,
                      rows_per_seg=M // 2)
    fns = {"dp": lambda: nat.gemm_fp8(a8, asc, w8, wsc, **kw), "ws": lambda: nat.gemm_fp8(a8, asc, w8, wsc, workspace=ws, **kw)}
    times = {k: [] for k in fns}
    for f in fns.values():
        f()
    for rnd in range(8):
        items = list(fns.items())
        for k, f in (items if rnd % 2 == 0 else items[::-1]):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                f()
            e1.record()
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / 10 * 1e3)
    med = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
    print(f"{name} M={M} N={N} K={K} sk_always={os.environ.get('FLITE_FP8_SK_ALWAYS', '0')}: dp {med['dp']:.1f} us  "
          f"ws {med['ws']:.1f} us", flush=True)
