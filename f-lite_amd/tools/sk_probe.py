"""Stream-K phase timeline: per-workgroup s_memrealtime stamps (100 MHz) of a diagnostic GEMM build.

    python f-lite_amd/tools/sk_probe.py [M N K]
Prints, over the persistent grid, the distribution of phase end times (us from the earliest start):
0 start, 1 data-parallel tiles done, 2 partial published, 3 finisher segment computed, 4 partials acquired,
5 end; plus the XCC / CU placement census.
"""
import ctypes
import os
import subprocess
import sys
from pathlib import Path

import torch

HERE = Path(__file__).resolve().parent
SO = HERE / "sk_probe.so"


def build():
    src = HERE / "sk_probe.hip"
    if not SO.exists() or SO.stat().st_mtime < max(src.stat().st_mtime, (HERE.parent / "csrc" / "gemm.hip").stat().st_mtime):
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                               str(src), "-o", str(SO)])


def main():
    M, N, K = (int(x) for x in sys.argv[1:4]) if len(sys.argv) >= 4 else (8224, 3072, 12288)
    build()
    lib = ctypes.CDLL(str(SO))
    sys.path.insert(0, str(HERE.parent))
    from f_lite import _native as nat
    dev = "cuda"
    a = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
    out = torch.empty(M, N, device=dev)
    ws = nat.gemm_workspace(dev)
    G = ws.numel() // (256 * 256 * 4 + 4)
    st = torch.zeros(G * 8, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    for it in range(4):
        st.zero_()
        rc = lib.sk_probe_gemm(ctypes.c_void_p(stream), M, N, K, ctypes.c_void_p(a.data_ptr()),
                               ctypes.c_void_p(w.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                               ctypes.c_void_p(ws.data_ptr()), ctypes.c_void_p(st.data_ptr()))
        assert rc == 0
        torch.cuda.synchronize()
    s = st.view(G, 8).cpu()
    t = s[:, :6].double()
    t0 = t[:, 0][t[:, 0] > 0].min()
    us = (t - t0) / 100.0  # 100 MHz
    print(f"M={M} N={N} K={K} G={G}")
    for i, name in enumerate(["start", "dp_done", "partial", "fin_comp", "acquired", "end"]):
        col = us[:, i][s[:, i] > 0]
        if col.numel():
            q = torch.quantile(col, torch.tensor([0.0, 0.5, 0.9, 1.0], dtype=torch.float64))
            print(f"  {name:9s} n={col.numel():4d} min {q[0]:8.1f} med {q[1]:8.1f} p90 {q[2]:8.1f} max {q[3]:8.1f} us")
    xcc = s[:, 6]
    hw = s[:, 7]
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 0x1
    se = (hw >> 13) & 0x7
    keys = set(zip(xcc.tolist(), se.tolist(), sh.tolist(), cu.tolist()))
    print(f"  distinct (xcc,se,sh,cu) slots used: {len(keys)} of {G} workgroups")
    late = (us[:, 0] > 5.0).sum().item()
    print(f"  workgroups starting > 5 us after the first: {late}")


if __name__ == "__main__":
    main()
