"""Attention schedule timeline: per-workgroup s_memrealtime stamps (100 MHz) of a diagnostic build.

    python f-lite_amd/tools/attn_probe.py [T Lk [split]]
Prints the distribution of workgroup start / main-loop-end / end times (us from the earliest start), split by
phase (A: full q-tiles, B: tail key ranges), and the per-XCD finish times.
"""
import ctypes
import subprocess
import sys
from pathlib import Path

import torch

HERE = Path(__file__).resolve().parent
SO = HERE / "attn_probe.so"


def build():
    src = HERE / "attn_probe.hip"
    dep = HERE.parent / "csrc" / "attention.hip"
    if not SO.exists() or SO.stat().st_mtime < max(src.stat().st_mtime, dep.stat().st_mtime):
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                               "-I" + str(HERE.parent / "csrc"), str(src), "-o", str(SO)])


def q(col):
    t = torch.quantile(col.double(), torch.tensor([0.0, 0.5, 0.9, 1.0], dtype=torch.float64))
    return "min %7.1f med %7.1f p90 %7.1f max %7.1f" % tuple(t.tolist())


def main():
    T, Lk = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) >= 3 else (4112, 4112)
    split = len(sys.argv) < 4 or sys.argv[3] != "0"
    H = 12
    build()
    lib = ctypes.CDLL(str(SO))
    sys.path.insert(0, str(HERE.parent))
    from f_lite import _native as nat
    dev = "cuda"
    qt = torch.nn.functional.normalize(torch.randn(2 * T, H, 256, device=dev), dim=-1).mul(16).bfloat16()
    kt = torch.nn.functional.normalize(torch.randn(2 * Lk, H, 256, device=dev), dim=-1).mul(16).bfloat16()
    vt = torch.randn(2 * Lk, H, 256, device=dev).bfloat16()
    o = torch.empty_like(qt)
    cu_q = torch.tensor([0, T, 2 * T], dtype=torch.int32, device=dev)
    cu_k = torch.tensor([0, Lk, 2 * Lk], dtype=torch.int32, device=dev)
    ws = nat.attn_workspace(dev, 2, H) if split else None
    nwg = 2 * H * ((T + 127) // 128 + 16)
    st = torch.zeros(nwg * 4, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    for _ in range(6):
        st.zero_()
        rc = lib.attn_probe(ctypes.c_void_p(stream), T, Lk, H, ctypes.c_void_p(qt.data_ptr()),
                            ctypes.c_void_p(kt.data_ptr()), ctypes.c_void_p(vt.data_ptr()), ctypes.c_void_p(o.data_ptr()),
                            ctypes.c_void_p(cu_q.data_ptr()), ctypes.c_void_p(cu_k.data_ptr()),
                            ctypes.c_void_p(ws.data_ptr() if ws is not None else 0),
                            ctypes.c_long(ws.numel() if ws is not None else 0), ctypes.c_void_p(st.data_ptr()))
        assert rc == 0
        torch.cuda.synchronize()
    s = st.view(-1, 4).cpu()
    used = s[:, 0] > 0
    s = s[used]
    t0 = s[:, 0].min()
    us = (s[:, :3] - t0).double() / 100.0
    n_main = T // 128 if split and T % 128 else (T + 127) // 128
    nA = 2 * H * n_main
    print(f"T={T} Lk={Lk} split={split} workgroups={s.shape[0]} (phase A {nA})")
    for name, sel in (("A", slice(0, nA)), ("B", slice(nA, None))):
        if us[sel].shape[0] == 0:
            continue
        print(f"  phase {name}: start {q(us[sel, 0])}")
        print(f"  phase {name}: loop  {q(us[sel, 1])}")
        print(f"  phase {name}: end   {q(us[sel, 2])}")
        dur = us[sel, 2] - us[sel, 0]
        print(f"  phase {name}: dur   {q(dur)}")
    xcc = (s[:, 3] >> 32) & 0xF
    for x in range(8):
        m = xcc == x
        if m.any():
            print(f"  xcc {x}: n={int(m.sum())} last end {us[m, 2].max():.1f} us")


if __name__ == "__main__":
    main()
