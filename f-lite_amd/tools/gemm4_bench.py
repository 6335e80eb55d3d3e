"""A/B of the 4-wave GEMM prototype (tools/gemm4_proto.hip) against the product bf16 GEMM (flite_gemm_bf16, STORE
epilogue, no bias) on the DiT shapes; correctness vs torch first. Usage:
  python tools/gemm4_bench.py build      (CPU container: hipcc -> tools/gemm4_proto.so)
  python tools/gemm4_bench.py            (GPU box)
"""
import ctypes
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
SO = HERE / "gemm4_proto.so"


def build():
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-fno-slp-vectorize", f"-I{HERE.parent / 'csrc'}", f"-I{HERE.parents[1] / 'include'}",
           str(HERE / "gemm4_proto.hip"), "-o", str(SO)]
    subprocess.run(cmd, check=True)
    print("built", SO)


def main():
    sys.path.insert(0, str(HERE.parent))
    import torch
    from f_lite import _native as nat

    lib = ctypes.CDLL(str(SO))
    lib.gemm4_proto.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3 + [ctypes.c_void_p]
    dev = "cuda"
    torch.manual_seed(0)
    stream = torch.cuda.current_stream().cuda_stream

    def g4(a, w, c):
        rc = lib.gemm4_proto(a.data_ptr(), w.data_ptr(), c.data_ptr(), a.shape[0], w.shape[0], a.shape[1], stream)
        assert rc == 0, rc

    shapes = [(8192, 8192, 8192), (8224, 9216, 3072), (8224, 3072, 3072), (8224, 3072, 12288),
              (8224, 24576, 3072), (16448, 3072, 3072)]
    for M, N, K in shapes:
        a = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        g4(a, w, c)
        ref = nat.gemm(a, w, None)
        torch.cuda.synchronize()
        err = ((c.float() - ref.float()).norm() / ref.float().norm()).item()
        ws = nat.gemm_workspace(dev)
        times = {"product": [], "product_sk": [], "proto4": []}
        fns = {"product": lambda: nat.gemm(a, w, None, out=ref),
               "product_sk": lambda: nat.gemm(a, w, None, out=ref, workspace=ws), "proto4": lambda: g4(a, w, c)}
        for _ in range(2):
            for f in fns.values():
                f()
        for rnd in range(6):
            for name, f in (fns.items() if rnd % 2 == 0 else reversed(list(fns.items()))):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    f()
                e1.record()
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1) / 10)
        fl = 2.0 * M * N * K
        med = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
        print(f"M={M} N={N} K={K}: rel_err {err:.2e}  product {med['product'] * 1e3:.1f} us "
              f"({fl / med['product'] / 1e9:.0f} TF/s)  +sk {med['product_sk'] * 1e3:.1f} us  proto4 {med['proto4'] * 1e3:.1f} us "
              f"({fl / med['proto4'] / 1e9:.0f} TF/s)  ratio {med['product'] / med['proto4']:.3f}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        build()
    else:
        main()
