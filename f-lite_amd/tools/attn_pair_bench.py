"""A/B of the two-waves-per-SIMD attention prototype (tools/attn_pair_proto.hip) against the product kernel
(flite_attn_varlen_fwd, bounded softmax) at T = 4096 (self, and cross onto 512 keys), B = 2, H = 12.
  python tools/attn_pair_bench.py build    (CPU container)
  python tools/attn_pair_bench.py          (GPU box)
"""
import ctypes
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
SO = HERE / "attn_pair_proto.so"


def build(name="", defines=()):
    out = HERE / f"attn_pair_proto{name}.so"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    f"-I{HERE.parent / 'csrc'}", f"-I{HERE.parents[1] / 'include'}", *defines,
                    str(HERE / "attn_pair_proto.hip"), "-o", str(out)], check=True)
    print("built", out)


def main():
    sys.path.insert(0, str(HERE.parent))
    import torch
    from f_lite import _native as nat

    import os
    lib = ctypes.CDLL(os.environ.get("PAIR_SO", str(SO)))
    lib.attn_pair_proto.argtypes = [ctypes.c_void_p] * 6 + [ctypes.c_int] * 3 + [ctypes.c_float] * 2 + [ctypes.c_void_p]
    torch.manual_seed(0)
    B, H, D = 2, 12, 256
    stream = torch.cuda.current_stream().cuda_stream
    for name, T, Lk in (("self", 4096, 4096), ("cross", 4096, 512)):
        q = torch.nn.functional.normalize(torch.randn(B * T, H, D, device="cuda"), dim=-1).mul(16).bfloat16()
        k = torch.nn.functional.normalize(torch.randn(B * Lk, H, D, device="cuda"), dim=-1).mul(16).bfloat16()
        v = torch.randn(B * Lk, H, D, device="cuda").bfloat16()
        cu_q = torch.tensor([0, T, 2 * T], dtype=torch.int32, device="cuda")
        cu_k = torch.tensor([0, Lk, 2 * Lk], dtype=torch.int32, device="cuda")
        out = torch.empty_like(q)
        o2 = torch.empty_like(q)
        prod = lambda: nat.attn_varlen(q, k, v, cu_q, cu_k, T, D ** -0.5, out=out, max_score=16.5, max_k=Lk)  # noqa
        pair = lambda: lib.attn_pair_proto(q.data_ptr(), k.data_ptr(), v.data_ptr(), o2.data_ptr(), cu_q.data_ptr(),  # noqa
                                           cu_k.data_ptr(), B, H, T, D ** -0.5, 16.5, stream)
        prod()
        assert pair() == 0
        torch.cuda.synchronize()
        err = ((o2.float() - out.float()).norm() / out.float().norm()).item()
        times = {"product": [], "pair": []}
        for rnd in range(6):
            for nm, f in ((("product", prod), ("pair", pair)) if rnd % 2 == 0 else (("pair", pair), ("product", prod))):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    f()
                e1.record()
                torch.cuda.synchronize()
                times[nm].append(e0.elapsed_time(e1) / 10 * 1e3)
        med = {kk: sorted(vv)[len(vv) // 2] for kk, vv in times.items()}
        fl = 4.0 * B * H * T * Lk * D
        print(f"[{os.environ.get('PAIR_SO', 'default').split('/')[-1]}] {name} T={T} Lk={Lk}: rel diff {err:.2e}  product {med['product']:.1f} us ({fl / med['product'] / 1e6:.0f} TF/s)"
              f"  pair {med['pair']:.1f} us ({fl / med['pair'] / 1e6:.0f} TF/s)  ratio {med['product'] / med['pair']:.3f}",
              flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        build(*(sys.argv[2:3] or [""]), defines=sys.argv[3:])
    else:
        main()
