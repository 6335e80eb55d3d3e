"""Our bf16 GEMM vs torch.mm (hipBLASLt) on the DiT shapes and 8192^3, random data, interleaved rounds
(diagnostic; run on the GPU box)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402
from f_lite import _native as nat  # noqa: E402

SHAPES = [(8192, 8192, 8192), (8224, 24576, 3072), (8224, 9216, 3072), (8224, 3072, 3072), (8224, 3072, 12288)]


def timeit(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    torch.manual_seed(0)
    ws = nat.gemm_workspace("cuda")
    for M, N, K in SHAPES:
        a = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        ours, blas = [], []
        for _ in range(3):
            ours.append(timeit(lambda: nat.gemm(a, w, out=out, workspace=ws)))
            blas.append(timeit(lambda: torch.mm(a, w.t(), out=out)))
        o, b = sorted(ours)[1], sorted(blas)[1]
        print(f"M={M} N={N} K={K}: ours {o*1e3:.1f} us {fl/o/1e9:.0f} TF/s | torch.mm {b*1e3:.1f} us "
              f"{fl/b/1e9:.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
