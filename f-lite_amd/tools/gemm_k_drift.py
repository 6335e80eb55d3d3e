"""Per-k-tile cost of one exact data-parallel round of 256x256 tiles (M = 5376, N = 3072: 252 tiles) as K grows, for
the gated-residual and the plain bf16-store epilogues (diagnostic: does a long K sweep lose L2 sharing between the
tiles of an XCD as they drift apart?)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from f_lite import _native as nat  # noqa: E402


def main():
    torch.manual_seed(0)
    M, N = 5376, 3072
    for K in (1536, 3072, 6144, 12288, 24576):
        a = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        for _ in range(3):
            nat.gemm(a, w, out=out, epilogue=nat.EPI_STORE_BF16)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(10):
            nat.gemm(a, w, out=out, epilogue=nat.EPI_STORE_BF16)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / 10 * 1e3
        print(f"K {K:6d}: {us:8.1f} us, {us / (K // 64):6.3f} us per k-tile, "
              f"{2 * M * N * K / us / 1e6 / 2516.6:.3f} of peak", flush=True)
        del a, w, out


if __name__ == "__main__":
    main()
