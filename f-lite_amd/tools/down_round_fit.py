"""Down-projection (K = 12288, N = 3072, gated residual) time vs M: one exact data-parallel round (M = 5376, 252
256-row tiles) against the metric's M = 8224 (396 tiles: one data-parallel round + stream-K over 140) -- how close
the stream-K leftover phase runs to its ideal share (diagnostic)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from f_lite import _native as nat  # noqa: E402


def main():
    torch.manual_seed(0)
    ws = nat.gemm_workspace("cuda")
    N, K = 3072, 12288
    w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    res = {}
    for M in (2688, 5376, 8224, 10752):
        a = torch.randn(M, K, device="cuda").bfloat16()
        out = torch.zeros(M, N, device="cuda")
        kw = dict(epilogue=nat.EPI_RESID_F32, gate=torch.randn(2, N, device="cuda"), gate_seg_stride=N,
                  rows_per_seg=(M + 1) // 2)
        for _ in range(3):
            nat.gemm(a, w, out=out, workspace=ws, **kw)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(20):
            nat.gemm(a, w, out=out, workspace=ws, **kw)
        e.record()
        torch.cuda.synchronize()
        res[M] = s.elapsed_time(e) / 20 * 1e3
        tiles = (M + 255) // 256 * 12
        print(f"M {M:6d}: {tiles:4d} tiles = {tiles / 256:.2f} rounds, {res[M]:7.1f} us, "
              f"{res[M] / (tiles / 256):7.1f} us per round-equivalent", flush=True)
        del a, out


if __name__ == "__main__":
    main()
