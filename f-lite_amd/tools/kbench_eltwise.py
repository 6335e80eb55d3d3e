"""Micro-benchmark of the HBM-bound kernels of the DiT step at the 10B/1024^2 CFG shape (M = 8224 rows,
D = 3072), with a torch device-copy of the same byte count as the box's bandwidth reference."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
from f_lite import _native as nat

dev = "cuda"
M, D, T = 8224, 3072, 4112


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0  # us


def main():
    x = torch.randn(M, D, device=dev)
    w = (1 + 0.1 * torch.randn(D, device=dev)).bfloat16()
    shift = torch.randn(2, D, device=dev) * 0.1
    scale = torch.randn(2, D, device=dev) * 0.1
    y = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    us = timeit(lambda: nat.rmsnorm_modulate(x, w, shift, scale, seg_rows=T, out=y))
    by = M * D * 4 + M * D * 2
    print(f"rmsnorm_mod  M={M} D={D}: {us:7.1f} us  {by / us / 1e6:6.2f} TB/s (x fp32 in, bf16 out)", flush=True)
    qkv = torch.randn(M, 3 * D, device=dev).bfloat16()
    cos, sin = nat.rope_tables(64, 64, 16, 10000.0, round_bf16=True)
    us = timeit(lambda: nat.rope_qknorm_(qkv, heads=24, rope_heads=24, cos=cos, sin=sin, tokens_per_seq=T))
    by = 2 * M * 2 * D * 2
    print(f"rope_qknorm  M={M} heads=24: {us:7.1f} us  {by / us / 1e6:6.2f} TB/s (q, k in place)", flush=True)
    src = torch.empty(by // 2, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    us = timeit(lambda: dst.copy_(src))
    print(f"torch copy {by / 2 / 1e6:.0f} MB: {us:7.1f} us  {by / us / 1e6:6.2f} TB/s (read + write)", flush=True)


if __name__ == "__main__":
    main()
