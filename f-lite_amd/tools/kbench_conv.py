"""Micro-benchmark of the implicit-GEMM 3x3 convolution (flite_conv3x3_bf16) at the Flux VAE decoder shapes of
a 1024^2 image (NHWC bf16, pad 1, optional nearest-2x upsample), with torch's conv2d (MIOpen, NCHW) beside it."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
from f_lite import _native as nat

dev = "cuda"
# (h, w, cin, cout, upsample): input spatial size, channels
SHAPES = [(128, 128, 512, 512, False), (128, 128, 512, 512, True), (256, 256, 512, 512, False),
          (256, 256, 512, 512, True), (512, 512, 512, 256, False), (512, 512, 256, 256, False),
          (512, 512, 256, 256, True), (1024, 1024, 256, 128, False), (1024, 1024, 128, 128, False)]


def timeit(fn, iters=20):
    for _ in range(3):
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
    torch.manual_seed(0)
    for h, w, cin, cout, up in SHAPES:
        x = torch.randn(h, w, cin, device=dev).bfloat16()
        wt = (torch.randn(cout, cin, 3, 3, device=dev) * 0.02).bfloat16()
        b = (torch.randn(cout, device=dev) * 0.1).bfloat16()
        H, W = (2 * h, 2 * w) if up else (h, w)
        flops = 2.0 * H * W * cout * 9 * cin
        out = nat.conv3x3(x, wt, b, upsample=up)
        us = timeit(lambda: nat.conv3x3(x, wt, b, upsample=up))
        xn = x.permute(2, 0, 1).unsqueeze(0).contiguous()
        if up:
            xn = torch.nn.functional.interpolate(xn, scale_factor=2, mode="nearest")
        ref = torch.nn.functional.conv2d(xn, wt, b, padding=1)
        err = (out.permute(2, 0, 1).float() - ref[0].float()).norm() / ref.float().norm()
        ut = timeit(lambda: torch.nn.functional.conv2d(xn, wt, b, padding=1))
        print(f"conv {h}x{w} {cin}->{cout} up={int(up)}: {us:8.1f} us {flops / us / 1e6:6.0f} TF/s | "
              f"torch {ut:8.1f} us {flops / ut / 1e6:6.0f} TF/s | rel_l2 {err.item():.2e}", flush=True)


if __name__ == "__main__":
    main()
