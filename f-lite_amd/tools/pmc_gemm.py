"""Standalone launches of the bench's dominant kernel for rocprofv3 counter passes.

    rocprofv3 --pmc FETCH_SIZE -d <dir> -- python3 f-lite_amd/tools/pmc_gemm.py [--launches N]

Runs the SwiGLU gate/up GEMM (gemm_bf16_kernel<EPI_SWIGLU_BF16>) at the 10B/1024^2 CFG shape the bench
probes (M = 2*4112 = 8224 rows, F = 12288, K = 3072), with operand tensors of the engine's sizes, a few times.
rocprofv3 7.2 crashes in --pmc passes over the full engine (Measurement), so the per-launch HBM
traffic of this kernel is collected here; the kernel, its shape and its launch configuration (stream-K workspace included) are the engine's.
"""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from f_lite import _native as nat  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=8)
    ap.add_argument("--M", type=int, default=8224)
    ap.add_argument("--F", type=int, default=12288)
    ap.add_argument("--K", type=int, default=3072)
    args = ap.parse_args()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    a = torch.randn(args.M, args.K, device=dev, generator=g).bfloat16()
    wg = (torch.randn(args.F, args.K, device=dev, generator=g) * 0.02).bfloat16()
    wu = (torch.randn(args.F, args.K, device=dev, generator=g) * 0.02).bfloat16()
    out = torch.empty(args.M, args.F, device=dev, dtype=torch.bfloat16)
    ws = nat.gemm_workspace(dev)  # the engine passes its stream-K workspace to every GEMM
    for _ in range(args.launches):
        nat.gemm(a, wg, out=out, epilogue=nat.EPI_SWIGLU_BF16, w2=wu, workspace=ws)
    torch.cuda.synchronize()
    print(f"[pmc_gemm] {args.launches} launches of SwiGLU GEMM M={args.M} F={args.F} K={args.K}")


if __name__ == "__main__":
    main()
