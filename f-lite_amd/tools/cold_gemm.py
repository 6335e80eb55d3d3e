"""Which cold operand costs the DiT GEMMs their in-pipeline time (diagnostic, GPU box).

In the sampling loop the proj / cross-q / qkv GEMMs run 11-16 % slower than back-to-back in a micro-benchmark
(profiles/r02al vs r02an). Between two uses of a block's weights the loop streams ~10 GB, so every launch starts
with its weights (and often its activations) beyond the 256 MiB Infinity Cache. This times single launches after
a 1 GiB flush write, optionally re-touching one operand (weights W, activations A, the fp32 residual x of the
gated epilogue) right before, or rewriting A (A_written: what a producing kernel leaves), against warm
back-to-back launches.
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402
from f_lite import _native as nat  # noqa: E402

SHAPES = [  # name, M, N, K, epilogue
    ("proj", 8224, 3072, 3072, "resid"),
    ("cross_q", 8224, 3072, 3072, "store"),
    ("qkv", 8224, 9216, 3072, "store"),
    ("gateup", 8224, 24576, 3072, "swiglu"),
]


def main(reps=8):
    torch.manual_seed(0)
    ws = nat.gemm_workspace("cuda")
    flush = torch.empty(1 << 28, device="cuda")  # 1 GiB
    for name, M, N, K, epi in SHAPES:
        a = torch.randn(M, K, device="cuda").bfloat16()
        x = None
        if epi == "swiglu":
            w = (torch.randn(N // 2, K, device="cuda") * 0.05).bfloat16()
            w2 = (torch.randn(N // 2, K, device="cuda") * 0.05).bfloat16()
            out = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
            kw = dict(epilogue=nat.EPI_SWIGLU_BF16, w2=w2)
            wts = [w, w2]
        elif epi == "resid":
            w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
            out = x = torch.zeros(M, N, device="cuda")
            kw = dict(epilogue=nat.EPI_RESID_F32, gate=torch.randn(1, N, device="cuda"), gate_seg_stride=0,
                      rows_per_seg=M)
            wts = [w]
        else:
            w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            kw = dict(epilogue=nat.EPI_STORE_BF16)
            wts = [w]
        run = lambda: nat.gemm(a, w, out=out, workspace=ws, **kw)  # noqa: E731
        sink = torch.zeros(1, device="cuda")

        def touch(t):  # read every byte once (a reduction: no temporary copy of t)
            sink.add_(t.sum().float() * 0)  # noqa: B023

        modes = {"warm": None, "cold": [], "cold+W": wts, "cold+A": [a], "cold+A_written": ["write", a],
                 "cold+A_written+read": ["write+read", a]}
        if x is not None:
            modes["cold+x"] = [x]
        line = [name]
        for mode, pre in modes.items():
            ts = []
            for _ in range(reps):
                if pre is not None:
                    flush.fill_(1.0)
                    if pre and isinstance(pre[0], str):  # rewrite the operand (as the producing kernel would)
                        for t in pre[1:]:
                            t.normal_()
                            if pre[0] == "write+read":  # and read it back in another kernel
                                touch(t)
                    else:
                        for t in pre:
                            touch(t)
                else:
                    run()
                s = torch.cuda.Event(enable_timing=True)
                e = torch.cuda.Event(enable_timing=True)
                s.record()
                run()
                e.record()
                torch.cuda.synchronize()
                ts.append(s.elapsed_time(e) * 1e3)
            ts.sort()
            line.append(f"{mode} {ts[len(ts) // 2]:.1f}us")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
