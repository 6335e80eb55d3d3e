"""Micro-benchmark of the attention kernel at the DiT shapes (1024^2: T=4112, B=2, H=12; cross Lk=512;
1344x896: T=4720). `split` passes the tail-split workspace (attention.hip "Schedule")."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
from f_lite import _native as nat

dev = "cuda"


def run(T, Lk, H=12, iters=20, bounded=True, split=False):
    B = 2
    D = 256
    q = torch.nn.functional.normalize(torch.randn(B * T, H, D, device=dev), dim=-1).mul(16).bfloat16()
    k = torch.nn.functional.normalize(torch.randn(B * Lk, H, D, device=dev), dim=-1).mul(16).bfloat16()
    v = torch.randn(B * Lk, H, D, device=dev).bfloat16()
    cu_q = torch.tensor([0, T, 2 * T], dtype=torch.int32, device=dev)
    cu_k = torch.tensor([0, Lk, 2 * Lk], dtype=torch.int32, device=dev)
    out = torch.empty_like(q)
    ms_ = 16.5 if bounded else 0.0
    ws = nat.attn_workspace(dev, B, H) if split else None
    for _ in range(3):
        nat.attn_varlen(q, k, v, cu_q, cu_k, T, D ** -0.5, out=out, max_score=ms_, workspace=ws, max_k=Lk)
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        nat.attn_varlen(q, k, v, cu_q, cu_k, T, D ** -0.5, out=out, max_score=ms_, workspace=ws, max_k=Lk)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / iters
    fl = 4.0 * B * H * T * Lk * D
    print(f"attn T={T} Lk={Lk} bounded={bounded} split={split}: {ms * 1000:.1f} us  {fl / ms / 1e9:.0f} TF/s",
          flush=True)


if __name__ == "__main__":
    if "--only" in sys.argv:  # one configuration (counter passes): --only T Lk
        i = sys.argv.index("--only")
        run(int(sys.argv[i + 1]), int(sys.argv[i + 2]), iters=5, split=True)
        sys.exit(0)
    if "--quick" in sys.argv:  # the bounded self-attention shape: whole rounds only, then with the split tail
        run(4096, 4112, iters=50, split=False)
        run(4112, 4112, iters=50, split=True)
        sys.exit(0)
    for b, sp in ((False, False), (True, False), (True, True)):
        run(4112, 4112, bounded=b, split=sp)
        run(4112, 512, bounded=b, split=sp)
    run(4720, 4720, split=False)
    run(4720, 4720, split=True)
    if "--rounds" in sys.argv:  # schedule probes: whole rounds of 256 full q-tiles, no tails
        run(4096, 4112, split=False)
        run(4096 + 128, 4112, split=False)
        run(4096 - 1280, 4112, split=False)
        run(16, 4112, split=False)
        run(16, 4112, split=True)
        run(16, 4112, split=True, H=1)
