"""Would a launch mixing the two attention kernels beat the 128-row kernel at 1024^2? (diagnostic)

The metric's self-attention is 2 sequences x 12 heads x 4112 rows over 4112 keys: 768 + tails 128-row q-tiles
(3 exact rounds) or 384 + tails 256-row tiles (1.5 rounds). Timed here as two back-to-back launches: (a) the
256-row kernel on 8 heads x 2 sequences x 4096 rows (256 whole tiles: one exact round), then (b) the 128-row kernel
on the other 4 heads x 2 sequences x 4112 rows (256 q-tiles + tails), against (c) the 128-row kernel on everything.
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from f_lite import _native as nat  # noqa: E402


def make(B, T, H, Tq=None):
    D = 256
    Tq = T if Tq is None else Tq
    q = torch.nn.functional.normalize(torch.randn(B * Tq, H, D, device="cuda"), dim=-1).mul(16).bfloat16()
    k = torch.nn.functional.normalize(torch.randn(B * T, H, D, device="cuda"), dim=-1).mul(16).bfloat16()
    v = torch.randn(B * T, H, D, device="cuda").bfloat16()
    cu_q = torch.tensor([0, Tq, 2 * Tq], dtype=torch.int32, device="cuda")
    cu_k = torch.tensor([0, T, 2 * T], dtype=torch.int32, device="cuda")
    ws = nat.attn_workspace("cuda", B, H, Tq, T)
    return (q, k, v, cu_q, cu_k, Tq, D ** -0.5), ws, T


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    torch.manual_seed(0)
    full, wsf, T = make(2, 4112, 12)
    a, wsa, _ = make(2, 4112, 8, Tq=4096)
    b, wsb, _ = make(2, 4112, 4)

    def run(args, ws, mode, max_k):
        nat.attn_set_q256(mode)
        nat.attn_varlen(*args, max_score=16.5, workspace=ws, max_k=max_k)

    for r in range(3):
        t_full = timeit(lambda: run(full, wsf, 0, T))
        t_a = timeit(lambda: run(a, wsa, 1, T))
        t_b = timeit(lambda: run(b, wsb, 0, T))
        t_ab = timeit(lambda: (run(a, wsa, 1, T), run(b, wsb, 0, T)))
        print(f"round {r}: 128-row everything {t_full:.1f} us; 256-row 8 heads x 4096 rows {t_a:.1f} + 128-row 4 heads "
              f"{t_b:.1f} = {t_a + t_b:.1f} us; back to back {t_ab:.1f} us", flush=True)
    nat.attn_set_q256(2)


if __name__ == "__main__":
    main()
