"""Bit-equality check of two builds of the attention kernel (e.g. a restructured key loop against the previous one).

    FLITE_LIB=a.so python f-lite_amd/tools/attn_equal.py dump out_a.pt
    FLITE_LIB=b.so python f-lite_amd/tools/attn_equal.py dump out_b.pt
    python f-lite_amd/tools/attn_equal.py compare out_a.pt out_b.pt
Cases: the DiT self/cross shapes with and without the tail split, ragged sequences, single-tile sequences.
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

CASES = [([4112, 4112], None, 12, True), ([4112, 4112], [512, 512], 12, True), ([4112, 4112], None, 12, False),
         ([300, 200], None, 2, True), ([130, 255], [24, 17], 2, True), ([64], [1], 1, False), ([80, 80], None, 2, False),
         ([1000, 77], [700, 0], 3, True), ([50], [4096], 1, True), ([129], [130], 2, False)]


def dump(path):
    from f_lite import _native as nat

    dev = "cuda"
    outs = []
    for lens_q, lens_k, H, split in CASES:
        lens_k = lens_q if lens_k is None else lens_k
        D = 256
        cu_q = torch.tensor([0] + list(torch.tensor(lens_q).cumsum(0)), dtype=torch.int32)
        cu_k = torch.tensor([0] + list(torch.tensor(lens_k).cumsum(0)), dtype=torch.int32)
        g = torch.Generator(device=dev).manual_seed(sum(lens_q) + H)
        q = torch.nn.functional.normalize(torch.randn(int(cu_q[-1]), H, D, device=dev, generator=g), dim=-1)
        k = torch.nn.functional.normalize(torch.randn(max(int(cu_k[-1]), 1), H, D, device=dev, generator=g), dim=-1)
        v = torch.randn(max(int(cu_k[-1]), 1), H, D, device=dev, generator=g).bfloat16()
        q, k = (q * 16).bfloat16(), (k * 16).bfloat16()
        ws = nat.attn_workspace(dev, len(lens_q), H) if split else None
        o = nat.attn_varlen(q, k, v, cu_q.to(dev), cu_k.to(dev), max(lens_q), D ** -0.5, max_score=16.5, workspace=ws,
                            max_k=max(lens_k))
        outs.append(o.cpu())
    torch.save(outs, path)
    print(f"dumped {len(outs)} cases to {path}", flush=True)


def compare(a, b):
    A, B = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    bad = 0
    for i, (x, y) in enumerate(zip(A, B)):
        # bit patterns, so NaNs in the same places compare equal
        eq = torch.equal(x.view(torch.int16), y.view(torch.int16))
        diff = (x.float() - y.float()).abs().nan_to_num(0.0).max().item()
        nans = (int(x.float().isnan().sum()), int(y.float().isnan().sum()))
        print(f"case {i} {CASES[i][:3]}: {'identical' if eq else 'DIFFERENT'} (max abs diff {diff:.3e}, NaNs {nans})",
              flush=True)
        bad += not eq
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        compare(sys.argv[2], sys.argv[3])
