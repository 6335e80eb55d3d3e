"""CPU: the MXFP8 fake-quant oracle (oracle/flite_ref.py) that pins the fp8 configuration (BASELINE.json
configs[4]; the reference has no fp8 path, so these are the format's own invariants)."""
import torch

from oracle import flite_ref as R


def _x(rows=37, K=256, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(rows, K, generator=g) * torch.logspace(-4, 3, K)[None]


def test_bytes_and_dequant_agree():
    x = _x()
    q = R.mx_quant(x)
    qb, sc = R.mx_quant_bytes(x)
    assert qb.dtype == torch.uint8 and sc.shape == (2, 256, 4)
    e = sc[:, :37].permute(1, 0, 2).reshape(37, 8).to(torch.int32) - 127
    deq = (qb.view(torch.float8_e4m3fn).float().reshape(37, 8, 32) * torch.ldexp(torch.ones(()), e)[..., None])
    assert torch.equal(deq.reshape(37, 256), q)


def test_idempotent_and_bounded():
    x = _x(seed=1)
    q = R.mx_quant(x)
    assert torch.equal(R.mx_quant(q), q)
    blocks = x.reshape(37, 8, 32)
    err = (q.reshape(37, 8, 32) - blocks).abs()
    amax = blocks.abs().amax(-1, keepdim=True)
    # e4m3 (3 mantissa bits): normal elements within 2^-4 relative; everything within 2^-9 of the block max
    # scale (the subnormal step) -- amax maps into (224, 448]
    assert (err <= amax * 2.0 ** -4 + 1e-30).all()


def test_scale_exponent_is_ceil_log2_of_amax_over_448():
    x = torch.zeros(4, 128)
    x[0, 3] = 448.0       # fits exactly: e = 0
    x[1, 0] = 448.5       # just above: e = 1
    x[2, 7] = 1.0         # 1/448 -> e = -8
    qb, sc = R.mx_quant_bytes(x)
    assert sc[0, :4, 0].tolist() == [127, 128, 119, 0]  # all-zero block: E8M0 0 (2^-127)
    assert torch.equal(R.mx_quant(x)[0], x[0])
