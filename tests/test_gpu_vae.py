"""GPU parity of the VAE decoder kernels and the whole decode against the CPU oracle (oracle/vae_ref.py).

Tolerances: conv (bf16 operands, fp32 accumulation) rel-L2 <= 1e-2; GroupNorm <= 1e-2; decoded uint8 image
PSNR >= 40 dB (peak 255) vs the fp32 restatement on identical bf16 weights and latents.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no ROCm device", allow_module_level=True)

from f_lite import _native as nat  # noqa: E402
from f_lite.vae import AutoencoderKL  # noqa: E402
from oracle import flite_ref as R  # noqa: E402
from oracle.vae_ref import RefVAEDecoder, decode_to_uint8, make_vae_state_dict  # noqa: E402

DEV = "cuda"


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return ((a - b).norm() / b.norm()).item()


@pytest.mark.parametrize("h,w,cin,cout,up", [(8, 8, 64, 64, False), (16, 12, 128, 256, False),
                                             (8, 8, 128, 128, True), (32, 32, 256, 128, False),
                                             (16, 16, 64, 3, False)])
def test_conv3x3(h, w, cin, cout, up):
    x = torch.randn(1, cin, h, w, device=DEV).bfloat16()
    wt = (torch.randn(cout, cin, 3, 3, device=DEV) / (9 * cin) ** 0.5).bfloat16()
    b = (0.1 * torch.randn(cout, device=DEV)).bfloat16()
    xi = F.interpolate(x.float(), scale_factor=2.0, mode="nearest") if up else x.float()
    ref = F.conv2d(xi.cpu(), wt.float().cpu(), b.float().cpu(), padding=1)[0].permute(1, 2, 0)
    out = nat.conv3x3(x[0].permute(1, 2, 0).contiguous(), wt, b, upsample=up, out_f32=True)
    assert rel(out, ref) < 1e-4
    out16 = nat.conv3x3(x[0].permute(1, 2, 0).contiguous(), wt, b, upsample=up)
    assert rel(out16, ref) < 1e-2


def test_conv3x3_residual():
    x = torch.randn(1, 64, 10, 10, device=DEV).bfloat16()
    wt = (torch.randn(64, 64, 3, 3, device=DEV) / 24).bfloat16()
    b = (0.1 * torch.randn(64, device=DEV)).bfloat16()
    r = torch.randn(10, 10, 64, device=DEV).bfloat16()
    ref = F.conv2d(x.float().cpu(), wt.float().cpu(), b.float().cpu(), padding=1)[0].permute(1, 2, 0) + r.float().cpu()
    out = nat.conv3x3(x[0].permute(1, 2, 0).contiguous(), wt, b, resid=r)
    assert rel(out, ref) < 1e-2


@pytest.mark.parametrize("C,silu", [(128, True), (256, False), (512, True)])
def test_group_norm(C, silu):
    rows = 1000
    x = (torch.randn(rows, C, device=DEV) * 2 + 0.5).bfloat16()
    g = (1 + 0.1 * torch.randn(C, device=DEV)).bfloat16()
    b = (0.1 * torch.randn(C, device=DEV)).bfloat16()
    y = nat.group_norm(x, 32, g, b, silu=silu)
    xr = x.float().cpu().t()[None]  # [1, C, rows]
    ref = F.group_norm(xr, 32, g.float().cpu(), b.float().cpu(), eps=1e-6)[0].t()
    if silu:
        ref = F.silu(ref)
    assert rel(y, ref) < 1e-2


@pytest.mark.parametrize("lh,lw", [(8, 8), (16, 12)])
def test_vae_decode_uint8(lh, lw):
    vae = AutoencoderKL.random(seed=0)
    ref = RefVAEDecoder(make_vae_state_dict(seed=0))
    g = torch.Generator().manual_seed(lh * lw)
    lat = torch.randn(2, 16, lh, lw, generator=g)
    img = vae.decode_to_uint8(lat.to(DEV))
    rimg = decode_to_uint8(ref, lat)
    assert img.shape == rimg.shape == (2, 8 * lh, 8 * lw, 3)
    p = R.psnr(img.float().cpu(), rimg.float(), peak=255.0)
    print(f"VAE {lh}x{lw} uint8 PSNR vs fp32 oracle: {p:.2f} dB")
    assert p >= 40.0
