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


@pytest.mark.parametrize("lh,lw", [(8, 8), (16, 12), (128, 128)])
def test_vae_decode_uint8(lh, lw):
    """(128, 128) is the metric workload's full 1024^2 decode (one image): the mid-block attention runs over
    16384 tokens (its 1 GiB fp32 score matrix and softmax_rows_kernel) and every up-block at full size."""
    vae = AutoencoderKL.random(seed=0)
    ref = RefVAEDecoder(make_vae_state_dict(seed=0))
    g = torch.Generator().manual_seed(lh * lw)
    lat = torch.randn(2 if lh * lw < 4096 else 1, 16, lh, lw, generator=g)
    img = vae.decode_to_uint8(lat.to(DEV))
    rimg = decode_to_uint8(ref, lat)
    assert img.shape == rimg.shape == (lat.shape[0], 8 * lh, 8 * lw, 3)
    p = R.psnr(img.float().cpu(), rimg.float(), peak=255.0)
    print(f"VAE {lh}x{lw} uint8 PSNR vs fp32 oracle: {p:.2f} dB")
    assert p >= 40.0


def _mx_conv_weight(w):
    """Fake-quantise a [Cout, Cin, 3, 3] weight the way the engine stores it: packed [Cout][ky][kx][Cin_pad64],
    MXFP8 per 32 along that row (blocks never straddle a tap since Cin_pad is a multiple of 64)."""
    cout, cin = w.shape[:2]
    cpad = (cin + 63) // 64 * 64
    t = F.pad(w.permute(0, 2, 3, 1), (0, cpad - cin)).reshape(cout, 9 * cpad)
    t = R.mx_quant(t).reshape(cout, 3, 3, cpad)[..., :cin]
    return t.permute(0, 3, 1, 2).contiguous()


# fp8 VAE (diffusers enable_layerwise_casting with an fp8 storage dtype): the 3x3 conv weights
# are stored as MXFP8 and expanded to bf16 per conv. Parity target: the fp32 oracle decoder run on the same
# fake-quantised weights (>= 40 dB, the bar of the bf16 decode); the distance to the bf16-weight decode is the
# quantisation cost, reported.
def test_vae_decode_fp8_weights():
    vae = AutoencoderKL.random(seed=0)
    sd = make_vae_state_dict(seed=0)
    sdq = {k: (_mx_conv_weight(v) if v.dim() == 4 and v.shape[-1] == 3 else v) for k, v in sd.items()}
    lat = torch.randn(1, 16, 8, 8, generator=torch.Generator().manual_seed(11))
    bf = vae.decode_to_uint8(lat.to(DEV))
    vae.enable_layerwise_casting(torch.float8_e4m3fn, torch.bfloat16)
    img = vae.decode_to_uint8(lat.to(DEV))
    assert torch.equal(img, vae.decode_to_uint8(lat.to(DEV)))
    p = R.psnr(img.float().cpu(), decode_to_uint8(RefVAEDecoder(sdq), lat).float(), peak=255.0)
    cost = R.psnr(img.float().cpu(), bf.float().cpu(), peak=255.0)
    print(f"VAE fp8 weights 8x8: {p:.2f} dB vs the oracle on MX-quantised weights, {cost:.2f} dB vs bf16 weights")
    assert p >= 40.0
    assert not torch.equal(img, bf)
    vae.disable_layerwise_casting()
    assert torch.equal(vae.decode_to_uint8(lat.to(DEV)), bf)


# Tiled decode (diffusers AutoencoderKL.tiled_decode, on in the reference via generate.py:77-78) against the oracle
# restatement, at a reduced tile size so the oracle stays cheap: tile_latent 16 (128 px), stride 12, 32-px blends,
# 96-px crops; 20 x 28 latents give a 2 x 3 grid with 8-row and 4-column edge tiles.
def test_vae_decode_tiled_uint8():
    from oracle.vae_ref import tiled_decode_to_uint8

    vae = AutoencoderKL.random(seed=0)
    vae.enable_tiling()
    vae.tile_latent_min_size, vae.tile_sample_min_size = 16, 128
    ref = RefVAEDecoder(make_vae_state_dict(seed=0))
    g = torch.Generator().manual_seed(7)
    lat = torch.randn(1, 16, 20, 28, generator=g)
    img = vae.decode_to_uint8(lat.to(DEV))
    rimg = tiled_decode_to_uint8(ref, lat, tile_latent=16, tile_sample=128)
    assert img.shape == rimg.shape == (1, 160, 224, 3)
    p = R.psnr(img.float().cpu(), rimg.float(), peak=255.0)
    print(f"VAE tiled 20x28 (tile 16) uint8 PSNR vs fp32 oracle: {p:.2f} dB")
    assert p >= 40.0
    again = vae.decode_to_uint8(lat.to(DEV))
    assert torch.equal(img, again)
    vae.disable_tiling()
    untiled = vae.decode_to_uint8(lat.to(DEV))
    assert not torch.equal(img, untiled)  # the tiles see only their own window (mid-block attention is global)


def test_vae_decode_tiled_default_grid():
    # the reference's default generate.py resolution: 1344 x 896 -> latents 112 x 168 > 128: 1 x 2 tiles of
    # 128 latents (stride 96, 256-px blends, 768-px crops) on the full-size Flux VAE, against the oracle's tiled
    # decode at the same default tile geometry
    from oracle.vae_ref import tiled_decode_to_uint8

    vae = AutoencoderKL.random(seed=0)
    vae.enable_tiling()
    lat = torch.randn(1, 16, 112, 168, generator=torch.Generator().manual_seed(3))
    img = vae.decode_to_uint8(lat.to(DEV))
    assert img.shape == (1, 896, 1344, 3)
    assert torch.equal(img, vae.decode_to_uint8(lat.to(DEV)))
    assert img.float().std().item() > 1.0
    rimg = tiled_decode_to_uint8(RefVAEDecoder(make_vae_state_dict(seed=0)), lat)
    p = R.psnr(img.float().cpu(), rimg.float(), peak=255.0)
    print(f"VAE tiled 112x168 (default tiles) uint8 PSNR vs fp32 oracle: {p:.2f} dB")
    assert p >= 40.0
