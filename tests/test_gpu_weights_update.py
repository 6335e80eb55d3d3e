"""GPU: derived weight copies follow IN-PLACE weight updates (load_state_dict copies into the existing storage,
so the parameter pointers do not change; only their version counters do).

The bf16 DiT path reads the bound storage directly; the fp8 path runs on engine-owned MXFP8 copies and the VAE
on engine-owned packed conv weights -- both must be remade (include/flite.h flite_dit_weights_updated /
flite_vae_weights_updated). Bar: after sample -> load_state_dict(new) -> sample, the output is bit-identical to a
model built fresh from the new weights, in bf16 and fp8 modes (including the hipGraph replay and an fp8
off/update/on toggle) and for the VAE in bf16 and fp8 weight storage."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no ROCm device", allow_module_level=True)

from f_lite import DiT, FLitePipeline  # noqa: E402
from f_lite.model import PRESETS  # noqa: E402
from f_lite.vae import AutoencoderKL  # noqa: E402

DEV = "cuda"


def _inputs():
    g = torch.Generator().manual_seed(13)
    lat = torch.randn(1, 16, 16, 16, generator=g).bfloat16().to(DEV)
    pos = torch.randn(1, 24, 128, generator=g).bfloat16().to(DEV)
    return lat, pos


def _sample(m, graph=True):
    lat, pos = _inputs()
    return FLitePipeline(m)(prompt_embeds=pos, latents=lat, height=128, width=128, num_inference_steps=4,
                            guidance_scale=6.0, output_type="latent", use_graph=graph).images.float().cpu()


def _fresh(seed, fp8):
    m = DiT.random(seed=seed, device=DEV, **PRESETS["tiny"])
    if fp8:
        m.enable_fp8(True)
    return m


@pytest.mark.parametrize("fp8", [False, True])
def test_dit_load_state_dict_in_place(fp8):
    m = _fresh(0, fp8)
    before = _sample(m)
    new_sd = DiT.random(seed=1, device=DEV, **PRESETS["tiny"]).state_dict()
    ptrs = [p.data_ptr() for p in m.parameters()]
    m.load_state_dict(new_sd)  # copies into the existing storage
    assert ptrs == [p.data_ptr() for p in m.parameters()]
    after = _sample(m)  # the cached hipGraph replays on the same pointers
    want = _sample(_fresh(1, fp8))
    assert not torch.equal(before, after)
    assert torch.equal(after, want)
    assert torch.equal(_sample(m, graph=False), want)


def test_dit_fp8_toggle_after_update():
    """enable_fp8(False) -> update -> enable_fp8(True) requantises (the copies from before are stale)."""
    m = _fresh(0, True)
    _sample(m)
    m.enable_fp8(False)
    m.load_state_dict(DiT.random(seed=2, device=DEV, **PRESETS["tiny"]).state_dict())
    m.enable_fp8(True)
    assert torch.equal(_sample(m), _sample(_fresh(2, True)))


def test_dit_random_init_in_place_and_rebind_keep_fp8():
    """random_init_ writes through raw pointers (no version bump): tracked by the model; rebinding one weight
    to NEW storage keeps fp8 mode on and requantises before the next run (flite.h flite_dit_enable_fp8)."""
    m = _fresh(0, True)
    _sample(m)
    m.random_init_(seed=4)
    assert torch.equal(_sample(m), _sample(_fresh(4, True)))
    w = m.blocks[1].mlp.down_proj
    w.weight = torch.nn.Parameter(w.weight.detach().clone() * 0.5)  # new storage
    ref = _fresh(4, False)
    with torch.no_grad():
        ref.blocks[1].mlp.down_proj.weight.mul_(0.5)
    ref.enable_fp8(True)
    got = _sample(m)
    assert torch.equal(got, _sample(ref))
    m.enable_fp8(False)
    assert not torch.equal(got, _sample(m))  # it really was the fp8 path


@pytest.mark.parametrize("fp8", [False, True])
def test_vae_load_state_dict_in_place(fp8):
    lat = torch.randn(1, 16, 8, 8, generator=torch.Generator().manual_seed(5)).to(DEV)

    def make(seed):
        v = AutoencoderKL.random(seed=seed)
        if fp8:
            v.enable_layerwise_casting(torch.float8_e4m3fn, torch.bfloat16)
        return v

    v = make(0)
    before = v.decode_to_uint8(lat).cpu()
    v.load_state_dict(AutoencoderKL.random(seed=1).state_dict())
    after = v.decode_to_uint8(lat).cpu()
    want = make(1).decode_to_uint8(lat).cpu()
    assert not torch.equal(before, after)
    assert torch.equal(after, want)
