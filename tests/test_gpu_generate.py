"""GPU: the `f_lite.generate` drop-in end to end (reference generate.py:13-113) and FLitePipeline.__call__ to
PIL images (pipeline.py:187-331), pinned by image PSNR against the CPU oracle (SURVEY §8c harness rows).

The tiny preset stands in for a checkpoint (none is reachable offline); the VAE is the FLUX-config decoder on
seeded weights. The CPU reference image: the fp32 sampling-loop oracle (oracle/flite_ref.py: sample) and the VAE
restatement (oracle/vae_ref.py) on the same latents and embeddings.
"""
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no ROCm device", allow_module_level=True)

from f_lite import DiT, FLitePipeline  # noqa: E402
from f_lite.model import PRESETS  # noqa: E402
from oracle import flite_ref as R  # noqa: E402
from oracle import vae_ref as VR  # noqa: E402

ROOT = Path(__file__).resolve().parents[1]


def psnr_u8(a, b):
    mse = ((a.astype(np.float64) - b.astype(np.float64)) ** 2).mean()
    return float("inf") if mse == 0 else 10 * np.log10(255.0 ** 2 / mse)


def test_call_to_pil_matches_cpu_oracle():
    from f_lite.vae import AutoencoderKL

    m = DiT.random(seed=0, device="cuda", **PRESETS["tiny"])
    vae = AutoencoderKL.random(seed=0, device="cuda")
    pipe = FLitePipeline(m, vae)
    g = torch.Generator().manual_seed(4)
    lat = torch.randn(1, 16, 16, 16, generator=g).bfloat16()
    pos = torch.randn(1, 24, 128, generator=g).bfloat16()
    out = pipe(prompt_embeds=pos.cuda(), latents=lat.cuda(), height=128, width=128, num_inference_steps=4,
               guidance_scale=6.0)  # output_type="pil" (the reference default)
    from PIL import Image

    assert len(out.images) == 1 and isinstance(out.images[0], Image.Image)
    assert out.images[0].size == (128, 128) and out.images[0].mode == "RGB"
    ref_lat = R.sample(R.RefDiT.random(R.PRESETS["tiny"], dtype=torch.float32), lat.float(), pos.float(),
                       torch.zeros_like(pos.float()), num_steps=4, guidance_scale=6.0, height=128, width=128,
                       t_dtype=torch.bfloat16, acc_dtype=torch.float32)
    dec = VR.RefVAEDecoder(VR.make_vae_state_dict())
    ref_img = VR.decode_to_uint8(dec, ref_lat, vae.config.scaling_factor, vae.config.shift_factor)[0].numpy()
    p = psnr_u8(np.asarray(out.images[0]), ref_img)
    print(f"__call__ -> PIL image vs CPU oracle image: {p:.2f} dB")
    assert p >= 30.0


def test_generate_cli_writes_named_pngs(tmp_path):
    """python -m f_lite.generate ... --num_images 2 -> out.png, out-1.png (generate.py:96-111)."""
    out = tmp_path / "img.png"
    cmd = [sys.executable, "-m", "f_lite.generate", "--prompt", "a lighthouse at dusk", "--output_file", str(out),
           "--model", "random:tiny", "--width", "128", "--height", "128", "--steps", "3", "--num_images", "2",
           "--seed", "7"]
    env = dict(__import__("os").environ, PYTHONPATH=f"{ROOT / 'f-lite_amd'}:{ROOT}")
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "SYNTHETIC prompt embeddings" in r.stdout
    from PIL import Image

    a = np.asarray(Image.open(out).convert("RGB"))
    b = np.asarray(Image.open(tmp_path / "img-1.png").convert("RGB"))
    assert a.shape == b.shape == (128, 128, 3)
    assert not np.array_equal(a, b)  # two images of the batch: different noise
    # deterministic for a seed
    r2 = subprocess.run(cmd[:-1] + ["7"], env=env, capture_output=True, text=True, timeout=240)
    assert r2.returncode == 0
    assert np.array_equal(np.asarray(Image.open(out).convert("RGB")), a)
