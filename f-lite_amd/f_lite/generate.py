"""`python -m f_lite.generate` -- the reference CLI (/root/reference/f_lite/generate.py:13-116) on the native path.

Same arguments, defaults and output naming as `generate_images` (generate.py:13-25, 93-111):

    python -m f_lite.generate --prompt "a mountain lake at sunset" --output_file out.png \
        --model /path/to/diffusers_folder --width 1344 --height 896 --steps 30 --guidance_scale 6 --seed 42

`--model` takes what can be resolved offline: a local diffusers folder (model_index.json; the reference's
LOADABLE_CLASSES registration of generate.py:61-66 is not needed), a raw `.pt` state dict (f_lite.pt), or
`random:<preset>` (7b, 10b, tiny, tiny_v2) for the synthetic seeded weights the benchmarks use. Hub names
such as the default "Freepik/F-Lite" cannot be downloaded here and raise.

Prompt embeddings: text encoding is outside this path. With no text encoder in the
pipeline, `--prompt_embeds file.safetensors` supplies them (keys `prompt_embeds` [P, L, C] and optionally
`negative_prompt_embeds`); without that file a SYNTHETIC embedding is derived deterministically from the
prompt string (a stand-in with the T5 context's shape [1, 512, C], not a text encoder) and the CLI says so.

There is no CPU fallback: the reference drops to CPU when CUDA is absent (generate.py:44-51); here the
native path needs a ROCm device and raises.
"""
from __future__ import annotations

import argparse
import zlib
from pathlib import Path
from typing import List, Optional

import torch

from .pipeline import FLitePipeline

SYNTHETIC_CONTEXT_LEN = 512  # T5 max_sequence_length of the reference encode_prompt (pipeline.py:131)


def output_paths(output_file: str, num_images: int) -> List[Path]:
    """generate.py:96-111: image 0 keeps the name; image i > 0 gets '-i' before the suffix."""
    p = Path(output_file)
    if num_images == 1:
        return [p]
    return [p.parent / f"{p.stem}{f'-{i}' if i > 0 else ''}{p.suffix}" for i in range(num_images)]


def load_pipeline(model: str, device) -> FLitePipeline:
    if model.startswith("random:"):
        from .model import PRESETS, DiT
        from .vae import AutoencoderKL

        preset = model.split(":", 1)[1]
        if preset not in PRESETS:
            raise ValueError(f"unknown preset {preset!r}; one of {sorted(PRESETS)}")
        return FLitePipeline(DiT.random(seed=0, device=device, **PRESETS[preset]),
                             AutoencoderKL.random(seed=0, device=device))
    p = Path(model)
    if p.suffix in (".pt", ".pth") and p.is_file():
        from .pt import load_f_lite_pt

        return load_f_lite_pt(p, device, dtype="bfloat16")
    if (p / "model_index.json").exists():
        return FLitePipeline.from_pretrained(p, torch_dtype=torch.bfloat16, device=device)
    raise FileNotFoundError(f"model {model!r}: not a local diffusers folder, .pt file or random:<preset> "
                            "(Hub names cannot be resolved offline)")


def synthetic_prompt_embeds(prompt: str, dim: int, device) -> torch.Tensor:
    """Deterministic stand-in for the text encoder output: the hash generator (flite_init_param) keyed by the
    prompt string, [1, 512, dim] bf16, std 1."""
    from . import _native

    ctx = torch.empty(1, SYNTHETIC_CONTEXT_LEN, dim, device=device, dtype=torch.bfloat16)
    return _native.init_param_(ctx, "prompt:" + prompt, seed=zlib.crc32(prompt.encode()) & 0xFFFF, std=1.0)


def resolve_embeds(pipe: FLitePipeline, prompt: str, negative_prompt: Optional[str], prompt_embeds: Optional[str],
                   device):
    """(prompt_embeds, negative_prompt_embeds, how) for a pipeline without a text encoder."""
    dim = pipe.dit_model.config.cross_attn_input_size
    if prompt_embeds is not None:
        from safetensors.torch import load_file

        d = load_file(str(prompt_embeds))
        pos = d["prompt_embeds"].to(device=device, dtype=torch.bfloat16)
        neg = d.get("negative_prompt_embeds")
        neg = None if neg is None else neg.to(device=device, dtype=torch.bfloat16)
        return pos, neg, f"embeddings from {prompt_embeds}"
    pos = synthetic_prompt_embeds(prompt, dim, device)
    neg = synthetic_prompt_embeds(negative_prompt, dim, device) if negative_prompt else None
    return pos, neg, "SYNTHETIC prompt embeddings (hash of the prompt text; no text encoder on this path)"


def attach_text_encoder(pipe: FLitePipeline, spec: str, tokenizer: Optional[str], device):
    """--text_encoder random:<t5 preset> (seeded synthetic T5 weights) or a local T5 folder (config.json +
    model*.safetensors); --tokenizer a local tokenizer folder (transformers AutoTokenizer, offline), else the
    byte-level SyntheticTokenizer."""
    from .text_encoder import T5_PRESETS, SyntheticTokenizer, T5Encoder

    if spec.startswith("random:"):
        preset = spec.split(":", 1)[1]
        if preset not in T5_PRESETS:
            raise ValueError(f"unknown T5 preset {preset!r}; one of {sorted(T5_PRESETS)}")
        enc = T5Encoder.random(seed=0, device=device, **T5_PRESETS[preset])
    else:
        enc = T5Encoder.from_pretrained(spec, device=device)
    if enc.config.d_model != pipe.dit_model.config.cross_attn_input_size:
        raise ValueError(f"text encoder width {enc.config.d_model} != DiT cross_attn_input_size "
                         f"{pipe.dit_model.config.cross_attn_input_size}")
    if tokenizer is not None:
        from transformers import AutoTokenizer

        tok = AutoTokenizer.from_pretrained(tokenizer, local_files_only=True)
    else:
        tok = SyntheticTokenizer(vocab_size=enc.config.vocab_size)
        print("Tokenizer: SYNTHETIC byte-level ids (no tokenizer files given)")
    pipe.text_encoder = enc
    pipe.processor = tok


def generate_images(
    prompt: str,
    output_file: str,
    model: str = "Freepik/F-Lite",
    negative_prompt: Optional[str] = None,
    seed: int = 0,
    guidance_scale: float = 6,
    steps: int = 30,
    width: int = 1344,
    height: int = 896,
    cpu_offload: bool = True,
    device: Optional[str] = None,
    num_images: int = 1,
    prompt_embeds: Optional[str] = None,
    text_encoder: Optional[str] = None,
    tokenizer: Optional[str] = None,
):
    """Generate images with the F-Lite pipeline (generate.py:13-113). Returns the written paths."""
    from . import _native

    if device is None:
        if not torch.cuda.is_available():
            raise _native.FliteError("no ROCm device: the native F-Lite path has no CPU fallback")
        device = "cuda"
    torch_device = torch.device(device)
    if torch_device.type != "cuda":
        raise _native.FliteError(f"device {device!r}: the native F-Lite path runs only on a ROCm device")
    print(f"Using device: {device}")
    print(f"Loading model: {model}")
    pipe = load_pipeline(model, torch_device)
    if text_encoder is not None:
        attach_text_encoder(pipe, text_encoder, tokenizer, torch_device)
    if cpu_offload:
        pipe.enable_model_cpu_offload()  # no-op: weights stay resident in HBM
    if pipe.vae is not None:  # generate.py:77-78
        pipe.vae.enable_slicing()
        pipe.vae.enable_tiling()
    kw = {}
    if pipe.text_encoder is None:
        pos, neg, how = resolve_embeds(pipe, prompt, negative_prompt, prompt_embeds, torch_device)
        kw = dict(prompt_embeds=pos, negative_prompt_embeds=neg)
        print(f"Prompt conditioning: {how}")
    print(f"Generating {num_images} image(s) with prompt: {prompt}")
    output = pipe(
        prompt=prompt,
        negative_prompt=negative_prompt,
        guidance_scale=guidance_scale,
        num_inference_steps=steps,
        width=width,
        height=height,
        generator=torch.Generator(device=torch_device).manual_seed(seed),
        num_images_per_prompt=num_images,
        **kw,
    )
    paths = output_paths(output_file, len(output.images))
    if paths:
        paths[0].parent.mkdir(parents=True, exist_ok=True)
    for image, path in zip(output.images, paths):
        print(f"Saving image to: {path}")
        image.save(path)
    print(f"{len(output.images)} image(s) generated successfully!")
    return paths


def build_parser() -> argparse.ArgumentParser:
    """The flags jsonargparse.auto_cli derives from generate_images (generate.py:115-116)."""
    ap = argparse.ArgumentParser(prog="python -m f_lite.generate", description=generate_images.__doc__)
    ap.add_argument("--prompt", required=True)
    ap.add_argument("--output_file", required=True)
    ap.add_argument("--model", default="Freepik/F-Lite")
    ap.add_argument("--negative_prompt", default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--guidance_scale", type=float, default=6)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--width", type=int, default=1344)
    ap.add_argument("--height", type=int, default=896)
    ap.add_argument("--cpu_offload", type=lambda s: s.lower() in ("1", "true", "yes"), default=True)
    ap.add_argument("--device", default=None)
    ap.add_argument("--num_images", type=int, default=1)
    ap.add_argument("--prompt_embeds", default=None, help="safetensors with prompt_embeds [P, L, C] "
                    "(+ negative_prompt_embeds); default: synthetic embeddings")
    ap.add_argument("--text_encoder", default=None, help="native T5 text encoder: random:<preset> "
                    "(t5-xxl, tiny) or a local T5 folder; prompts are then encoded (pipeline.py:126-175)")
    ap.add_argument("--tokenizer", default=None, help="local tokenizer folder for --text_encoder "
                    "(default: byte-level synthetic ids)")
    return ap


def main(argv=None):
    args = build_parser().parse_args(argv)
    generate_images(**vars(args))


if __name__ == "__main__":
    main()
