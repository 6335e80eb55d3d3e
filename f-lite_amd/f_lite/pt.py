"""`f_lite.pt.load_f_lite_pt` -- a raw `.pt` DiT state dict into an FLitePipeline on the native path.

Mirrors /root/reference/f_lite/pt.py:15-179: depth inferred from the largest block index (pt.py:84-86),
num_heads = width // 256 (pt.py:89), the DDP / torch.compile key prefixes stripped (pt.py:98-101). The
model_v2.py (per-block adaLN) layout is recognised from its keys.

Differences, each one a consequence of this path's scope:
  * the checkpoint is read with torch.load(weights_only=True): nothing in the file is executed;
  * missing keys raise (the reference's strict=False leaves them at their init values; here the storage is
    uninitialised device memory, so running with a missing tensor would be silently wrong);
  * residual_v defaults to False: the reference's default (True) names a value-residual DiT that its own
    model.py does not accept (stale); True raises here too;
  * a LoRA adapter (lora_path, pt.py:107-135) is folded into the weights (f_lite/lora.py) instead of kept as
    unmerged peft modules: same function, the native GEMMs unchanged. As in the reference, the adapter's scaling
    is lora_alpha / r = 1 and lora_scale is not applied (pt.py:130 only logs it). The T5 encoder and its tokenizer come from
    `text_encoder_path` as in pt.py:147-155 (subfolders text_encoder_2 / tokenizer_2 of a local FLUX-layout
    folder; the encoder runs natively, f_lite.text_encoder.T5Encoder); without it the pipeline takes
    prompt_embeds. The Flux VAE is loaded from `vae_path` (a local diffusers folder) when given -- hub names
    cannot be resolved offline, which is also why neither path defaults to "black-forest-labs/FLUX.1-schnell";
  * compile_model is a no-op: the denoise loop is already one hipGraph.
"""
from __future__ import annotations

import logging
from pathlib import Path
from typing import Optional, Union

import torch

from .model import DiT, clean_state_dict
from .pipeline import FLitePipeline

logger = logging.getLogger(__name__)

_DTYPES = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}


def infer_dit_config(state_dict, patch_size=2, width=3072, mlp_ratio=4.0, cross_attn_input_size=4096,
                     train_bias_and_rms=False):
    """DiT constructor kwargs for a raw state dict (pt.py:84-96) and whether it is the model_v2 layout."""
    blocks = [int(k.split(".")[1]) for k in state_dict if k.startswith("blocks.")]
    if not blocks:
        raise ValueError("state dict has no blocks.* keys: not an F-Lite DiT checkpoint")
    depth = max(blocks) + 1
    per_block = any(k.startswith("blocks.") and ".adaLN_modulation." in k for k in state_dict)
    cfg = dict(in_channels=16, patch_size=patch_size, depth=depth, num_heads=width // 256, mlp_ratio=mlp_ratio,
               cross_attn_input_size=cross_attn_input_size, hidden_size=width,
               train_bias_and_rms=train_bias_and_rms, per_block_adaln=per_block)
    return cfg


def load_f_lite_pt(
    model_path: Union[str, Path],
    device: torch.device,
    dtype: str = "float32",
    vae_path: Optional[Union[str, Path]] = None,
    text_encoder_path: Optional[Union[str, Path]] = None,
    lora_path: Optional[Union[str, Path]] = None,
    lora_scale: float = 1.0,
    lora_rank: int = 128,
    lora_target_modules: str = "qkv,q,context_kv,proj",
    patch_size: int = 2,
    width: int = 3072,
    mlp_ratio: float = 4.0,
    cross_attn_input_size: int = 4096,
    residual_v: bool = False,
    train_bias_and_rms: bool = False,
    enable_vae_slicing: bool = True,
    enable_vae_tiling: bool = False,
    compile_model: bool = False,
) -> FLitePipeline:
    """Load an F-Lite DiT from a .pt state dict (pt.py:15-179). `dtype` names the model dtype as in the
    reference; the native path computes in bf16, so float32/float16 requests are loaded as bf16 with a
    warning (the reference itself converts to bf16 right after: f_lite_to_hf.py:86)."""
    if residual_v:
        raise NotImplementedError("residual_v=True: the value-residual DiT is not in f_lite/model.py (pt.py:93 is "
                                  "stale against the reference's own DiT)")
    if dtype not in _DTYPES:
        raise ValueError(f"dtype must be one of {sorted(_DTYPES)}")
    if _DTYPES[dtype] != torch.bfloat16:
        logger.warning("load_f_lite_pt: the native DiT computes in bf16; loading %s weights as bf16", dtype)
    sd = torch.load(str(model_path), map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "state_dict" in sd and isinstance(sd["state_dict"], dict):
        sd = sd["state_dict"]
    sd = clean_state_dict(sd)
    cfg = infer_dit_config(sd, patch_size, width, mlp_ratio, cross_attn_input_size, train_bias_and_rms)
    logger.info("Inferred model depth from state dict: %d", cfg["depth"])
    with torch.device("meta"):
        probe = DiT(**cfg)
    expected = set(probe.state_dict())
    missing = sorted(expected - set(sd))
    unexpected = sorted(set(sd) - expected)
    if missing:
        raise KeyError(f"checkpoint lacks {len(missing)} DiT tensors, e.g. {missing[:4]}")
    if unexpected:  # the reference loads with strict=False and logs the status (pt.py:104-105)
        logger.warning("ignoring %d unexpected keys, e.g. %s", len(unexpected), unexpected[:4])
        sd = {k: v for k, v in sd.items() if k in expected}
    dit = DiT.from_state_dict(sd, device=device, torch_dtype=torch.bfloat16, **cfg)
    if lora_path is not None:  # pt.py:107-135
        from .lora import merge_lora_

        logger.info("Loading LoRA weights from %s", lora_path)
        lsd = torch.load(str(lora_path), map_location="cpu", weights_only=True)
        merge_lora_(dit, lsd, scaling=1.0, target_modules=lora_target_modules.split(","), rank=lora_rank)
        logger.info("Successfully loaded LoRA weights with scale %s", lora_scale)
    vae = None
    if vae_path is not None:
        from .vae import AutoencoderKL

        p = Path(vae_path)
        vae = AutoencoderKL.from_pretrained(p / "vae" if (p / "vae").exists() else p, device=device)
    else:
        logger.warning("no vae_path: the Flux VAE cannot be fetched offline; decode needs a VAE "
                       "(output_type='latent' works without one)")
    text_encoder, tokenizer = None, None
    if text_encoder_path is not None:  # pt.py:147-155
        text_encoder, tokenizer = load_t5_from_folder(text_encoder_path, device)
    else:
        logger.warning("no text_encoder_path: T5 cannot be fetched offline; pass prompt_embeds to the pipeline")
    pipe = FLitePipeline(dit_model=dit, vae=vae, text_encoder=text_encoder, tokenizer=tokenizer)
    if enable_vae_slicing:
        pipe.enable_vae_slicing()
    if enable_vae_tiling:
        pipe.enable_vae_tiling()
    if compile_model:
        logger.info("compile_model: the native denoise loop is captured in a hipGraph already")
    return pipe


def load_t5_from_folder(path: Union[str, Path], device):
    """T5 encoder + tokenizer from a local FLUX-layout folder (pt.py:149-155: subfolders text_encoder_2 and
    tokenizer_2; a folder holding config.json directly is taken as the encoder itself). The encoder runs on the
    native path (bf16, as pt.py's torch_dtype); the tokenizer is transformers' fast tokenizer loaded offline."""
    from .text_encoder import T5Encoder

    p = Path(path)
    enc_dir = p / "text_encoder_2" if (p / "text_encoder_2" / "config.json").exists() else p
    text_encoder = T5Encoder.from_pretrained(enc_dir, torch_dtype=torch.bfloat16, device=device)
    tok_dir = next((d for d in (p / "tokenizer_2", p / "tokenizer", p) if (d / "tokenizer_config.json").exists()
                    or (d / "tokenizer.json").exists() or (d / "spiece.model").exists()), None)
    if tok_dir is None:
        raise FileNotFoundError(f"no tokenizer files under {p} (tokenizer_2/ as pt.py:150 expects)")
    from transformers import AutoTokenizer

    tokenizer = AutoTokenizer.from_pretrained(str(tok_dir), local_files_only=True)
    return text_encoder, tokenizer
