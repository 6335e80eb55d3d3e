"""FLitePipeline -- the F-Lite text-to-image sampling path, MI355X-native.

Drop-in for the reference `f_lite.pipeline.FLitePipeline` (/root/reference/f_lite/pipeline.py:46-331):
same constructor components (dit_model, vae, text_encoder, processor), same `__call__` signature and
defaults (pipeline.py:188-202), same outputs (FLitePipelineOutput(images=[PIL.Image])), same schedule, CFG
batch order (uncond first), APG, decode scaling and uint8 post-processing.

Differences by design:
  * the 30-step loop runs natively (libflite_hip.so: flite_dit_sample) and is captured in one hipGraph;
    the CFG pair runs as one batch per launch; cross-attention K/V of the (step-invariant) context are
    computed once per call;
  * the Euler accumulator, the residual stream and the modulate/gate/CFG math are fp32 (the reference
    rounds each to bf16; SURVEY §8d shows this is what lifts parity above the reference's own bf16 floor);
  * text encoding (pipeline.py:126-175) runs natively when the text encoder is the T5 v1.1 encoder of
    f_lite.text_encoder (the 4096-wide context of the 7B / 10B DiTs); any other transformers encoder is called
    the reference's way (processor -> encoder(..., output_hidden_states=True).hidden_states[-8]) on torch;
    `prompt_embeds` skips the step.
"""
from __future__ import annotations

import json
import math
from dataclasses import dataclass
from pathlib import Path
from typing import List, Optional, Union

import numpy as np
import torch

from . import _native
from .model import DiT

# The system message of the reference's caption template (pipeline.py:106): part of the text the encoder sees,
# so it is part of the interface.
_SYSTEM_PROMPT = (
    "You are a text-to-image generation model engineered to transform user-provided textual captions directly "
    "into high-quality, visually rich image tokens. Your core objective is to generate the best possible, "
    "highest-fidelity image that creatively interprets and expands upon the user's intent while maintaining "
    "strong semantic alignment with the original caption. You are designed for maximum visual quality, artistic "
    "flair, and implicit adherence to best practices in image generation (e.g., proper anatomy, clear focus, "
    "compelling composition), ensuring a stunning visual result from even concise descriptions."
)


@dataclass
class APGConfig:
    """pipeline.py:25-30"""

    enabled: bool = True
    orthogonal_threshold: float = 0.03


@dataclass
class FLitePipelineOutput:
    """pipeline.py:33-43"""

    images: Union[List["Image.Image"], np.ndarray, torch.Tensor]  # noqa: F821


def randn_tensor(shape, generator=None, device=None, dtype=None):
    """diffusers.utils.torch_utils.randn_tensor semantics (pipeline.py:236): draw on the generator's device
    (a CPU generator gives the same noise whatever the target device), then move to `device`."""
    if isinstance(generator, (list, tuple)):  # one generator per image, as diffusers allows
        if len(generator) != shape[0]:
            raise ValueError(f"{len(generator)} generators for a batch of {shape[0]}")
        return torch.cat([randn_tensor((1,) + tuple(shape[1:]), g, device, dtype) for g in generator])
    gen_dev = generator.device if generator is not None else torch.device(device or "cpu")
    return torch.randn(shape, generator=generator, device=gen_dev, dtype=dtype).to(device)


def flow_schedule(num_inference_steps: int, latent_h: int, latent_w: int, alpha: Optional[float] = None):
    """Shifted rectified-flow schedule (pipeline.py:239-257): [(t, dt)], t in python float64."""
    if alpha is None:
        alpha = 2 * math.sqrt(latent_h * latent_w / (64 * 64))
    out = []
    for i in range(num_inference_steps, 0, -1):
        t = i / num_inference_steps
        tn = (i - 1) / num_inference_steps
        t = t * alpha / (1 + (alpha - 1) * t)
        tn = tn * alpha / (1 + (alpha - 1) * tn)
        out.append((t, t - tn))
    return out


def resolve_dit_class(entry):
    """model_index.json's ["module", "class"] for dit_model -> the DiT class. The reference registers the DiT
    with diffusers' loader under "f_lite" and "f_lite.model" (generate.py:61-66); a model_v2.py folder names
    "f_lite.model_v2" (per-block adaLN, the 10B layout)."""
    module, cls = entry
    if cls != "DiT":
        raise ValueError(f"dit_model: unsupported class {module}.{cls}")
    if module in ("f_lite", "f_lite.model"):
        return DiT
    if module == "f_lite.model_v2":
        from .model_v2 import DiT as DiTv2

        return DiTv2
    raise ValueError(f"dit_model: unknown module {module!r} (expected f_lite.model or f_lite.model_v2)")


class FLitePipeline:
    model_cpu_offload_seq = "text_encoder->dit_model->vae"

    def __init__(self, dit_model: DiT, vae=None, text_encoder=None, processor=None, tokenizer=None):
        self.dit_model = dit_model
        self.vae = vae
        self.text_encoder = text_encoder
        self.processor = processor if processor is not None else tokenizer  # pt.py:158 passes tokenizer=
        self.caption_to_text = None  # optional prompt templating hook (the reference's chat template, pipeline.py:105)
        self.vae_scale_factor = 8
        self.return_index = -8
        self._progress_bar_config = {}
        self._cfg_parallel = False
        self._cfg_group = None
        self._seq_parallel = False
        self._sp_group = None
        self._sp_ring = False
        self._data_parallel = False
        self._dp_group = None

    # ---------------------------------------------------------------- loading
    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path, torch_dtype=torch.bfloat16, device="cuda", **kwargs):
        """Local diffusers-layout pipeline folder (model_index.json; dit_model/, vae/ subfolders). The
        diffusers LOADABLE_CLASSES registration of generate.py:61-66 is not needed: components are resolved
        here without diffusers. Text encoders are not loaded (prompt_embeds are required)."""
        root = Path(pretrained_model_name_or_path)
        if not (root / "model_index.json").exists():
            raise FileNotFoundError(f"{root}/model_index.json not found (Hub names cannot be resolved offline)")
        index = json.loads((root / "model_index.json").read_text())
        dit_cls = resolve_dit_class(index.get("dit_model", ["f_lite.model", "DiT"]))
        dit = dit_cls.from_pretrained(root, subfolder="dit_model", torch_dtype=torch_dtype, device=device)
        vae = None
        if "vae" in index and (root / "vae").exists():
            from .vae import AutoencoderKL

            vae = AutoencoderKL.from_pretrained(root / "vae", torch_dtype=torch_dtype, device=device)
        text_encoder, processor = None, None
        te = root / "text_encoder"
        if "text_encoder" in index and (te / "config.json").exists():
            cfg = json.loads((te / "config.json").read_text())
            if cfg.get("model_type") == "t5":
                from .text_encoder import T5Encoder

                text_encoder = T5Encoder.from_pretrained(te, torch_dtype=torch_dtype, device=device)
        for sub in ("tokenizer", "processor"):
            if sub in index and (root / sub).exists():
                from transformers import AutoTokenizer

                processor = AutoTokenizer.from_pretrained(str(root / sub), local_files_only=True)
                break
        return cls(dit, vae, text_encoder, processor)

    def save_pretrained(self, path):
        root = Path(path)
        root.mkdir(parents=True, exist_ok=True)
        index = {"_class_name": "FLitePipeline", "dit_model": [self.dit_model.module_name, "DiT"]}
        self.dit_model.save_pretrained(root / "dit_model")
        if self.text_encoder is not None and hasattr(self.text_encoder, "save_pretrained"):
            index["text_encoder"] = ["transformers", "T5EncoderModel"]
            self.text_encoder.save_pretrained(root / "text_encoder")
        if self.vae is not None:
            index["vae"] = ["diffusers", "AutoencoderKL"]
            self.vae.save_pretrained(root / "vae")
        (root / "model_index.json").write_text(json.dumps(index, indent=2))

    # ---------------------------------------------------------------- reference API surface
    def enable_vae_slicing(self):
        """pipeline.py:85-88 (the native decoder processes one image at a time already)."""
        if self.vae is not None and hasattr(self.vae, "enable_slicing"):
            self.vae.enable_slicing()

    def enable_vae_tiling(self):
        """pipeline.py:90-93: diffusers tiled decode once a latent side exceeds sample_size / 8 (e.g. the
        1344x896 default of generate.py); at <= 1024^2 the decode stays untiled, as in the reference."""
        if self.vae is not None and hasattr(self.vae, "enable_tiling"):
            self.vae.enable_tiling()

    def enable_cfg_parallel(self, group=None):
        """Single-image latency mode (no reference counterpart): the uncond and cond
        branches run on the two ranks of `group` (torch.distributed, RCCL), exchanging their outputs once per
        step. Every rank calls the pipeline with the same inputs and gets the same images."""
        import torch.distributed as dist

        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) != 2:
            raise ValueError("enable_cfg_parallel needs an initialised process group of exactly 2 ranks")
        self._cfg_group = group
        self._cfg_parallel = True

    def disable_cfg_parallel(self):
        self._cfg_parallel = False

    def enable_data_parallel(self, group=None):
        """One reference batch of images over every rank of `group` (no reference counterpart):
        image i of the batch runs on rank i mod N; with APG the batch-global sums are all-reduced per step, so
        the batch comes out as the single-GPU batched loop's. Every rank calls the pipeline with the same inputs
        and gets every image (the final latents are all-gathered; each rank decodes the whole batch)."""
        import torch.distributed as dist

        if not (dist.is_available() and dist.is_initialized()):
            raise ValueError("enable_data_parallel needs an initialised torch.distributed process group")
        self._dp_group = group
        self._data_parallel = True

    def disable_data_parallel(self):
        self._data_parallel = False

    def enable_sequence_parallel(self, group=None, ring: bool = False):
        """Single-image latency over every rank of `group` (no reference counterpart):
        each rank computes a slice of the token rows of every DiT launch, exchanging K/V rows per block
        (distributed.sequence_parallel_sample; ring=True: N - 1 neighbour shifts instead of one all-gather).
        Every rank calls the pipeline with the same inputs and gets the same images."""
        import torch.distributed as dist

        if not (dist.is_available() and dist.is_initialized()):
            raise ValueError("enable_sequence_parallel needs an initialised torch.distributed process group")
        self._sp_group = group
        self._sp_ring = bool(ring)
        self._seq_parallel = True

    def disable_sequence_parallel(self):
        self._seq_parallel = False

    def enable_model_cpu_offload(self, *a, **k):
        """generate.py:72 (no-op: weights stay resident in the 288 GB HBM)."""

    def set_progress_bar_config(self, **kwargs):
        self._progress_bar_config = kwargs

    def to(self, torch_device=None, torch_dtype=None, silence_dtype_warnings=False):
        for m in (self.dit_model, self.vae, self.text_encoder):
            if m is not None and hasattr(m, "to"):
                m.to(device=torch_device, dtype=torch_dtype)
        return self

    @property
    def _execution_device(self):
        return self.dit_model.device

    def _convert_caption_to_messages(self, caption: str) -> str:
        """pipeline.py:105-124: the system + user chat messages of a caption through the processor's chat
        template (text only, generation prompt appended)."""
        messages = [
            {"role": "system", "content": _SYSTEM_PROMPT},
            {"role": "user", "content": [{"type": "text", "text": caption}]},
        ]
        return self.processor.apply_chat_template(messages, tokenize=False, add_generation_prompt=True)

    def encode_prompt(self, prompt, negative_prompt=None, device=None, dtype=None, max_sequence_length=512,
                      return_index=-8):
        """pipeline.py:126-175: hidden_states[return_index] of the text encoder over the tokenized prompts
        (padding "longest" to a multiple of 8, truncation at max_sequence_length); zeros for a missing negative
        prompt. The native T5 encoder runs only the layers that state needs."""
        from .text_encoder import T5Encoder

        if self.text_encoder is None:
            raise ValueError("FLitePipeline has no text encoder: pass prompt_embeds / negative_prompt_embeds, or "
                             "build the pipeline with text_encoder=T5Encoder(...) and its tokenizer")
        if self.processor is None:
            raise ValueError("the text encoder needs a tokenizer / processor (FLitePipeline(..., processor=...))")
        if isinstance(prompt, str):
            prompt = [prompt]
        enc = self.text_encoder
        device = device or enc.device
        if self.caption_to_text is not None:
            texts = [self.caption_to_text(p) for p in prompt]
        elif getattr(self.processor, "chat_template", None):  # Qwen2.5-VL & co: the reference's template
            texts = [self._convert_caption_to_messages(p) for p in prompt]
        else:  # T5 tokenizers have no chat template: raw captions (pt.py's T5 pipeline)
            texts = list(prompt)
        tok = self.processor(text=texts, padding="longest", pad_to_multiple_of=8, max_length=max_sequence_length,
                             truncation=True, return_tensors="pt")
        if isinstance(enc, T5Encoder):
            emb = enc.encode(tok["input_ids"], tok.get("attention_mask"), return_index=return_index)
        else:  # a transformers encoder, called as the reference calls it (pipeline.py:148-154)
            tok = {k: v.to(device) for k, v in tok.items()}
            emb = enc(**tok, use_cache=False, return_dict=True, output_hidden_states=True).hidden_states[return_index]
        dtype = dtype or next(enc.parameters()).dtype
        emb = emb.to(device=device, dtype=dtype)
        if negative_prompt is None:
            neg = torch.zeros_like(emb)
        else:
            neg = self.encode_prompt(negative_prompt, device=device, dtype=dtype,
                                     max_sequence_length=max_sequence_length, return_index=return_index)[0]
        return emb, neg

    # ---------------------------------------------------------------- sampling
    @torch.no_grad()
    def __call__(self, prompt: Union[str, List[str], None] = None, height: Optional[int] = 1024,
                 width: Optional[int] = 1024, num_inference_steps: int = 30, guidance_scale: float = 6.0,
                 negative_prompt: Optional[Union[str, List[str]]] = None, num_images_per_prompt: int = 1,
                 generator: Optional[torch.Generator] = None, dtype: Optional[torch.dtype] = None,
                 alpha: Optional[float] = None, apg_config: Optional[APGConfig] = None,
                 prompt_embeds: Optional[torch.Tensor] = None,
                 negative_prompt_embeds: Optional[torch.Tensor] = None, latents: Optional[torch.Tensor] = None,
                 output_type: str = "pil", use_graph: bool = True, **kwargs):
        height = 1024 if height is None else height
        width = 1024 if width is None else width
        dit = self.dit_model
        dtype = dtype or dit.dtype
        apg_config = apg_config or APGConfig(enabled=False)
        device = self._execution_device
        if height % (self.vae_scale_factor * dit.config.patch_size) or \
                width % (self.vae_scale_factor * dit.config.patch_size):
            raise ValueError("height and width must be multiples of 16")

        # 2. prompt embeddings (pipeline.py:215-226)
        if prompt_embeds is None:
            prompt_embeds, neg = self.encode_prompt(prompt, negative_prompt, device=device, dtype=dtype)
            if negative_prompt_embeds is None:
                negative_prompt_embeds = neg
        prompt_embeds = prompt_embeds.to(device=device, dtype=dtype)
        if negative_prompt_embeds is None:
            negative_prompt_embeds = torch.zeros_like(prompt_embeds)  # pipeline.py:160-161
        negative_prompt_embeds = negative_prompt_embeds.to(device=device, dtype=dtype)
        prompt_embeds = prompt_embeds.repeat_interleave(num_images_per_prompt, dim=0)
        negative_prompt_embeds = negative_prompt_embeds.repeat_interleave(num_images_per_prompt, dim=0)
        batch_size = prompt_embeds.shape[0]

        # 3. initial latents (pipeline.py:228-237): randn in the model dtype, same generator semantics
        lh, lw = height // self.vae_scale_factor, width // self.vae_scale_factor
        if latents is None:
            latents = randn_tensor((batch_size, 16, lh, lw), generator=generator, device=device, dtype=dtype)
        latents = latents.to(device=device, dtype=dtype)
        acc = latents.float().contiguous()  # fp32 Euler accumulator (reference: model dtype)

        # 4-6. schedule + native denoise loop (pipeline.py:239-297)
        sched = flow_schedule(num_inference_steps, lh, lw, alpha)
        t_list = [t for t, _ in sched]
        dt_list = [dt for _, dt in sched]
        do_cfg = guidance_scale >= 1.0
        if apg_config.enabled and not do_cfg:
            apg_config = APGConfig(enabled=False)
        eng = dit.engine()
        L = prompt_embeds.shape[1]
        if negative_prompt_embeds.shape[1] != L:
            raise ValueError("prompt and negative prompt embeddings must have the same length")
        if self._seq_parallel:
            from .distributed import sequence_parallel_sample

            acc = sequence_parallel_sample(dit, latents, prompt_embeds, negative_prompt_embeds, num_inference_steps,
                                           guidance_scale, alpha, group=self._sp_group,
                                           ring=self._sp_ring, apg=apg_config)
        elif self._cfg_parallel and do_cfg:
            from .distributed import cfg_parallel_sample

            acc = cfg_parallel_sample(dit, latents, prompt_embeds, negative_prompt_embeds, num_inference_steps,
                                      guidance_scale, alpha, group=self._cfg_group, apg=apg_config)
        elif self._data_parallel and do_cfg:
            from .distributed import data_parallel_sample

            acc = data_parallel_sample(dit, latents, prompt_embeds, negative_prompt_embeds, num_inference_steps,
                                       guidance_scale, alpha, group=self._dp_group, apg=apg_config)
        else:
            if do_cfg:
                ctx = torch.cat([negative_prompt_embeds, prompt_embeds])  # uncond first (pipeline.py:266)
            else:
                ctx = prompt_embeds
            nseq = ctx.shape[0]
            eng.prepare(nseq, lh, lw, nseq * L, num_inference_steps)
            eng.set_context(ctx.reshape(nseq * L, -1).contiguous(), [i * L for i in range(nseq + 1)])
            eng.sample(acc, batch_size, t_list, dt_list, guidance_scale, do_cfg, apg_config.enabled,
                       apg_config.orthogonal_threshold, use_graph)

        if output_type == "latent":
            return FLitePipelineOutput(images=acc.to(dtype))

        # 7. decode (pipeline.py:299-307)
        if self.vae is None:
            raise ValueError("no VAE: use output_type='latent'")
        scaling = getattr(self.vae.config, "scaling_factor", 0.18215)
        shift = getattr(self.vae.config, "shift_factor", 0.0)
        images_u8 = self.vae.decode_to_uint8(acc, scaling, shift)  # [B, H, W, 3] uint8 on device
        if output_type == "uint8":
            return FLitePipelineOutput(images=images_u8)
        from PIL import Image

        arr = images_u8.cpu().numpy()
        return FLitePipelineOutput(images=[Image.fromarray(a) for a in arr])
