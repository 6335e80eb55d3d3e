"""T5 v1.1 text encoder (the prompt-embedding step), MI355X-native.

The reference encodes each prompt once per call (f_lite/pipeline.py:126-175: `hidden_states[return_index]`,
return_index = -8, of the text encoder run with `output_hidden_states=True`); the F-Lite 7B / 10B DiTs take a
4096-wide context (cross_attn_input_size = 4096, train.py:685-698), T5-XXL's d_model, which pt.py:150-155 loads
as FLUX's `text_encoder_2` (transformers T5EncoderModel + T5TokenizerFast).

`T5Encoder` mirrors transformers' T5EncoderModel for that use: the same module tree and state-dict keys
(`shared`, `encoder.block.{i}.layer.{0,1}...`, `encoder.final_layer_norm`), `forward(input_ids,
attention_mask, output_hidden_states=True)` returning `.last_hidden_state` / `.hidden_states` (embeddings, the
output of every layer, then the final-normed output: 25 entries for 24 layers), and `from_pretrained` for a
local folder (config.json + model*.safetensors). The layer math is transformers' T5 (the reference's
dependency): RMSNorm without mean or bias, self-attention without 1/sqrt(d) and with a bucketed relative
position bias computed from layer 0's table and shared by every layer, a gated-GELU (tanh) feed-forward,
residual adds. It runs on the native kernels: the DiT GEMM (GEGLU and residual epilogues), the RMSNorm kernel,
flite_t5_attention and flite_embed_rows_f32 (csrc/t5.hip). The residual stream is fp32 (transformers' bf16
model keeps it in bf16); hidden states are returned in bf16. There is no CPU path.
"""
from __future__ import annotations

import json
import math
from pathlib import Path
from types import SimpleNamespace
from typing import Optional

import torch
from torch import nn

from . import _native

# transformers T5Config field names; "t5-xxl" = google/t5-v1_1-xxl (FLUX text_encoder_2)
T5_PRESETS = {
    "t5-xxl": dict(vocab_size=32128, d_model=4096, d_kv=64, d_ff=10240, num_layers=24, num_heads=64,
                   relative_attention_num_buckets=32, relative_attention_max_distance=128, layer_norm_epsilon=1e-6),
    "tiny": dict(vocab_size=1000, d_model=256, d_kv=64, d_ff=512, num_layers=4, num_heads=4,
                 relative_attention_num_buckets=32, relative_attention_max_distance=128, layer_norm_epsilon=1e-6),
}


def relative_position_bucket(relative_position: torch.Tensor, num_buckets=32, max_distance=128) -> torch.Tensor:
    """Bidirectional bucket of (key - query) (transformers T5Attention._relative_position_bucket, the Mesh
    TensorFlow scheme): half the buckets per sign; |rel| < num_buckets/4 exact, then log-spaced up to
    max_distance, clamped. Evaluated with the same float32 torch ops on the CPU so boundary cases round alike."""
    num_buckets //= 2
    buckets = (relative_position > 0).to(torch.long) * num_buckets
    rel = torch.abs(relative_position)
    max_exact = num_buckets // 2
    is_small = rel < max_exact
    large = max_exact + (torch.log(rel.float() / max_exact) / math.log(max_distance / max_exact)
                         * (num_buckets - max_exact)).to(torch.long)
    large = torch.min(large, torch.full_like(large, num_buckets - 1))
    return buckets + torch.where(is_small, rel, large)


class T5LayerNorm(nn.Module):
    def __init__(self, d, eps=1e-6):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d))
        self.variance_epsilon = eps


class T5Attention(nn.Module):
    def __init__(self, cfg, has_relative_attention_bias=False):
        super().__init__()
        inner = cfg.num_heads * cfg.d_kv
        self.q = nn.Linear(cfg.d_model, inner, bias=False)
        self.k = nn.Linear(cfg.d_model, inner, bias=False)
        self.v = nn.Linear(cfg.d_model, inner, bias=False)
        self.o = nn.Linear(inner, cfg.d_model, bias=False)
        if has_relative_attention_bias:
            self.relative_attention_bias = nn.Embedding(cfg.relative_attention_num_buckets, cfg.num_heads)


class T5LayerSelfAttention(nn.Module):
    def __init__(self, cfg, has_relative_attention_bias=False):
        super().__init__()
        self.SelfAttention = T5Attention(cfg, has_relative_attention_bias)
        self.layer_norm = T5LayerNorm(cfg.d_model, cfg.layer_norm_epsilon)


class T5DenseGatedActDense(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.wi_0 = nn.Linear(cfg.d_model, cfg.d_ff, bias=False)
        self.wi_1 = nn.Linear(cfg.d_model, cfg.d_ff, bias=False)
        self.wo = nn.Linear(cfg.d_ff, cfg.d_model, bias=False)


class T5LayerFF(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.DenseReluDense = T5DenseGatedActDense(cfg)
        self.layer_norm = T5LayerNorm(cfg.d_model, cfg.layer_norm_epsilon)


class T5Block(nn.Module):
    def __init__(self, cfg, has_relative_attention_bias=False):
        super().__init__()
        self.layer = nn.ModuleList([T5LayerSelfAttention(cfg, has_relative_attention_bias), T5LayerFF(cfg)])


class T5Stack(nn.Module):
    def __init__(self, cfg, embed_tokens):
        super().__init__()
        self.embed_tokens = embed_tokens
        self.block = nn.ModuleList([T5Block(cfg, has_relative_attention_bias=(i == 0)) for i in range(cfg.num_layers)])
        self.final_layer_norm = T5LayerNorm(cfg.d_model, cfg.layer_norm_epsilon)


class T5Encoder(nn.Module):
    """transformers T5EncoderModel (encoder only, gated-GELU v1.1 layout) on the native path."""

    def __init__(self, **cfg):
        super().__init__()
        base = dict(T5_PRESETS["t5-xxl"])
        base.update({k: v for k, v in cfg.items() if k in base})
        ff = cfg.get("feed_forward_proj", "gated-gelu")
        if ff != "gated-gelu":
            raise NotImplementedError(f"feed_forward_proj={ff!r}: only the T5 v1.1 gated-gelu layout is supported")
        if base["d_kv"] != 64:
            raise NotImplementedError("T5 heads of 64 only (flite_t5_attention)")
        self.config = SimpleNamespace(**base, feed_forward_proj=ff)
        self.shared = nn.Embedding(base["vocab_size"], base["d_model"])
        self.encoder = T5Stack(self.config, self.shared)
        self._bucket_cache = {}

    # ------------------------------------------------------------------ construction / IO
    @classmethod
    def empty(cls, device="cuda", dtype=torch.bfloat16, **cfg):
        with torch.device("meta"):
            m = cls(**cfg)
        m = m.to_empty(device=device).to(dtype)
        m.encoder.embed_tokens = m.shared  # keep the tie after to_empty
        return m

    @classmethod
    def random(cls, seed=0, device="cuda", dtype=torch.bfloat16, **cfg):
        """Seeded synthetic weights on the device (the DiT's hash generator, uniform), with the per-tensor scales
        of transformers' T5 initialisation (T5PreTrainedModel._init_weights, factor 1) so activations stay O(1)
        through the stack: embedding 1, q (d_model d_kv)^-1/2, k / v / wi d_model^-1/2, o (H d_kv)^-1/2,
        wo d_ff^-1/2, relative bias d_model^-1/2, norm weights 1."""
        m = cls.empty(device=device, dtype=dtype, **cfg)
        c = m.config
        std_of = {"q": (c.d_model * c.d_kv) ** -0.5, "k": c.d_model ** -0.5, "v": c.d_model ** -0.5,
                  "o": (c.num_heads * c.d_kv) ** -0.5, "wi_0": c.d_model ** -0.5, "wi_1": c.d_model ** -0.5,
                  "wo": c.d_ff ** -0.5, "relative_attention_bias": c.d_model ** -0.5, "shared": 1.0}
        with torch.no_grad():
            for name, p in m.named_parameters():
                key = name.split(".")[-2]
                _native.init_param_(p.data, "t5." + name, seed=seed, std=std_of.get(key, 0.02),
                                    ones=name.endswith("layer_norm.weight"))
        torch.cuda.synchronize()
        return m

    @classmethod
    def from_pretrained(cls, path, subfolder=None, torch_dtype=torch.bfloat16, device="cuda", **kwargs):
        """Local transformers folder: config.json + model*.safetensors (e.g. FLUX's text_encoder_2)."""
        from safetensors.torch import load_file

        p = Path(path) / subfolder if subfolder else Path(path)
        if not (p / "config.json").exists():
            raise FileNotFoundError(f"{p}/config.json not found (only local folders are supported)")
        cfg = json.loads((p / "config.json").read_text())
        files = sorted(p.glob("model*.safetensors"))
        if not files:
            raise FileNotFoundError(f"no model*.safetensors in {p}")
        sd = {}
        for f in files:
            sd.update(load_file(str(f)))
        # config.json also holds transformers' own keys ("dtype"/"torch_dtype", "architectures", ...): keep only
        # the architecture fields (the loader's torch_dtype / device win)
        arch = {k: v for k, v in cfg.items() if k in T5_PRESETS["t5-xxl"] or k == "feed_forward_proj"}
        m = cls.empty(device=device, dtype=torch_dtype, **arch)
        if "shared.weight" not in sd and "encoder.embed_tokens.weight" in sd:
            sd["shared.weight"] = sd["encoder.embed_tokens.weight"]
        sd.setdefault("encoder.embed_tokens.weight", sd["shared.weight"])
        m.load_state_dict(sd, strict=True)
        return m

    def save_pretrained(self, path):
        """config.json (transformers T5Config keys) + model.safetensors (shared embedding stored once)."""
        from safetensors.torch import save_file

        p = Path(path)
        p.mkdir(parents=True, exist_ok=True)
        cfg = dict(vars(self.config), model_type="t5", architectures=["T5EncoderModel"], is_gated_act=True,
                   dense_act_fn="gelu_new")
        (p / "config.json").write_text(json.dumps(cfg, indent=2))
        sd = {k: v.detach().contiguous().cpu() for k, v in self.state_dict().items()
              if k != "encoder.embed_tokens.weight"}
        save_file(sd, str(p / "model.safetensors"))

    @property
    def device(self):
        return self.shared.weight.device

    @property
    def dtype(self):
        return self.shared.weight.dtype

    def _bucket_table(self, L):
        t = self._bucket_cache.get(L)
        if t is None:
            rel = torch.arange(-(L - 1), L, dtype=torch.long)  # key - query
            b = relative_position_bucket(rel, self.config.relative_attention_num_buckets,
                                         self.config.relative_attention_max_distance)
            t = b.to(torch.int32).to(self.device)
            self._bucket_cache[L] = t
        return t

    # ------------------------------------------------------------------ forward
    @torch.no_grad()
    def forward(self, input_ids, attention_mask=None, output_hidden_states=False, return_dict=True,
                num_layers: Optional[int] = None, **kwargs):
        """T5EncoderModel.forward for prompt encoding: hidden_states = (embeddings, the output after 1, 2, ...,
        num_layers - 1 layers, the final-normed output), num_layers + 1 entries as in transformers' T5Stack.
        `num_layers` (not a transformers argument) stops after that many layers; last_hidden_state is then that
        layer's raw output."""
        cfg = self.config
        dev = self.device
        if not self.shared.weight.is_cuda:
            raise _native.FliteError("T5Encoder parameters are on the CPU: the native path runs only on a ROCm "
                                     "device; there is no CPU fallback")
        if self.dtype != torch.bfloat16:
            raise _native.FliteError("T5Encoder computes with bf16 parameters; call .to(torch.bfloat16)")
        ids = input_ids.to(device=dev, dtype=torch.int32).contiguous()
        B, L = ids.shape
        D, H, dk = cfg.d_model, cfg.num_heads, cfg.d_kv
        inner = H * dk
        n_run = cfg.num_layers if num_layers is None else int(num_layers)
        if not 0 <= n_run <= cfg.num_layers:
            raise ValueError(f"num_layers must be in [0, {cfg.num_layers}]")
        lib = _native.load()
        stream = _native.stream_ptr(dev)
        M = B * L
        x = torch.empty(M, D, device=dev, dtype=torch.float32)
        _native.check(lib.flite_embed_rows_f32(stream, self.shared.weight.data_ptr(), ids.data_ptr(), x.data_ptr(), M,
                                               D, cfg.vocab_size), "flite_embed_rows_f32")
        mask = None
        if attention_mask is not None:
            am = attention_mask.to(device=dev).reshape(B, L)
            mask = torch.zeros(B, L, device=dev, dtype=torch.float32).masked_fill_(am == 0, float("-inf"))
        bucket = self._bucket_table(L)
        rel_w = self.encoder.block[0].layer[0].SelfAttention.relative_attention_bias.weight
        hidden = [x.to(torch.bfloat16).view(B, L, D)] if output_hidden_states else None
        qkv = torch.empty(M, 3 * inner, device=dev, dtype=torch.bfloat16)
        att = torch.empty(M, inner, device=dev, dtype=torch.bfloat16)
        for i in range(n_run):
            sa, ff = self.encoder.block[i].layer
            a = sa.SelfAttention
            h = _native.rmsnorm_modulate(x, w=sa.layer_norm.weight, eps=cfg.layer_norm_epsilon)
            for j, lin in enumerate((a.q, a.k, a.v)):
                _native.gemm(h, lin.weight, out=qkv[:, j * inner:(j + 1) * inner])
            _native.check(lib.flite_t5_attention(stream, qkv.data_ptr(), 3 * inner, qkv[:, inner:].data_ptr(), 3 * inner,
                                                 qkv[:, 2 * inner:].data_ptr(), 3 * inner, att.data_ptr(), inner,
                                                 bucket.data_ptr(), rel_w.data_ptr(), _native._ptr(mask), B, L, H),
                          "flite_t5_attention")
            _native.gemm(att, a.o.weight, out=x, epilogue=_native.EPI_RESID_F32)
            h = _native.rmsnorm_modulate(x, w=ff.layer_norm.weight, eps=cfg.layer_norm_epsilon)
            d = ff.DenseReluDense
            f = _native.gemm(h, d.wi_0.weight, w2=d.wi_1.weight, epilogue=_native.EPI_GEGLU_BF16)
            _native.gemm(f, d.wo.weight, out=x, epilogue=_native.EPI_RESID_F32)
            if output_hidden_states and i + 1 < cfg.num_layers:  # the last layer's raw output is not a state
                hidden.append(x.to(torch.bfloat16).view(B, L, D))
        if n_run == cfg.num_layers:
            last = _native.rmsnorm_modulate(x, w=self.encoder.final_layer_norm.weight,
                                            eps=cfg.layer_norm_epsilon).view(B, L, D)
        else:
            last = x.to(torch.bfloat16).view(B, L, D)
        if output_hidden_states:
            if n_run == cfg.num_layers:
                hidden.append(last)
            hidden = tuple(hidden)
        out = SimpleNamespace(last_hidden_state=last, hidden_states=hidden)
        return out if return_dict else (last,) + ((hidden,) if output_hidden_states else ())

    def encode(self, input_ids, attention_mask=None, return_index: int = -8):
        """hidden_states[return_index] of a full forward, running only the layers it needs (the reference's
        encode_prompt contract, pipeline.py:153-154)."""
        n_states = self.config.num_layers + 1
        if not -n_states <= return_index < n_states:
            raise IndexError(f"return_index {return_index} out of range for {n_states} hidden states")
        idx = return_index % n_states  # = the number of layers before that state
        return self.forward(input_ids, attention_mask, num_layers=idx).last_hidden_state


class SyntheticTokenizer:
    """Offline stand-in for T5TokenizerFast when no tokenizer files are available: UTF-8 bytes -> ids
    (byte + 3, ByT5's convention), EOS id 1 appended, pad id 0. The call signature and the returned
    input_ids / attention_mask follow the transformers tokenizer call encode_prompt makes (pipeline.py:139-146).
    Embeddings from it are not those of a real T5 vocabulary; it exists so that prompt strings can flow through
    the native encoder end to end."""

    pad_token_id = 0
    eos_token_id = 1

    def __init__(self, vocab_size=32128):
        self.vocab_size = vocab_size

    def __call__(self, text=None, padding="longest", pad_to_multiple_of=None, max_length=512, truncation=True,
                 return_tensors="pt", **kwargs):
        texts = [text] if isinstance(text, str) else list(text)
        seqs = []
        for t in texts:
            ids = [min(b + 3, self.vocab_size - 1) for b in t.encode("utf-8")]
            if truncation and max_length is not None:
                ids = ids[: max_length - 1]
            seqs.append(ids + [self.eos_token_id])
        L = max(len(x) for x in seqs)
        if padding == "max_length" and max_length is not None:
            L = max_length
        if pad_to_multiple_of:
            L = -(-L // pad_to_multiple_of) * pad_to_multiple_of
            if max_length is not None:
                L = min(L, max(max_length, max(len(x) for x in seqs)))
        ids = torch.zeros(len(seqs), L, dtype=torch.long)
        mask = torch.zeros(len(seqs), L, dtype=torch.long)
        for i, x in enumerate(seqs):
            ids[i, : len(x)] = torch.tensor(x)
            mask[i, : len(x)] = 1
        return {"input_ids": ids, "attention_mask": mask}
