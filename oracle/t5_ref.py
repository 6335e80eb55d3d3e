"""TEST INFRASTRUCTURE ONLY. CPU restatement of the T5 v1.1 encoder the reference's encode_prompt runs.

The reference takes prompt embeddings from `text_encoder(..., output_hidden_states=True).hidden_states[-8]`
(f_lite/pipeline.py:148-154) with a transformers T5EncoderModel as FLUX's text_encoder_2 (f_lite/pt.py:150-155;
the 4096-wide context of cross_attn_input_size = 4096). The encoder is a third-party dependency (transformers,
5.x in this image); this file restates its published algorithm (the T5 v1.1 "gated-gelu" encoder stack):
  - embeddings: shared[ids] (no scaling);
  - per layer: h = RMSNorm(x) (no mean, no bias, weight); q, k, v = h Wq, h Wk, h Wv (heads of d_kv);
    scores = q k^T + bias[h][bucket(key - query)] + mask (NO 1/sqrt(d)); the bucket table is layer 0's
    relative_attention_bias and is shared by every layer; x += softmax(scores) v Wo;
    h = RMSNorm(x); x += (gelu_tanh(h Wi0) * (h Wi1)) Wo;
  - hidden_states = (embeddings, output after 1 .. n-1 layers, final RMSNorm(output after n layers)).
The restatement is pinned against transformers' own T5EncoderModel on the same weights
(tests/test_text_encoder_cpu.py), and is what the GPU tests check the native encoder against.
"""
from __future__ import annotations

import math

import torch


def relative_position_bucket(rel: torch.Tensor, num_buckets=32, max_distance=128) -> torch.Tensor:
    """Bidirectional T5 bucketing of (key - query)."""
    half = num_buckets // 2
    out = (rel > 0).long() * half
    a = rel.abs()
    max_exact = half // 2
    large = max_exact + (torch.log(a.float() / max_exact) / math.log(max_distance / max_exact)
                         * (half - max_exact)).long()
    large = large.clamp(max=half - 1)
    return out + torch.where(a < max_exact, a, large)


def rms_norm(x, w, eps):
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w


def gelu_tanh(x):
    return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * x.pow(3))))


def t5_encoder_hidden_states(sd: dict, cfg: dict, input_ids: torch.Tensor, attention_mask=None, num_layers=None):
    """fp32 hidden states (tuple, transformers T5Stack order) of a T5 v1.1 encoder state dict `sd`
    (T5EncoderModel keys). cfg: d_model, d_kv, num_heads, num_layers, relative_attention_num_buckets,
    relative_attention_max_distance, layer_norm_epsilon. num_layers < cfg num_layers stops early (the last
    entry is then that layer's raw output)."""
    f = {k: v.float() for k, v in sd.items()}
    B, L = input_ids.shape
    H, dk, eps = cfg["num_heads"], cfg["d_kv"], cfg["layer_norm_epsilon"]
    n_all = cfg["num_layers"]
    n = n_all if num_layers is None else num_layers
    x = f["shared.weight"][input_ids]
    pos = torch.arange(L)
    bucket = relative_position_bucket(pos[None, :] - pos[:, None], cfg["relative_attention_num_buckets"],
                                      cfg["relative_attention_max_distance"])
    bias = f["encoder.block.0.layer.0.SelfAttention.relative_attention_bias.weight"][bucket].permute(2, 0, 1)
    if attention_mask is not None:
        bias = bias[None] + (1.0 - attention_mask[:, None, None, :].float()) * torch.finfo(torch.float32).min
    else:
        bias = bias[None]
    states = [x]
    for i in range(n):
        p = f"encoder.block.{i}.layer."
        h = rms_norm(x, f[p + "0.layer_norm.weight"], eps)
        q, k, v = (h @ f[p + f"0.SelfAttention.{c}.weight"].t() for c in "qkv")
        q, k, v = (t.view(B, L, H, dk).transpose(1, 2) for t in (q, k, v))
        s = q @ k.transpose(-1, -2) + bias
        a = torch.softmax(s, dim=-1) @ v
        x = x + a.transpose(1, 2).reshape(B, L, H * dk) @ f[p + "0.SelfAttention.o.weight"].t()
        h = rms_norm(x, f[p + "1.layer_norm.weight"], eps)
        g = gelu_tanh(h @ f[p + "1.DenseReluDense.wi_0.weight"].t()) * (h @ f[p + "1.DenseReluDense.wi_1.weight"].t())
        x = x + g @ f[p + "1.DenseReluDense.wo.weight"].t()
        if i + 1 < n_all:
            states.append(x)
    if n == n_all:
        states.append(rms_norm(x, f["encoder.final_layer_norm.weight"], eps))
    return tuple(states)
