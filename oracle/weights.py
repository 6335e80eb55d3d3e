"""TEST INFRASTRUCTURE ONLY. Deterministic parameter generator + parameter inventory of the reference DiT.

The generator is a counter-based hash (splitmix64) so that the CPU oracle (numpy, here) and the GPU
(f-lite_amd/csrc/init.hip, flite_init_param) produce bit-identical parameters without shipping weights:

    base    = splitmix64(seed ^ fnv1a64(name))
    bits(i) = splitmix64(base + i)                      (i = flat element index, row-major)
    s       = (bits >> 40) - 2**23                      (24-bit signed, in [-2**23, 2**23))
    value   = float32(2*s + 1) * float32(std * sqrt(3) / 2**24)   -> uniform, mean 0, std `std`

Norm weights are 1.0 (LigerRMSNorm / RMSNorm init, model.py:97,238); every other tensor (matrices,
biases, register tokens) uses std 0.02 (the reference's own zero-init of the adaLN /
final layers would make the DiT output exactly 0, so every parameter is re-initialised).
"""
from __future__ import annotations

import math

import numpy as np
import torch

M64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15


def fnv1a64(name: str) -> int:
    h = 0xCBF29CE484222325
    for b in name.encode():
        h ^= b
        h = (h * 0x100000001B3) & M64
    return h


def splitmix64_scalar(x: int) -> int:
    z = (x + GOLDEN) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def _splitmix64_np(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def hash_uniform(name: str, numel: int, std: float, seed: int = 0, chunk: int = 1 << 24) -> np.ndarray:
    """fp32 values of the generator for `numel` elements of parameter `name`."""
    base = splitmix64_scalar((seed ^ fnv1a64(name)) & M64)
    scale = np.float32(std * math.sqrt(3.0) / float(1 << 24))
    out = np.empty(numel, dtype=np.float32)
    for s0 in range(0, numel, chunk):
        n = min(chunk, numel - s0)
        idx = np.arange(s0, s0 + n, dtype=np.uint64)
        with np.errstate(over="ignore"):
            bits = _splitmix64_np(idx + np.uint64(base))
        s = (bits >> np.uint64(40)).astype(np.int64) - (1 << 23)
        out[s0 : s0 + n] = (2 * s + 1).astype(np.float32) * scale
    return out


def param_shapes(cfg: dict) -> "dict[str, tuple]":
    """State-dict keys and shapes of DiT(**cfg) (model.py:417-479; model_v2.py per-block adaLN).

    cfg keys: in_channels, patch_size, hidden_size, depth, num_heads, mlp_ratio, cross_attn_input_size,
    train_bias_and_rms, per_block_adaln (v2 layout).
    """
    D = cfg["hidden_size"]
    C = cfg["in_channels"]
    p = cfg["patch_size"]
    F = int(D * cfg.get("mlp_ratio", 4.0))
    Cc = cfg["cross_attn_input_size"]
    bias = cfg.get("train_bias_and_rms", True)
    v2 = cfg.get("per_block_adaln", False)
    s = {}
    s["context_proj.weight"] = (D, Cc)
    s["context_proj.bias"] = (D,)
    s["context_norm.weight"] = (D,)
    s["patch_embed.patch_proj.weight"] = (D, C, p, p)
    s["patch_embed.patch_proj.bias"] = (D,)
    s["register_tokens"] = (1, 16, D)
    if not cfg.get("use_rope", True):
        s["positional_embedding"] = (1, 2048, D)  # model.py:444
    s["time_embed.0.weight"] = (4 * D, D)
    s["time_embed.0.bias"] = (4 * D,)
    s["time_embed.2.weight"] = (D, 4 * D)
    s["time_embed.2.bias"] = (D,)
    if not v2:
        s["adaLN_modulation.1.weight"] = (9 * D, D)
        s["adaLN_modulation.1.bias"] = (9 * D,)
    for i in range(cfg["depth"]):
        pre = f"blocks.{i}."
        cross = True if v2 else (i % 4 == 0 or i < 8)
        s[pre + "norm1.weight"] = (D,)
        s[pre + "self_attn.qkv.weight"] = (3 * D, D)
        if bias:
            s[pre + "self_attn.qkv.bias"] = (3 * D,)
        s[pre + "self_attn.proj.weight"] = (D, D)
        if cross:
            s[pre + "norm2.weight"] = (D,)
            s[pre + "cross_attn.q.weight"] = (D, D)
            if bias:
                s[pre + "cross_attn.q.bias"] = (D,)
            s[pre + "cross_attn.context_kv.weight"] = (2 * D, D)
            if bias:
                s[pre + "cross_attn.context_kv.bias"] = (2 * D,)
            s[pre + "cross_attn.proj.weight"] = (D, D)
        s[pre + "norm3.weight"] = (D,)
        s[pre + "mlp.gate_proj.weight"] = (F, D)
        s[pre + "mlp.up_proj.weight"] = (F, D)
        s[pre + "mlp.down_proj.weight"] = (D, F)
        if v2:
            s[pre + "adaLN_modulation.1.weight"] = (9 * D, D)
            s[pre + "adaLN_modulation.1.bias"] = (9 * D,)
    s["final_modulation.1.weight"] = (2 * D, D)
    s["final_modulation.1.bias"] = (2 * D,)
    if bias:
        s["final_norm.weight"] = (D,)
    s["final_proj.weight"] = (p * p * C, D)
    s["final_proj.bias"] = (p * p * C,)
    return s


def is_norm_weight(name: str) -> bool:
    return name.endswith("norm1.weight") or name.endswith("norm2.weight") or name.endswith("norm3.weight") or \
        name in ("context_norm.weight", "final_norm.weight")


def make_param(name: str, shape, seed: int = 0, std: float = 0.02) -> torch.Tensor:
    """fp32 tensor holding the bf16-representable generator values (the bf16 model's exact weights)."""
    n = int(np.prod(shape))
    if is_norm_weight(name):
        return torch.ones(shape, dtype=torch.float32)
    v = torch.from_numpy(hash_uniform(name, n, std, seed)).reshape(shape)
    return v.to(torch.bfloat16).to(torch.float32)


def make_state_dict(cfg: dict, seed: int = 0, std: float = 0.02, names=None) -> "dict[str, torch.Tensor]":
    shapes = param_shapes(cfg)
    keys = names if names is not None else shapes.keys()
    return {k: make_param(k, shapes[k], seed, std) for k in keys}
