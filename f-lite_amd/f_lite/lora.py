"""LoRA adapters for inference, merged into the DiT's weights (the reference's peft path).

The reference attaches peft LoRA adapters at load time and keeps them unmerged:
  * `load_f_lite_pt(..., lora_path, lora_rank, lora_target_modules)` (/root/reference/f_lite/pt.py:107-135):
    LoraConfig(r=lora_rank, lora_alpha=lora_rank, target_modules=[...], bias="none"), `add_adapter`, then
    `set_peft_model_state_dict` of the torch.load-ed file. `lora_scale` is only logged there (pt.py:130): the
    adapter's scaling is lora_alpha / r = 1.
  * `DiT.load_lora_weights(dir)` / `save_lora_weights(dir)` (/root/reference/f_lite/model.py:487-495): the peft
    state dict in `<dir>/lora_weights.pt`.
A peft-wrapped Linear computes base(x) + lora_B(lora_A(x)) * scaling. Here the adapter is folded into the base
weight once, W <- W + scaling * B @ A (fp32 sum, one rounding to the weight's dtype), so the native engine runs
the same GEMMs as without LoRA. The in-place update bumps the parameters' versions, so the engine rebinds and
re-derives every copy (MXFP8 weights, the cross-attention K/V cache) on its next call (DiT.engine).

State-dict keys (peft's get_peft_model_state_dict, adapter name removed): "<module>.lora_A.weight" [r, in] and
"<module>.lora_B.weight" [out, r]; keys that still carry the adapter name ("<module>.lora_A.<name>.weight") are
accepted too. A target entry t matches a module named t or ending in "." + t, as peft matches strings.
"""
from __future__ import annotations

import re
from typing import Dict, Iterable, Optional, Tuple

import torch

_KEY = re.compile(r"^(?P<mod>.+)\.lora_(?P<ab>[AB])(?:\.[^.]+)?\.weight$")


def lora_pairs(state_dict: Dict[str, torch.Tensor]) -> Dict[str, Tuple[torch.Tensor, torch.Tensor]]:
    """{module name: (A [r, in], B [out, r])} from a peft LoRA state dict. Raises on a half pair or on keys that
    are not LoRA A/B weights (e.g. lora_magnitude_vector, bias="all" tensors: configurations pt.py never builds)."""
    a, b = {}, {}
    for k, v in state_dict.items():
        k = k.replace("base_model.model.", "", 1) if k.startswith("base_model.model.") else k
        m = _KEY.match(k)
        if m is None:
            raise KeyError(f"not a LoRA A/B weight: {k!r}")
        (a if m.group("ab") == "A" else b)[m.group("mod")] = v
    if set(a) != set(b):
        raise KeyError(f"LoRA A/B weights do not pair up: {sorted(set(a) ^ set(b))[:4]}")
    return {mod: (a[mod], b[mod]) for mod in a}


def _targeted(name: str, targets: Optional[Iterable[str]]) -> bool:
    if targets is None:
        return True
    return any(name == t or name.endswith("." + t) for t in targets)


@torch.no_grad()
def merge_lora_(model: torch.nn.Module, state_dict: Dict[str, torch.Tensor], scaling: float = 1.0,
                target_modules: Optional[Iterable[str]] = None, rank: Optional[int] = None) -> int:
    """Fold every adapter of `state_dict` into `model` in place: W <- W + scaling * B @ A. Returns the number of
    merged modules. Every adapter must name an nn.Linear of the model that `target_modules` selects, with
    matching shapes (and rank `rank` when given) -- peft's set_peft_model_state_dict would not load it either."""
    targets = None if target_modules is None else [t.strip() for t in target_modules if t.strip()]
    modules = dict(model.named_modules())
    pairs = lora_pairs(state_dict)
    for mod, (A, B) in pairs.items():
        lin = modules.get(mod)
        if not isinstance(lin, torch.nn.Linear):
            raise KeyError(f"LoRA adapter for {mod!r}: no such Linear in the model")
        if not _targeted(mod, targets):
            raise KeyError(f"LoRA adapter for {mod!r} is not among the target modules {targets}")
        W = lin.weight
        r = A.shape[0]
        if A.shape != (r, W.shape[1]) or B.shape != (W.shape[0], r):
            raise ValueError(f"LoRA shapes for {mod!r}: A {tuple(A.shape)}, B {tuple(B.shape)} vs weight "
                             f"{tuple(W.shape)}")
        if rank is not None and r != rank:
            raise ValueError(f"LoRA rank of {mod!r} is {r}, lora_rank says {rank}")
        delta = B.to(W.device, torch.float32) @ A.to(W.device, torch.float32)
        W.copy_((W.float() + scaling * delta).to(W.dtype))
    return len(pairs)
