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

import logging
import re
from typing import Dict, Iterable, Optional, Tuple

import torch

logger = logging.getLogger(__name__)

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
    """Fold every adapter of `state_dict` into `model` in place: W <- W_base + scaling * B @ A. Returns the number of
    merged modules.

    Loading REPLACES, as peft's set_peft_model_state_dict does for the model's one ("default") adapter
    (/root/reference/f_lite/model.py:492-495, pt.py:123-126): a module that already carries a merged adapter is
    first restored to its base weight (kept on the host at the first merge), so loading the same file twice leaves
    the weights bit-identical, and a second adapter does not stack on the first. Modules the new file does not name
    keep the adapter they had, as peft's do. If a merged weight was overwritten since (load_state_dict, random_init_),
    its current value is taken as the new base. "Still holds our merge" is decided by the weight's CONTENT (a 64-bit
    fingerprint of its bits recorded after the merge), not by its version counter or storage pointer: a write through
    `p.data` (which bumps no version) is seen, and a `.to(device)` after the merge (new pointer, same bits) still
    restores the kept base. Cost: the base of every merged module stays on the host (bf16: 2 bytes per weight) for
    the model's lifetime, which is what makes a reload bit-identical rather than W - B@A rounded twice.

    Adapters on modules that do not exist or that `target_modules` does not select are skipped with a warning (peft
    loads with strict=False and reports them as unexpected keys). A shape or rank mismatch raises: peft would
    refuse to copy such a tensor too."""
    targets = None if target_modules is None else [t.strip() for t in target_modules if t.strip()]
    modules = dict(model.named_modules())
    pairs = lora_pairs(state_dict)
    todo, skipped = [], []
    for mod, (A, B) in pairs.items():
        lin = modules.get(mod)
        if not isinstance(lin, torch.nn.Linear) or not _targeted(mod, targets):
            skipped.append(mod)
            continue
        W = lin.weight
        r = A.shape[0]
        if A.shape != (r, W.shape[1]) or B.shape != (W.shape[0], r):
            raise ValueError(f"LoRA shapes for {mod!r}: A {tuple(A.shape)}, B {tuple(B.shape)} vs weight "
                             f"{tuple(W.shape)}")
        if rank is not None and r != rank:
            raise ValueError(f"LoRA rank of {mod!r} is {r}, lora_rank says {rank}")
        todo.append((mod, lin, A, B))
    if skipped:
        logger.warning("LoRA: skipped %d adapter(s) on modules that are missing or not targeted (%s): %s",
                       len(skipped), targets, ", ".join(sorted(skipped)[:8]) + (" ..." if len(skipped) > 8 else ""))
    merged = getattr(model, "_lora_merged", None)
    if merged is None:
        merged = {}
        object.__setattr__(model, "_lora_merged", merged)
    for mod, lin, A, B in todo:
        W = lin.weight
        rec = merged.get(mod)
        if rec is not None and rec["fp"] == _fingerprint(W):
            base = rec["base"]  # the weight still holds our merge: start from the kept base
        else:
            base = W.detach().to("cpu", copy=True)
        delta = B.to(W.device, torch.float32) @ A.to(W.device, torch.float32)
        W.copy_((base.to(W.device, torch.float32) + scaling * delta).to(W.dtype))
        merged[mod] = {"A": A.detach().cpu(), "B": B.detach().cpu(), "scaling": scaling, "base": base,
                       "fp": _fingerprint(W)}
    return len(todo)


_INT_OF = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}


_FP_CHUNK = 1 << 24  # elements per fingerprint pass: bounds the int64 temporaries to ~0.7 GB


def _fingerprint(W: torch.Tensor) -> Tuple[int, int, int]:
    """Position-weighted 64-bit sums of the tensor's raw bits (wrapping), on its own device: equal contents give equal
    fingerprints wherever the tensor lives; a changed element changes them but for a 2^-64-scale accident. Hashed in
    chunks of _FP_CHUNK elements (the sums wrap the same way chunked or whole)."""
    flat = W.detach().contiguous().reshape(-1).view(_INT_OF[W.element_size()])
    acc = torch.zeros(3, dtype=torch.int64, device=flat.device)
    for c0 in range(0, flat.numel(), _FP_CHUNK):
        bits = flat[c0:c0 + _FP_CHUNK].to(torch.int64)
        idx = torch.arange(c0, c0 + bits.numel(), device=bits.device, dtype=torch.int64)
        mult = (idx * 2654435761 + 97) % 2147483629 + 1
        acc[0] += bits.sum()
        acc[1] += (bits * mult).sum()
        acc[2] += (bits * bits * (idx % 8191 + 1)).sum()
    return tuple(int(v) for v in acc.tolist())


def merged_state_dict(model: torch.nn.Module) -> Dict[str, torch.Tensor]:
    """The adapters currently merged into `model`, as a peft state dict ("<module>.lora_A.weight" / "lora_B")."""
    out = {}
    for mod, rec in sorted(getattr(model, "_lora_merged", {}).items()):
        out[f"{mod}.lora_A.weight"] = rec["A"]
        out[f"{mod}.lora_B.weight"] = rec["B"]
    return out
