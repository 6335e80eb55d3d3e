"""`f_lite.model_v2.DiT` (reference f_lite/model_v2.py): the per-block-adaLN layout with cross-attention in
every block -- the "10B" configuration. Same native engine as f_lite.model."""
from .model import DiT as _DiT


class DiT(_DiT):
    _per_block_adaln_default = True


__all__ = ["DiT"]
