"""Golden fixtures for the RELEASED-checkpoint layout, train_bias_and_rms=False (run in the build container only).

pt.py:31 loads the released F-Lite checkpoints with train_bias_and_rms=False: no qkv / q / context_kv biases
(model.py:465 qkv_bias=train_bias_and_rms) and a final RMSNorm without weight (model.py:474 trainable=...).
Same stub-loading as make_golden.py; the reference DiT of each tiny layout is built with that flag, loaded
strictly with the generator's no-bias state dict (which also pins the parameter inventory) and run in fp32 on
make_golden.py's stored inputs (golden.safetensors in.x / in.ctx / in.mask / in.t).

    python tests/golden/make_golden_nobias.py     -> tests/golden/golden_nobias.safetensors (~100 KB)
"""
from __future__ import annotations

import sys

sys.dont_write_bytecode = True

from pathlib import Path  # noqa: E402

import torch  # noqa: E402
from safetensors.torch import load_file, save_file  # noqa: E402

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
import make_golden as MG  # noqa: E402


def main():
    MG.install_stubs()
    model = MG.load_ref("model")
    model_v2 = MG.load_ref("model_v2")
    g = load_file(str(HERE / "golden.safetensors"))
    x, ctx, mask, ts = g["in.x"], g["in.ctx"], g["in.mask"], g["in.t"]
    T = {}
    with torch.no_grad():
        tiny = dict(MG.TINY, train_bias_and_rms=False)
        d = MG.build(model, tiny, False, torch.float32)
        assert d.final_norm.weight is None and d.blocks[0].self_attn.qkv.bias is None
        T["dit.tiny.nobias.f32.nomask"] = d(x, ctx, None, ts)
        T["dit.tiny.nobias.f32.mask"] = d(x, ctx, mask, ts)
        tiny_v2 = dict(MG.TINY_V2, train_bias_and_rms=False)
        d2 = MG.build(model_v2, tiny_v2, True, torch.float32)
        T["dit.tiny_v2.nobias.f32.nomask"] = MG.v2_forward_fixed(d2, model_v2, x, ctx, None, ts)
    save_file({k: v.contiguous().float() for k, v in T.items()}, str(HERE / "golden_nobias.safetensors"))
    print("wrote", sorted(T))


if __name__ == "__main__":
    main()
