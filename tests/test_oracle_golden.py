"""CPU: the oracle restatement (oracle/flite_ref.py) against golden vectors produced by the reference
itself (tests/golden/make_golden.py). fp32 paths must agree to ~1e-5 relative."""
import math

import pytest
import torch

from oracle import flite_ref as R
from oracle.weights import make_state_dict, param_shapes


def rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm()).item()


def test_timestep_embedding(golden):
    t = golden["op.temb_bf16t.t"].bfloat16()
    assert rel(R.timestep_embedding(t * 1000, 512), golden["op.temb_bf16t.out"]) < 1e-6
    t = golden["op.temb_f32t.t"]
    assert rel(R.timestep_embedding(t * 1000, 512), golden["op.temb_f32t.out"]) < 1e-6


def test_rope_tables(golden):
    cos, sin = R.rope_tables(12, 20, 128, 10000.0, 16, torch.float32)
    assert torch.equal(cos, golden["op.rope.cos"]) and torch.equal(sin, golden["op.rope.sin"])
    cb, sb = R.rope_tables(12, 20, 128, 10000.0, 16, torch.bfloat16)
    assert torch.equal(cb.float(), golden["op.rope_bf16.cos"]) and torch.equal(sb.float(), golden["op.rope_bf16.sin"])


def test_apply_rope(golden):
    cos, sin = golden["op.rope.cos"][:256][None], golden["op.rope.sin"][:256][None]
    assert rel(R.apply_rotary_emb(golden["op.apply_rope.x"], cos, sin), golden["op.apply_rope.out"]) < 1e-6


def test_rmsnorm(golden):
    x = golden["op.rmsnorm.x"]
    assert rel(R.own_rmsnorm(x, golden["op.rmsnorm.w"]), golden["op.rmsnorm.out"]) < 1e-6
    assert rel(R.own_rmsnorm(x, None), golden["op.rmsnorm_noweight.out"]) < 1e-6


@pytest.fixture(scope="module")
def tiny32():
    return R.RefDiT.random(R.PRESETS["tiny"], dtype=torch.float32)


@pytest.mark.parametrize("key,mask,tbf", [("nomask", False, False), ("mask", True, False), ("bf16t", False, True)])
def test_dit_tiny_fp32(golden, tiny32, key, mask, tbf):
    t = golden["in.t"].bfloat16() if tbf else golden["in.t"]
    out = tiny32(golden["in.x"], golden["in.ctx"], golden["in.mask"] if mask else None, t)
    assert rel(out, golden[f"dit.tiny.f32.{key}"]) < 2e-5


def test_dit_tiny_bf16(golden):
    d = R.RefDiT.random(R.PRESETS["tiny"], dtype=torch.bfloat16)
    out = d(golden["in.x"].bfloat16(), golden["in.ctx"].bfloat16(), None, golden["in.t"].bfloat16()).float()
    # same rounding points as the reference; CPU bf16 GEMM accumulation order may differ slightly
    assert rel(out, golden["dit.tiny.bf16.nomask"]) < 2e-2


def test_dit_tiny_v2_fp32(golden):
    d = R.RefDiT.random(R.PRESETS["tiny_v2"], dtype=torch.float32)
    out = d(golden["in.x"], golden["in.ctx"], None, golden["in.t"])
    assert rel(out, golden["dit.tiny_v2.f32.nomask"]) < 2e-5


def test_schedule(golden_meta):
    for key, rows in golden_meta["schedule"].items():
        hw, n = key.split(".")
        h, w = map(int, hw.split("x"))
        got = R.schedule(int(n), h, w)
        assert len(got) == len(rows)
        for (t, dt), (rt, rdt) in zip(got, rows):
            assert t == rt and dt == rdt


@pytest.mark.parametrize("key,g,apg", [("cfg6", 6.0, False), ("cfg1", 1.0, False), ("apg", 6.0, True),
                                      ("nocfg", 0.5, False)])
def test_pipeline_fp32(golden, tiny32, key, g, apg):
    lat = R.sample(tiny32, golden["pipe.in.latents"], golden["pipe.in.pos"], torch.zeros_like(golden["pipe.in.pos"]),
                   num_steps=4, guidance_scale=g, apg=R.APG(enabled=apg), height=128, width=128)
    ref = golden[f"pipe.f32.{key}"]  # = latents / 0.3611 + 0.1159 (pipeline.py:304)
    assert rel(lat / 0.3611 + 0.1159, ref) < 2e-5


def test_param_inventory_counts():
    # 7B = 6,836,981,824 params; 10B-v2 = 11,056,776,256
    for name, n in (("7b", 6836981824), ("10b", 11056776256)):
        shapes = param_shapes(R.PRESETS[name].as_dict())
        assert sum(math.prod(s) for s in shapes.values()) == n


def test_generator_deterministic():
    a = make_state_dict(R.PRESETS["tiny"].as_dict(), names=["blocks.0.self_attn.qkv.weight"])
    b = make_state_dict(R.PRESETS["tiny"].as_dict(), names=["blocks.0.self_attn.qkv.weight"])
    w = a["blocks.0.self_attn.qkv.weight"]
    assert torch.equal(w, b["blocks.0.self_attn.qkv.weight"])
    assert abs(w.std().item() - 0.02) < 1e-3 and abs(w.mean().item()) < 1e-3
    assert torch.equal(w, w.bfloat16().float())


@pytest.mark.parametrize("preset,key,mask", [("tiny", "tiny", False), ("tiny", "tiny", True),
                                             ("tiny_v2", "tiny_v2", False)])
def test_dit_released_layout_fp32(golden, golden_nobias, preset, key, mask):
    """train_bias_and_rms=False (the layout pt.py:31 loads): no qkv / q / context_kv biases (model.py:465) and
    a weight-less final RMSNorm (model.py:474), pinned to the stub-loaded reference (make_golden_nobias.py)."""
    import dataclasses

    cfg = dataclasses.replace(R.PRESETS[preset], train_bias_and_rms=False)
    d = R.RefDiT.random(cfg, dtype=torch.float32)
    assert "final_norm.weight" not in d.p and not any(k.endswith("qkv.bias") for k in d.p)
    out = d(golden["in.x"], golden["in.ctx"], golden["in.mask"] if mask else None, golden["in.t"])
    assert rel(out, golden_nobias[f"dit.{key}.nobias.f32.{'mask' if mask else 'nomask'}"]) < 2e-5
