"""The premise of dit.cpp's uniform-context collapse, checked on the oracle (the reference's arithmetic restated,
oracle/flite_ref.py, pinned to the stub-loaded reference's fixtures): a context whose rows are all equal -- the
pipeline's zero negative prompt (pipeline.py:160-161) or any repeated row -- stays a set of equal rows through
context_proj + context_norm (model.py:527-530), context_kv and the key QK-norm (model.py:189-197), so the
cross-attention of every query is the value row itself (softmax over equal scores, model.py:203-210), and the
sub-block's output is gate_ca * (v . Wproj^T) whatever the query (model.py:291-297). The GPU test
(test_gpu_dit.py::test_uniform_context_collapse_matches_full_computation) checks the HIP path against the full
computation; this one checks the algebra the HIP path relies on, on CPU."""
import pytest
import torch

from oracle import flite_ref as R


@pytest.mark.parametrize("kind", ["zero", "const"])
def test_uniform_context_cross_attention_is_the_value_row(kind):
    cfg = R.PRESETS["tiny"]
    ref = R.RefDiT.random(cfg, dtype=torch.float32)
    g = torch.Generator().manual_seed(3)
    C, D, H = cfg.cross_attn_input_size, cfg.hidden_size, cfg.num_heads
    row = torch.zeros(1, 1, C) if kind == "zero" else torch.randn(1, 1, C, generator=g)
    ctx = row.expand(1, 24, C).contiguous()
    c = R.liger_rmsnorm(ref._lin(ctx, "context_proj"), ref.p["context_norm.weight"])
    ctx_flat, ctx_cu, _, _ = R.prepare_varlen(c)
    assert torch.equal(ctx_flat, ctx_flat[:1].expand_as(ctx_flat))  # row-wise ops keep equal rows equal
    T = 80
    q = R.own_rmsnorm(torch.randn(T, H, D // H, generator=g), None)
    cu = torch.tensor([0, T], dtype=torch.int32)
    checked = 0
    for i in range(cfg.depth):
        if not cfg.cross(i):
            continue
        pre = f"blocks.{i}."
        kv = ref._lin(ctx_flat, pre + "cross_attn.context_kv")
        kk, vv = kv.reshape(kv.shape[0], 2, H, -1).permute(1, 0, 2, 3).unbind(0)
        kk = R.own_rmsnorm(kk, None)
        assert torch.equal(kk, kk[:1].expand_as(kk)) and torch.equal(vv, vv[:1].expand_as(vv))
        a = R.attention_varlen(q, kk, vv, cu, ctx_cu, (D // H) ** -0.5)
        err = (a - vv[:1]).abs().max().item() / vv.abs().max().item()
        assert err < 1e-6, (i, err)  # the softmax weights are 1/24 each: v to fp32 rounding
        # the sub-block's output is then one row, whatever the query: gate * (v . Wproj^T)
        out = ref._lin(a.reshape(T, -1), pre + "cross_attn.proj", bias=False)
        c_row = ref._lin(vv[:1].reshape(1, -1), pre + "cross_attn.proj", bias=False)
        assert (out - c_row).abs().max().item() <= 1e-5 * max(c_row.abs().max().item(), 1e-12)
        checked += 1
    assert checked == sum(cfg.cross(i) for i in range(cfg.depth))
