"""GPU: the native T5 v1.1 text encoder (f_lite.text_encoder, csrc/t5.hip) against the CPU restatement
(oracle/t5_ref.py, itself pinned to transformers' T5EncoderModel by tests/test_text_encoder_cpu.py), and the
encode_prompt path of FLitePipeline (pipeline.py:126-175) end to end.

Bars: the attention kernel and the GEGLU GEMM vs fp32 torch >= 45 dB; every hidden state of the encoder vs the
fp32 oracle >= 40 dB (bf16 weights and GEMM inputs; fp32 residual stream); hidden_states[-8] at the T5-XXL
layer width (d_model 4096, 64 heads, d_ff 10240, L = 512 with padding) >= 40 dB.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no ROCm device", allow_module_level=True)

from f_lite import _native as nat  # noqa: E402
from f_lite.text_encoder import T5_PRESETS, SyntheticTokenizer, T5Encoder  # noqa: E402
from oracle import t5_ref  # noqa: E402

DEV = "cuda"


def psnr(a, ref):
    a, ref = a.double().cpu(), ref.double().cpu()
    mse = (a - ref).pow(2).mean().item()
    return float("inf") if mse == 0 else 10 * math.log10(ref.abs().max().item() ** 2 / mse)


def cfg_dict(m):
    return {k: getattr(m.config, k) for k in T5_PRESETS["tiny"]}


@pytest.mark.parametrize("L", [8, 77, 512])
def test_t5_attention_kernel(L):
    B, H = 2, 4
    g = torch.Generator().manual_seed(L)
    qkv = (torch.randn(B * L, 3 * H * 64, generator=g) * 0.5).bfloat16()
    rel_w = torch.randn(32, H, generator=g).bfloat16()
    mask = torch.zeros(B, L)
    mask[1, L * 2 // 3:] = float("-inf")
    pos = torch.arange(L)
    bucket = t5_ref.relative_position_bucket(pos[None, :] - pos[:, None])
    bias = rel_w.float()[bucket].permute(2, 0, 1)  # [H, L, L]
    q, k, v = (qkv.float().view(B, L, 3, H, 64)[:, :, i].transpose(1, 2) for i in range(3))
    s = q @ k.transpose(-1, -2) + bias[None] + mask[:, None, None, :]
    ref = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B * L, H * 64)
    table = t5_ref.relative_position_bucket(torch.arange(-(L - 1), L)).to(torch.int32).to(DEV)
    qd, rel_d, mask_d = qkv.to(DEV), rel_w.to(DEV), mask.to(DEV)  # held: the kernel runs after the call returns
    out = torch.empty(B * L, H * 64, device=DEV, dtype=torch.bfloat16)
    lib = nat.load()
    nat.check(lib.flite_t5_attention(nat.stream_ptr(), qd.data_ptr(), 3 * H * 64, qd[:, H * 64:].data_ptr(),
                                     3 * H * 64, qd[:, 2 * H * 64:].data_ptr(), 3 * H * 64, out.data_ptr(), H * 64,
                                     table.data_ptr(), rel_d.data_ptr(), mask_d.data_ptr(), B, L, H),
              "flite_t5_attention")
    p = psnr(out.float(), ref)
    print(f"t5 attention L={L}: {p:.2f} dB vs fp32")
    assert p >= 45.0


def test_geglu_gemm():
    M, F, K = 600, 1024, 512
    g = torch.Generator().manual_seed(3)
    a = torch.randn(M, K, generator=g).bfloat16()
    w0 = (torch.randn(F, K, generator=g) * 0.05).bfloat16()
    w1 = (torch.randn(F, K, generator=g) * 0.05).bfloat16()
    out = nat.gemm(a.to(DEV), w0.to(DEV), w2=w1.to(DEV), epilogue=nat.EPI_GEGLU_BF16)
    ref = t5_ref.gelu_tanh(a.float() @ w0.float().t()) * (a.float() @ w1.float().t())
    p = psnr(out.float(), ref)
    print(f"GEGLU GEMM: {p:.2f} dB vs fp32")
    assert p >= 45.0


def _ids(B, L, vocab, seed, pad_from=None):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(2, vocab, (B, L), generator=g)
    mask = torch.ones(B, L, dtype=torch.long)
    if pad_from is not None:
        ids[-1, pad_from:] = 0
        mask[-1, pad_from:] = 0
    return ids, mask


def test_tiny_encoder_all_hidden_states():
    m = T5Encoder.random(seed=0, **T5_PRESETS["tiny"])
    ids, mask = _ids(2, 40, 1000, 1, pad_from=23)
    got = m(ids.to(DEV), mask.to(DEV), output_hidden_states=True).hidden_states
    sd = {k: v.cpu() for k, v in m.state_dict().items()}
    want = t5_ref.t5_encoder_hidden_states(sd, cfg_dict(m), ids, mask)
    assert len(got) == len(want) == 5
    for i, (x, y) in enumerate(zip(got, want)):
        p = psnr(x.float(), y)
        print(f"tiny T5 hidden_states[{i}]: {p:.2f} dB vs fp32 oracle")
        assert p >= 40.0
    # encode() = hidden_states[-8 mod 5] without running the later layers
    e = m.encode(ids.to(DEV), mask.to(DEV), return_index=-3)
    assert torch.equal(e.cpu(), got[2].cpu())


def test_xxl_width_layers_hidden_state():
    """T5-XXL layer shapes (d_model 4096, 64 heads, d_ff 10240) at L = 512 with a padded second prompt; 3
    layers so the CPU oracle stays quick (every XXL layer runs the same kernels)."""
    cfg = dict(T5_PRESETS["t5-xxl"], num_layers=3)
    m = T5Encoder.random(seed=1, **cfg)
    ids, mask = _ids(2, 512, 32128, 2, pad_from=300)
    got = m(ids.to(DEV), mask.to(DEV), output_hidden_states=True).hidden_states
    sd = {k: v.cpu() for k, v in m.state_dict().items()}
    want = t5_ref.t5_encoder_hidden_states(sd, cfg, ids, mask)
    for i in (1, 2, 3):
        p = psnr(got[i].float(), want[i])
        print(f"XXL-width T5 hidden_states[{i}] (L=512): {p:.2f} dB vs fp32 oracle")
        assert p >= 40.0


def test_xxl_full_encode_deterministic():
    m = T5Encoder.random(seed=2, **T5_PRESETS["t5-xxl"])
    ids, mask = _ids(1, 512, 32128, 3)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    a = m.encode(ids.to(DEV), mask.to(DEV))  # hidden_states[-8]: 17 layers
    e.record()
    torch.cuda.synchronize()
    b = m.encode(ids.to(DEV), mask.to(DEV))
    assert a.shape == (1, 512, 4096) and torch.isfinite(a.float()).all() and torch.equal(a, b)
    print(f"T5-XXL encode (17 layers, 512 tokens): {s.elapsed_time(e):.1f} ms")


def test_pipeline_encode_prompt_end_to_end():
    from f_lite import DiT, FLitePipeline
    from f_lite.model import PRESETS

    dit_cfg = dict(PRESETS["tiny"], cross_attn_input_size=256)
    dit = DiT.random(seed=0, device=DEV, **dit_cfg)
    enc = T5Encoder.random(seed=0, **dict(T5_PRESETS["tiny"], num_layers=8))  # hidden_states[-8] = after 1 layer
    tok = SyntheticTokenizer(vocab_size=1000)
    pipe = FLitePipeline(dit, text_encoder=enc, processor=tok)
    pos, neg = pipe.encode_prompt("a red fox at dusk")
    t = tok(text=["a red fox at dusk"], padding="longest", pad_to_multiple_of=8, max_length=512)
    want = t5_ref.t5_encoder_hidden_states({k: v.cpu() for k, v in enc.state_dict().items()}, cfg_dict(enc),
                                           t["input_ids"], t["attention_mask"])[-8]
    assert pos.shape == (1, 24, 256) and torch.equal(neg, torch.zeros_like(pos))
    assert psnr(pos.float(), want) >= 40.0
    lat = torch.randn(1, 16, 16, 16, generator=torch.Generator().manual_seed(0)).bfloat16().to(DEV)
    a = pipe(prompt="a red fox at dusk", latents=lat, height=128, width=128, num_inference_steps=3,
             output_type="latent").images
    b = pipe(prompt_embeds=pos, negative_prompt_embeds=neg, latents=lat, height=128, width=128,
             num_inference_steps=3, output_type="latent").images
    assert torch.equal(a, b)
