"""CPU: the T5 text-encoder restatement (oracle/t5_ref.py) pinned against transformers' T5EncoderModel, the
reference's dependency for encode_prompt (pipeline.py:126-175, pt.py:150-155), plus the host-side pieces of
f_lite.text_encoder (bucket table, state-dict layout, tokenizer stand-in)."""
import pytest
import torch

from oracle import t5_ref

transformers = pytest.importorskip("transformers")
from transformers import T5Config, T5EncoderModel  # noqa: E402

TINY = dict(vocab_size=1000, d_model=256, d_kv=64, d_ff=512, num_layers=4, num_heads=4,
            relative_attention_num_buckets=32, relative_attention_max_distance=128, layer_norm_epsilon=1e-6)


def hf_tiny(seed=0):
    cfg = T5Config(**TINY, feed_forward_proj="gated-gelu", dropout_rate=0.0, is_encoder_decoder=False)
    torch.manual_seed(seed)
    m = T5EncoderModel(cfg).eval()
    with torch.no_grad():  # non-trivial norm weights and a bias table with structure
        for n, p in m.named_parameters():
            if n.endswith("layer_norm.weight"):
                p.copy_(1 + 0.1 * torch.randn_like(p))
    return m


def test_bucket_table_matches_transformers():
    from f_lite.text_encoder import relative_position_bucket
    from transformers.models.t5.modeling_t5 import T5Attention

    rel = torch.arange(-1023, 1024)
    want = T5Attention._relative_position_bucket(rel, bidirectional=True, num_buckets=32, max_distance=128)
    assert torch.equal(relative_position_bucket(rel), want)
    assert torch.equal(t5_ref.relative_position_bucket(rel), want)


def test_module_tree_matches_transformers():
    from f_lite.text_encoder import T5Encoder

    with torch.device("meta"):
        ours = T5Encoder(**TINY)
    theirs = hf_tiny()
    a = {k: tuple(v.shape) for k, v in ours.state_dict().items()}
    b = {k: tuple(v.shape) for k, v in theirs.state_dict().items()}
    assert a == b


@pytest.mark.parametrize("masked", [False, True])
def test_oracle_matches_transformers(masked):
    m = hf_tiny()
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(2, 1000, (2, 40), generator=g)
    mask = None
    if masked:
        mask = torch.ones(2, 40, dtype=torch.long)
        mask[1, 23:] = 0
        ids[1, 23:] = 0
    with torch.no_grad():
        want = m(input_ids=ids, attention_mask=mask, output_hidden_states=True).hidden_states
        got = t5_ref.t5_encoder_hidden_states(m.state_dict(), TINY, ids, mask)
    assert len(got) == len(want) == TINY["num_layers"] + 1
    for i, (x, y) in enumerate(zip(got, want)):
        err = ((x - y).norm() / y.norm()).item()
        assert err < 1e-5, (i, err)
    # early stop: the state after 2 layers
    with torch.no_grad():
        part = t5_ref.t5_encoder_hidden_states(m.state_dict(), TINY, ids, mask, num_layers=2)
    assert len(part) == 3 and torch.allclose(part[2], want[2], rtol=1e-5, atol=1e-5)


def test_synthetic_tokenizer():
    from f_lite.text_encoder import SyntheticTokenizer

    tok = SyntheticTokenizer()
    out = tok(text=["a fox", "a red fox at dusk"], padding="longest", pad_to_multiple_of=8, max_length=512,
              truncation=True, return_tensors="pt")
    ids, mask = out["input_ids"], out["attention_mask"]
    assert ids.shape == (2, 24) and mask.shape == (2, 24)  # 17 bytes + EOS -> 18 -> 24
    assert mask[0].sum() == 6 and mask[1].sum() == 18
    assert ids[0, 5] == 1 and (ids[0, 6:] == 0).all()
    long = tok(text=["x" * 2000], max_length=512, truncation=True, pad_to_multiple_of=8)
    assert long["input_ids"].shape == (1, 512) and long["input_ids"][0, -1] == 1


def test_save_and_load_local_folder(tmp_path):
    """T5Encoder.save_pretrained -> from_pretrained (config.json + model.safetensors, T5EncoderModel keys); a
    transformers-saved folder loads the same way."""
    from f_lite.text_encoder import T5Encoder

    m = hf_tiny()
    m.save_pretrained(str(tmp_path / "hf"), safe_serialization=True)
    ours = T5Encoder.from_pretrained(str(tmp_path / "hf"), torch_dtype=torch.float32, device="cpu")
    want = m.state_dict()
    got = ours.state_dict()
    assert set(got) == set(want)
    assert all(torch.equal(got[k], want[k].float()) for k in want)
    ours.save_pretrained(tmp_path / "ours")
    again = T5Encoder.from_pretrained(tmp_path / "ours", torch_dtype=torch.float32, device="cpu")
    assert all(torch.equal(again.state_dict()[k], got[k]) for k in got)
