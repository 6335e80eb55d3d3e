"""CPU: host-side logic of the drop-in boundary (no kernels): parameter inventory, config, schedule,
FLOP accounting, fail-loudly behaviour."""
import json
import math

import pytest
import torch

from f_lite import APGConfig, DiT, FLitePipeline, FLitePipelineOutput
from f_lite._native import FliteError
from f_lite.model import PRESETS
from f_lite.pipeline import flow_schedule
from oracle import flite_ref as R
from oracle.vae_ref import vae_param_shapes
from oracle.weights import param_shapes


def test_public_names():
    import f_lite

    assert set(f_lite.__all__) == {"FLitePipeline", "FLitePipelineOutput", "APGConfig", "DiT"}
    assert APGConfig().enabled is True and APGConfig().orthogonal_threshold == 0.03


@pytest.mark.parametrize("name", ["7b", "10b", "tiny", "tiny_v2"])
def test_state_dict_inventory_matches_reference(name):
    with torch.device("meta"):
        m = DiT(**PRESETS[name])
    sd = m.state_dict()
    ref = param_shapes(dict(PRESETS[name]))
    assert set(sd) == set(ref)
    assert all(tuple(sd[k].shape) == tuple(ref[k]) for k in ref)


@pytest.mark.parametrize("name", ["tiny", "tiny_v2"])
def test_state_dict_inventory_learned_positional_embedding(name):
    """use_rope=False adds positional_embedding [1, 2048, D] (model.py:444)."""
    with torch.device("meta"):
        m = DiT(**PRESETS[name], use_rope=False)
    sd = m.state_dict()
    ref = param_shapes(dict(PRESETS[name], use_rope=False))
    assert "positional_embedding" in ref and set(sd) == set(ref)
    assert all(tuple(sd[k].shape) == tuple(ref[k]) for k in ref)


def test_reference_ctor_defaults():
    with torch.device("meta"):
        m = DiT()
    c = m.config
    assert (c.in_channels, c.patch_size, c.hidden_size, c.depth, c.num_heads, c.mlp_ratio, c.cross_attn_input_size) \
        == (4, 2, 1152, 28, 16, 4.0, 128)
    # reference zero-init of the adaLN / final layers (model.py:455-456,476-479)
    assert m.adaLN_modulation[1].weight.is_meta


def test_v2_module_alias():
    from f_lite.model_v2 import DiT as DiT2

    with torch.device("meta"):
        m = DiT2(**{k: v for k, v in PRESETS["tiny"].items() if k != "per_block_adaln"})
    assert m.per_block_adaln and all(b.cross_attn is not None for b in m.blocks)


def test_schedule_matches_reference(golden_meta):
    for key, rows in golden_meta["schedule"].items():
        hw, n = key.split(".")
        h, w = map(int, hw.split("x"))
        got = flow_schedule(int(n), h // 8, w // 8)
        assert [(t, dt) for t, dt in got] == [tuple(r) for r in rows]


def test_schedule_explicit_alpha():
    """__call__'s alpha (reference pipeline.py:239-256): an explicit alpha replaces 2*sqrt(tokens / 64^2); alpha = 1
    is the unshifted linear schedule t = i/n, dt = 1/n; the shifted t stay in (0, 1], decrease, and the dt sum to 1."""
    lin = flow_schedule(8, 128, 128, alpha=1.0)
    assert [t for t, _ in lin] == [i / 8 for i in range(8, 0, -1)]
    assert all(abs(dt - 1 / 8) < 1e-15 for _, dt in lin)
    for a in (0.5, 3.0, 7.5):
        s = flow_schedule(30, 96, 160, alpha=a)
        ts = [t for t, _ in s]
        assert ts[0] == 1.0 and all(0.0 < x <= 1.0 for x in ts) and all(x > y for x, y in zip(ts, ts[1:]))
        assert abs(sum(dt for _, dt in s) - 1.0) < 1e-12
        i = 10  # the 21st step: t = i/n shifted by alpha
        assert s[30 - i][0] == (i / 30) * a / (1 + (a - 1) * (i / 30))
    assert flow_schedule(30, 128, 128) == flow_schedule(30, 128, 128, alpha=2 * (128 * 128 / 64 ** 2) ** 0.5)


def test_forward_on_cpu_raises():
    m = DiT(**PRESETS["tiny"])
    with pytest.raises(FliteError):
        m(torch.zeros(1, 16, 8, 8), torch.zeros(1, 4, 128), torch.tensor([0.5]))
    with pytest.raises(TypeError):
        m(torch.zeros(1, 16, 8, 8), torch.zeros(1, 4, 128))


def test_pipeline_requires_embeddings_without_text_encoder():
    m = DiT(**PRESETS["tiny"])
    p = FLitePipeline(m)
    with pytest.raises(ValueError):
        p.encode_prompt("a cat")


def test_save_and_load_config_roundtrip(tmp_path):
    m = DiT(**PRESETS["tiny"])
    m.save_pretrained(tmp_path / "dit_model")
    cfg = json.loads((tmp_path / "dit_model" / "config.json").read_text())
    assert cfg["hidden_size"] == 512 and cfg["_class_name"] == "DiT"
    m2 = DiT.from_pretrained(tmp_path, subfolder="dit_model", torch_dtype=torch.float32, device="cpu")
    for (k, a), (k2, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert k == k2 and torch.equal(a, b)


def test_vae_inventory():
    from f_lite.vae import AutoencoderKL

    with torch.device("meta"):
        v = AutoencoderKL()
    sd = v.state_dict()
    ref = vae_param_shapes()
    assert set(sd) == set(ref) and all(tuple(sd[k].shape) == ref[k] for k in ref)
    assert sum(math.prod(s) for s in ref.values()) == 49545475


def test_flop_accounting_matches_survey():
    import bench

    f_step, f_once = bench.dit_flops(PRESETS["10b"], 1024, 1024, 30)
    assert abs(f_step / 1e12 - 65.23) < 0.01 and abs(f_once / 1e9 - 786.0) < 0.1
    f_step7, f_once7 = bench.dit_flops(PRESETS["7b"], 1024, 1024, 30)
    assert abs(f_step7 / 1e12 - 60.88) < 0.01 and abs(f_once7 / 1e9 - 322.1) < 0.1
    from f_lite.vae import decoder_flops

    assert abs(decoder_flops(1024, 1024) / 1e12 - 10.47) < 0.01


def test_cpu_baseline_threads_follow_cgroup_quota(monkeypatch):
    """bench.cpu_threads: every CPU the cgroup quota grants, else the affinity set capped by
    OMP_NUM_THREADS, with the reason recorded."""
    import bench

    info = {"affinity_cores": 256, "cgroup_cpus": 16.0, "cgroup_cpu_max": "cpu.max: 1600000 100000"}
    monkeypatch.setattr(bench, "host_info", lambda: dict(info))
    n, why = bench.cpu_threads()
    assert n == 16 and "quota grants 16" in why
    info.update(cgroup_cpus=None, cgroup_cpu_max="cpu.max: max 100000")
    monkeypatch.setenv("OMP_NUM_THREADS", "16")
    n, why = bench.cpu_threads()
    assert n == 16 and "OMP_NUM_THREADS=16" in why
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.cpu_threads()[0] == 256
    q = bench.cgroup_cpu_quota()
    assert set(q) == {"cgroup_cpu_max", "cgroup_cpus"}


def test_cpu_baseline_whole_step_with_component_check():
    """bench.cpu_baseline_full (the default `cpu_baseline` since round 6): whole measured CFG
    step(s) of the fp32 port extrapolated x steps/K, and the per-component sample beside it (shape of the record on
    a tiny model; the GPU box runs the 10B 1024^2 workload)."""
    import bench
    from oracle.weights import make_param, param_shapes

    cfg = dict(PRESETS["tiny"])

    class _Params:
        def named_parameters(self):
            return [(k, make_param(k, v)) for k, v in param_shapes(cfg).items()]

    full = bench.cpu_baseline_full(_Params(), None, cfg, 64, 64, 4, k_steps=1)
    assert full["kind"] == "port" and full["extrapolated"] and full["value"] > 0
    assert "1 whole CFG-6 steps of the 4-step schedule" in full["sample"]
    chk = bench.cpu_baseline_sample(_Params(), None, cfg, 64, 64, 4, n_blocks=1, vae_s=full["components_s"]["vae_s"])
    assert chk["value"] > 0 and chk["components_s"]["vae_s"] == 0.0


class _PointwiseDecoder:
    """Stand-in decoder whose pixel (y, x) depends only on latent (y // 8, x // 8): any correct tiling of it
    (grid, in-place blends of equal overlaps, crops, concatenation) reproduces the untiled output exactly."""

    def decode(self, z):
        return z[:, :3].repeat_interleave(8, dim=2).repeat_interleave(8, dim=3) * 0.5


@pytest.mark.parametrize("h,w,tl", [(112, 168, 128), (20, 28, 16), (16, 40, 16), (33, 7, 8)])
def test_vae_tiled_decode_grid_is_exact_for_pointwise_decoder(h, w, tl):
    from oracle.vae_ref import tiled_decode

    g = torch.Generator().manual_seed(h * w)
    z = torch.randn(1, 16, h, w, generator=g)
    dec = _PointwiseDecoder()
    out = tiled_decode(dec, z, tile_latent=tl, tile_sample=8 * tl, overlap=0.25)
    assert out.shape == (1, 3, 8 * h, 8 * w)
    torch.testing.assert_close(out, dec.decode(z), rtol=0, atol=1e-6)


def test_vae_tiling_flags():
    from f_lite.vae import AutoencoderKL

    vae = AutoencoderKL.empty(device="cpu")
    assert (vae.tile_latent_min_size, vae.tile_sample_min_size, vae.tile_overlap_factor) == (128, 1024, 0.25)
    assert not vae.use_tiling
    FLitePipeline(None, vae).enable_vae_tiling()  # pipeline.py:90-93 forwards to the VAE
    assert vae.use_tiling


class _ChatProcessor:
    """A processor with a chat template (Qwen2.5-VL's AutoProcessor shape): records what it is asked to render
    and tokenize."""

    chat_template = "{{ messages }}"

    def __init__(self):
        self.rendered = []

    def apply_chat_template(self, messages, tokenize=False, add_generation_prompt=False):
        assert tokenize is False and add_generation_prompt is True
        self.rendered.append(messages)
        return "<chat>" + messages[0]["content"][:16] + "|" + messages[1]["content"][0]["text"] + "</chat>"

    def __call__(self, text=None, **kw):
        self.texts = list(text)
        n = max(len(t) for t in text)
        return {"input_ids": torch.ones(len(text), n, dtype=torch.long),
                "attention_mask": torch.ones(len(text), n, dtype=torch.long)}


class _HiddenStatesEncoder(torch.nn.Module):
    """Stands in for a transformers encoder called the reference's way (pipeline.py:148-154)."""

    def __init__(self):
        super().__init__()
        self.w = torch.nn.Parameter(torch.zeros(1))

    @property
    def device(self):
        return torch.device("cpu")

    def forward(self, input_ids=None, attention_mask=None, use_cache=False, return_dict=True,
                output_hidden_states=True):
        from types import SimpleNamespace

        h = input_ids.float()[..., None].expand(-1, -1, 8)
        return SimpleNamespace(hidden_states=[h] * 9)


def test_encode_prompt_applies_reference_chat_template():
    """pipeline.py:105-124,139-142: a processor with a chat template gets the reference's system + user messages
    for every caption (negative prompts too); the rendered strings are what gets tokenized."""
    import re

    from f_lite.pipeline import _SYSTEM_PROMPT

    proc = _ChatProcessor()
    p = FLitePipeline(DiT(**PRESETS["tiny"]), text_encoder=_HiddenStatesEncoder(), processor=proc)
    pos, neg = p.encode_prompt(["a cat", "a dog"], negative_prompt="blurry", dtype=torch.float32)
    assert pos.shape[0] == 2 and neg.shape[0] == 1
    assert [m[1]["content"][0]["text"] for m in proc.rendered] == ["a cat", "a dog", "blurry"]
    for m in proc.rendered:
        assert m[0] == {"role": "system", "content": _SYSTEM_PROMPT}
        assert m[1]["role"] == "user" and m[1]["content"][0]["type"] == "text"
    assert proc.texts == ["<chat>" + _SYSTEM_PROMPT[:16] + "|blurry</chat>"]
    # the system prompt is the reference's text, character for character
    src = open("/root/reference/f_lite/pipeline.py").read() if __import__("os").path.exists(
        "/root/reference/f_lite/pipeline.py") else None
    if src is not None:
        assert re.search(r'system_prompt = "(.*?)"\n', src).group(1) == _SYSTEM_PROMPT
    # an explicit caption_to_text hook wins over the template
    p.caption_to_text = lambda c: "raw:" + c
    p.encode_prompt("x", dtype=torch.float32)
    assert proc.texts == ["raw:x"]


def test_apg_step_scalar_algebra_matches_reference():
    """distributed.apg_step (the two-phase APG used by the CFG-parallel and data-parallel modes) with torch sums
    equals pipeline.py:276-287's whole-batch APG on the same branch outputs."""
    from f_lite.distributed import apg_step

    g = torch.Generator().manual_seed(3)
    u = torch.randn(3, 16, 8, 8, generator=g)
    c = u + 0.3 * torch.randn(3, 16, 8, 8, generator=g)
    acc = torch.randn(3, 16, 8, 8, generator=g)

    def sums(u_, c_, k, phase):
        if phase == 0:
            return torch.stack([(c_ * (c_ - u_)).sum(), (c_ * c_).sum()])
        o = (c_ - u_) - k * c_
        return torch.stack([o.sum(), (o * o).sum()])

    def update(a, u_, c_, gs, k, sc, dt):
        a += dt * (c_ + (gs - 1) * sc * ((c_ - u_) - k * c_))

    got = apg_step(acc.clone(), u, c, 0.1, 6.0, 0.03, u.numel(), sums, update)
    dy, dd = c, c - u
    orth = dd - (dy * dd).sum() / (dy * dy).sum() * dy
    want = acc + 0.1 * (dy + 5.0 * orth * min(1, 0.03 / orth.std()))
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-6)


def test_fp8_policy_parsing():
    """_native.fp8_class_mask refuses a bool and an empty class set (`--fp8-classes ''` silently ran
    bf16); fp8_block_masks expands the per-block policy strings of bench.py --fp8-block-classes
    (include/flite.h flite_dit_set_fp8_block_classes)."""
    from f_lite import _native as nat

    assert nat.fp8_class_mask(None) == 63 and nat.fp8_class_mask("all") == 63 and nat.fp8_class_mask(0) == 0
    assert nat.fp8_class_mask(["gate_up", "qkv"]) == 17
    for bad in (True, "", [], "nope"):
        with pytest.raises(nat.FliteError):
            nat.fp8_class_mask(bad)
    m = nat.fp8_block_masks("0-3:none;4-7:gate_up+qkv;39:32", 40, default=63)
    assert m[:4] == [0] * 4 and m[4:8] == [17] * 4 and m[8:39] == [63] * 31 and m[39] == 32
    assert nat.fp8_block_masks("", 3, default=5) == [5, 5, 5]
    for bad in ("0-40:all", "3", "2-1:all", "0:64"):
        with pytest.raises(nat.FliteError):
            nat.fp8_block_masks(bad, 40)
