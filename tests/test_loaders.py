"""CPU: the loading surface of the drop-in -- diffusers-folder round trips for both layouts (model_index.json's
dit_model module decides, generate.py:61-68), raw .pt checkpoints (pt.py:78-104), and the f_lite.generate CLI
(generate.py:13-116: arguments, defaults, output naming). No kernels run here."""
import inspect
import json
import subprocess
import sys
from pathlib import Path

import pytest
import torch

from f_lite import DiT, FLitePipeline
from f_lite.model import PRESETS
from f_lite.model_v2 import DiT as DiTv2

ROOT = Path(__file__).resolve().parents[1]


def _filled(cls, preset, seed=0):
    cfg = dict(PRESETS[preset])
    m = cls(**cfg)
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.randn(p.shape, generator=g))
    return m


def _same_weights(a, b):
    sa, sb = a.state_dict(), b.state_dict()
    return set(sa) == set(sb) and all(torch.equal(sa[k].float(), sb[k].float()) for k in sa)


@pytest.mark.parametrize("preset,module", [("tiny", "f_lite.model"), ("tiny_v2", "f_lite.model_v2")])
def test_pipeline_folder_round_trip(tmp_path, preset, module):
    m = _filled(DiT, preset)
    FLitePipeline(m).save_pretrained(tmp_path)
    index = json.loads((tmp_path / "model_index.json").read_text())
    assert index["dit_model"] == [module, "DiT"]
    cfg = json.loads((tmp_path / "dit_model" / "config.json").read_text())
    assert "per_block_adaln" not in cfg  # reference config.json keys only (model.py:419-433)
    pipe = FLitePipeline.from_pretrained(tmp_path, torch_dtype=torch.float32, device="cpu")
    assert isinstance(pipe.dit_model, DiTv2 if module.endswith("v2") else DiT)
    assert pipe.dit_model.per_block_adaln == module.endswith("v2")
    assert _same_weights(pipe.dit_model, m)


def test_reference_shaped_v2_folder(tmp_path):
    """A folder as the reference would save a model_v2 DiT: ["f_lite.model_v2", "DiT"] and no layout key."""
    m = _filled(DiTv2, "tiny_v2")
    (tmp_path / "dit_model").mkdir(parents=True)
    m.save_pretrained(tmp_path / "dit_model")
    (tmp_path / "model_index.json").write_text(json.dumps(
        {"_class_name": "FLitePipeline", "dit_model": ["f_lite.model_v2", "DiT"],
         "vae": ["diffusers", "AutoencoderKL"], "text_encoder": ["transformers", "T5EncoderModel"]}))
    pipe = FLitePipeline.from_pretrained(tmp_path, torch_dtype=torch.float32, device="cpu")
    assert pipe.dit_model.per_block_adaln and _same_weights(pipe.dit_model, m)


def test_layout_mismatch_is_refused(tmp_path):
    m = _filled(DiTv2, "tiny_v2")
    FLitePipeline(m).save_pretrained(tmp_path)
    idx = json.loads((tmp_path / "model_index.json").read_text())
    idx["dit_model"] = ["f_lite.model", "DiT"]  # wrong module for per-block adaLN weights
    (tmp_path / "model_index.json").write_text(json.dumps(idx))
    with pytest.raises(ValueError, match="model_v2"):
        FLitePipeline.from_pretrained(tmp_path, torch_dtype=torch.float32, device="cpu")
    idx["dit_model"] = ["somewhere.else", "DiT"]
    (tmp_path / "model_index.json").write_text(json.dumps(idx))
    with pytest.raises(ValueError, match="unknown module"):
        FLitePipeline.from_pretrained(tmp_path, torch_dtype=torch.float32, device="cpu")


@pytest.mark.parametrize("preset", ["tiny", "tiny_v2"])
def test_pt_checkpoint(tmp_path, preset):
    """load_f_lite_pt: depth from the block indices, heads = width // 256, DDP / compile prefixes stripped."""
    from f_lite.pt import infer_dit_config, load_f_lite_pt

    m = _filled(DiT, preset)
    sd = {("module._orig_mod." if i % 2 else "") + k: v for i, (k, v) in enumerate(m.state_dict().items())}
    path = tmp_path / "ckpt.pt"
    torch.save(sd, path)
    cfg = infer_dit_config({k.replace("module.", "").replace("_orig_mod.", ""): v for k, v in sd.items()},
                           width=512, cross_attn_input_size=128, train_bias_and_rms=True)
    assert cfg["depth"] == PRESETS[preset]["depth"] and cfg["num_heads"] == 2
    assert cfg["per_block_adaln"] == PRESETS[preset]["per_block_adaln"]
    pipe = load_f_lite_pt(path, "cpu", dtype="bfloat16", width=512, cross_attn_input_size=128,
                          train_bias_and_rms=True)
    assert pipe.dit_model.dtype == torch.bfloat16
    ref = {k: v.bfloat16() for k, v in m.state_dict().items()}
    got = pipe.dit_model.state_dict()
    assert set(got) == set(ref) and all(torch.equal(got[k], ref[k]) for k in ref)


def test_pt_checkpoint_errors(tmp_path):
    from f_lite.pt import load_f_lite_pt

    m = _filled(DiT, "tiny")
    sd = m.state_dict()
    sd.pop("final_proj.bias")
    torch.save(sd, tmp_path / "bad.pt")
    with pytest.raises(KeyError):
        load_f_lite_pt(tmp_path / "bad.pt", "cpu", width=512, cross_attn_input_size=128, train_bias_and_rms=True)
    with pytest.raises(NotImplementedError):
        load_f_lite_pt(tmp_path / "bad.pt", "cpu", residual_v=True)


def _lora_sd(model, targets=("qkv", "q", "context_kv", "proj"), rank=4, seed=1):
    """A peft-format LoRA state dict (get_peft_model_state_dict keys: "<module>.lora_A.weight" [r, in],
    "<module>.lora_B.weight" [out, r]) for every Linear whose name ends in one of `targets`."""
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for name, mod in model.named_modules():
        if isinstance(mod, torch.nn.Linear) and any(name == t or name.endswith("." + t) for t in targets):
            sd[f"{name}.lora_A.weight"] = torch.randn(rank, mod.in_features, generator=g) * 0.1
            sd[f"{name}.lora_B.weight"] = torch.randn(mod.out_features, rank, generator=g) * 0.1
    return sd


@pytest.mark.parametrize("preset", ["tiny", "tiny_v2"])
def test_lora_merge(preset):
    """LoRA folded into the weights (f_lite/lora.py; the reference keeps peft modules, pt.py:107-135):
    W <- bf16(W + B @ A) for exactly the adapted Linears (qkv, cross q, context_kv, both proj), nothing else."""
    from f_lite.lora import merge_lora_

    m = _filled(DiT if preset == "tiny" else DiTv2, preset).to(torch.bfloat16)
    before = {k: v.clone() for k, v in m.state_dict().items()}
    lsd = _lora_sd(m)
    mods = {k.rsplit(".lora_", 1)[0] for k in lsd}
    assert any(k.endswith("self_attn.qkv") for k in mods) and any(k.endswith("cross_attn.q") for k in mods)
    assert not any(k.endswith(("context_proj", "final_proj", "gate_proj")) for k in mods)
    assert merge_lora_(m, lsd, target_modules=["qkv", "q", "context_kv", "proj"], rank=4) == len(mods)
    for k, v in m.state_dict().items():
        mod = k[: -len(".weight")] if k.endswith(".weight") else None
        if mod in mods:
            want = (before[k].float() + lsd[f"{mod}.lora_B.weight"] @ lsd[f"{mod}.lora_A.weight"]).bfloat16()
            assert torch.equal(v, want), k
        else:
            assert torch.equal(v, before[k]), k


def test_lora_pt_loader_and_dit_methods(tmp_path):
    """load_f_lite_pt(lora_path=...) (pt.py:107-135) and DiT.load_lora_weights / save_lora_weights
    (model.py:487-495) give the same merged weights; a wrong rank or a half-paired adapter raises, an untargeted one
    is skipped."""
    from f_lite.lora import merge_lora_
    from f_lite.pt import load_f_lite_pt

    m = _filled(DiT, "tiny")
    torch.save(m.state_dict(), tmp_path / "model.pt")
    lsd = _lora_sd(m, rank=8)
    torch.save(lsd, tmp_path / "lora.pt")
    kw = dict(width=512, cross_attn_input_size=128, train_bias_and_rms=True)
    pipe = load_f_lite_pt(tmp_path / "model.pt", "cpu", dtype="bfloat16", lora_path=tmp_path / "lora.pt",
                          lora_rank=8, **kw)
    ref = m.to(torch.bfloat16)
    merge_lora_(ref, lsd)
    got = pipe.dit_model.state_dict()
    assert all(torch.equal(got[k], v) for k, v in ref.state_dict().items())
    # the DiT methods: save the loaded adapter, load it into a fresh copy of the base weights
    pipe.dit_model.save_lora_weights(tmp_path)
    fresh = load_f_lite_pt(tmp_path / "model.pt", "cpu", dtype="bfloat16", **kw).dit_model
    fresh.load_lora_weights(tmp_path)
    assert all(torch.equal(fresh.state_dict()[k], v) for k, v in got.items())
    with pytest.raises(ValueError):  # lora_rank disagrees with the file (peft would refuse the shapes)
        load_f_lite_pt(tmp_path / "model.pt", "cpu", lora_path=tmp_path / "lora.pt", lora_rank=4, **kw)
    # an adapter on a module outside lora_target_modules is skipped with a warning (peft's strict=False load)
    only_qkv = load_f_lite_pt(tmp_path / "model.pt", "cpu", dtype="bfloat16", lora_path=tmp_path / "lora.pt",
                              lora_rank=8, lora_target_modules="qkv", **kw).dit_model
    base = load_f_lite_pt(tmp_path / "model.pt", "cpu", dtype="bfloat16", **kw).dit_model.state_dict()
    for k, v in only_qkv.state_dict().items():
        assert torch.equal(v, got[k] if k.endswith("self_attn.qkv.weight") else base[k]), k
    half = {k: v for k, v in lsd.items() if not k.startswith("blocks.0.self_attn.qkv.lora_B")}
    assert len(half) == len(lsd) - 1
    with pytest.raises(KeyError):
        merge_lora_(fresh, half)


def test_lora_load_replaces_like_peft(tmp_path):
    """loading an adapter REPLACES the merged one per module, as set_peft_model_state_dict does for
    peft's one adapter (model.py:492-495): the same file twice leaves the weights bit-identical, a second adapter
    does not stack on the first, modules the second file omits keep the first adapter, and save_lora_weights
    writes the union (latest per module)."""
    from f_lite.lora import merge_lora_

    m = _filled(DiT, "tiny").to(torch.bfloat16)
    base = {k: v.clone() for k, v in m.state_dict().items()}
    a1 = _lora_sd(m, rank=4, seed=1)
    torch.save(a1, tmp_path / "lora_weights.pt")
    m.load_lora_weights(tmp_path)
    once = {k: v.clone() for k, v in m.state_dict().items()}
    m.load_lora_weights(tmp_path)
    assert all(torch.equal(m.state_dict()[k], v) for k, v in once.items())
    # a second adapter on the qkv modules only: qkv = base + B2 A2, the rest keeps adapter 1
    a2 = _lora_sd(m, targets=("qkv",), rank=4, seed=2)
    merge_lora_(m, a2)
    for k, v in m.state_dict().items():
        mod = k[: -len(".weight")]
        if f"{mod}.lora_A.weight" in a2:
            want = (base[k].float() + a2[f"{mod}.lora_B.weight"] @ a2[f"{mod}.lora_A.weight"]).bfloat16()
            assert torch.equal(v, want), k
        else:
            assert torch.equal(v, once[k]), k
    m.save_lora_weights(tmp_path)
    saved = torch.load(tmp_path / "lora_weights.pt", weights_only=True)
    assert set(saved) == set(a1)
    for k, v in saved.items():
        assert torch.equal(v, (a2 if k in a2 else a1)[k]), k
    # a weight overwritten since the merge (load_state_dict) becomes the new base
    m.load_state_dict(base)
    merge_lora_(m, a2)
    k = next(k for k in a2 if k.endswith("lora_A.weight")).replace(".lora_A.weight", "")
    want = (base[k + ".weight"].float() + a2[k + ".lora_B.weight"] @ a2[k + ".lora_A.weight"]).bfloat16()
    assert torch.equal(m.state_dict()[k + ".weight"], want)
    # "still holds our merge" is decided by content. A move to new storage after the merge (same bits,
    # new pointer; .to(device) on a GPU) still restores the kept base, so reloading stays bit-identical ...
    m.to(torch.float32).to(torch.bfloat16)
    merge_lora_(m, a2)
    assert torch.equal(m.state_dict()[k + ".weight"], want)
    # ... and a write through .data (no version bump) becomes the new base instead of being silently undone
    W = dict(m.named_modules())[k].weight
    W.data.copy_(base[k + ".weight"] * 2)
    merge_lora_(m, a2)
    want2 = ((base[k + ".weight"] * 2).float() + a2[k + ".lora_B.weight"] @ a2[k + ".lora_A.weight"]).bfloat16()
    assert torch.equal(m.state_dict()[k + ".weight"], want2)


def test_weights_updated_bumps_generation():
    m = _filled(DiT, "tiny")
    g = m._wgen
    assert m.weights_updated() is m and m._wgen == g + 1
    from f_lite.vae import AutoencoderKL

    v = AutoencoderKL(block_out_channels=(32, 32), layers_per_block=1, norm_num_groups=8)
    g = v._wgen
    v.weights_updated()
    assert v._wgen == g + 1


def test_generate_signature_matches_reference():
    """generate_images keeps the reference's parameters and defaults (generate.py:13-25)."""
    from f_lite.generate import build_parser, generate_images

    sig = inspect.signature(generate_images)
    ref = dict(prompt=inspect.Parameter.empty, output_file=inspect.Parameter.empty, model="Freepik/F-Lite",
               negative_prompt=None, seed=0, guidance_scale=6, steps=30, width=1344, height=896, cpu_offload=True,
               device=None, num_images=1)
    for k, v in ref.items():
        assert sig.parameters[k].default == v, k
    args = build_parser().parse_args(["--prompt", "a cat", "--output_file", "o.png"])
    for k, v in ref.items():
        if v is not inspect.Parameter.empty:
            assert getattr(args, k) == v, k


def test_generate_output_naming():
    from f_lite.generate import output_paths

    assert output_paths("out/img.png", 1) == [Path("out/img.png")]
    assert output_paths("out/img.png", 3) == [Path("out/img.png"), Path("out/img-1.png"), Path("out/img-2.png")]


def test_generate_fails_loudly_without_gpu(tmp_path):
    from f_lite._native import FliteError
    from f_lite.generate import generate_images

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(FliteError):
        generate_images("a cat", str(tmp_path / "x.png"), model="random:tiny")
    with pytest.raises(FliteError):
        generate_images("a cat", str(tmp_path / "x.png"), model="random:tiny", device="cpu")


def test_bench_refuses_world_size_mismatch():
    """bench.py --gpus N must run one rank per GPU: a torchrun world of another size is refused before any GPU
    call (here WORLD_SIZE=1 with --gpus 2)."""
    env = dict(__import__("os").environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2"], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode != 0 and "one rank per GPU" in r.stderr
