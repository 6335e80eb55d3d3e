"""ctypes binding of libflite_hip.so (the C ABI in include/flite.h).

This is the ONLY compute path of the package: there is no CPU or PyTorch fallback. If the library is
missing, or a tensor is not on a ROCm device, the call raises.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch

_LIB_PATH = Path(__file__).resolve().parent / "libflite_hip.so"
_lib = None

EPI_STORE_BF16 = 0
EPI_STORE_F32 = 1
EPI_RESID_F32 = 2
EPI_SWIGLU_BF16 = 3
EPI_GEGLU_BF16 = 6
EPI_RESID_BF16 = 7

_vp = ctypes.c_void_p
_i = ctypes.c_int
_l = ctypes.c_long
_f = ctypes.c_float
_d = ctypes.c_double
_cp = ctypes.c_char_p
_ull = ctypes.c_ulonglong


class DitConfig(ctypes.Structure):
    """flite_dit_config (include/flite.h)."""

    _fields_ = [
        ("in_channels", _i),
        ("patch_size", _i),
        ("hidden_size", _i),
        ("depth", _i),
        ("num_heads", _i),
        ("mlp_hidden", _i),
        ("cross_attn_input_size", _i),
        ("train_bias_and_rms", _i),
        ("per_block_adaln", _i),
        ("n_register_tokens", _i),
        ("rope_base", _f),
        ("bf16_timestep_quant", _i),
        ("bf16_rope_tables", _i),
        ("use_rope", _i),
    ]


# name -> (restype, argtypes); every symbol declared in include/flite.h
SIGNATURES = {
    "flite_last_error": (_cp, []),
    "flite_version": (_i, []),
    "flite_gemm_bf16": (_i, [_vp, _i, _i, _i, _vp, _l, _vp, _l, _vp, _vp, _i, _vp, _l, _vp, _l, _i]),
    "flite_gemm_workspace_bytes": (_l, []),
    "flite_gemm_bf16_ws": (_i, [_vp, _i, _i, _i, _vp, _l, _vp, _l, _vp, _vp, _i, _vp, _l, _vp, _l, _i, _vp]),
    "flite_attn_varlen_fwd": (_i, [_vp, _vp, _vp, _vp, _vp, _l, _l, _l, _l, _l, _vp, _vp, _i, _i, _i, _i, _f, _f]),
    "flite_attn_workspace_bytes": (_l, [_i, _i]),
    "flite_attn_workspace_bytes_for": (_l, [_i, _i, _i, _i]),
    "flite_attn_set_q256": (_i, [_i]),
    "flite_attn_varlen_fwd_ws": (_i, [_vp, _vp, _vp, _vp, _vp, _l, _l, _l, _l, _l, _vp, _vp, _i, _i, _i, _i, _i, _f,
                                      _f, _vp, _l]),
    "flite_rmsnorm_modulate": (_i, [_vp, _vp, _i, _l, _vp, _l, _vp, _vp, _vp, _l, _l, _l, _i, _f]),
    "flite_rope_qknorm": (_i, [_vp, _vp, _l, _l, _i, _i, _vp, _vp, _l, _f]),
    "flite_gather_rows": (_i, [_vp, _vp, _vp, _vp, _l, _i]),
    "flite_t5_attention": (_i, [_vp, _vp, _l, _vp, _l, _vp, _l, _vp, _l, _vp, _vp, _vp, _i, _i, _i]),
    "flite_embed_rows_f32": (_i, [_vp, _vp, _vp, _vp, _l, _i, _l]),
    "flite_rope_tables": (_i, [_vp, _vp, _vp, _i, _i, _i, _f, _i]),
    "flite_timestep_embedding": (_i, [_vp, _vp, _vp, _i, _i, _i]),
    "flite_init_param": (_i, [_vp, _vp, _i, _l, _cp, _ull, _d, _i]),
    "flite_dit_create": (_i, [ctypes.POINTER(DitConfig), ctypes.POINTER(_vp)]),
    "flite_dit_destroy": (_i, [_vp]),
    "flite_dit_bind": (_i, [_vp, _cp, _vp, _l]),
    "flite_dit_prepare": (_i, [_vp, _i, _i, _i, _i, _i]),
    "flite_dit_set_context": (_i, [_vp, _vp, _vp, ctypes.POINTER(_i), _i]),
    "flite_dit_set_timesteps": (_i, [_vp, _vp, _vp, _i, _i]),
    "flite_dit_forward": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _vp, _i]),
    "flite_dit_sample": (_i, [_vp, _vp, _vp, _i, _i, ctypes.POINTER(_f), ctypes.POINTER(_f), _f, _i, _i, _f, _i]),
    "flite_cfg_euler": (_i, [_vp, _vp, _vp, _vp, _l, _f, _f, _i]),
    "flite_apg_sums": (_i, [_vp, _vp, _vp, _l, _f, _i, _vp]),
    "flite_apg_sums_dev": (_i, [_vp, _vp, _vp, _l, _i, _vp]),
    "flite_apg_euler_dev": (_i, [_vp, _vp, _vp, _vp, _l, _f, _f, _l, _vp, _f]),
    "flite_apg_euler": (_i, [_vp, _vp, _vp, _vp, _l, _f, _f, _f, _f]),
    "flite_conv3x3_pack_weight":(_i, [_vp, _vp, _vp, _i, _i, _i]),
    "flite_conv3x3_bf16": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _i]),
    "flite_group_norm": (_i, [_vp, _vp, _vp, _l, _i, _i, _vp, _vp, _f, _i, _vp]),
    "flite_vae_create": (_i, [_vp, ctypes.POINTER(_vp)]),
    "flite_vae_destroy": (_i, [_vp]),
    "flite_vae_bind": (_i, [_vp, _cp, _vp, _l]),
    "flite_vae_prepare": (_i, [_vp, _i, _i]),
    "flite_vae_enable_fp8_weights": (_i, [_vp, _i]),
    "flite_vae_decode_uint8": (_i, [_vp, _vp, _vp, _i, _vp, _f, _f]),
    "flite_vae_prepare_tiled": (_i, [_vp, _i, _i, _i, _i, _f]),
    "flite_vae_decode_tiled_uint8": (_i, [_vp, _vp, _vp, _i, _vp, _f, _f]),
    "flite_quant_fp8_rows": (_i, [_vp, _vp, _l, _l, _i, _vp, _l, _vp, _l]),
    "flite_quant_fp8_gateup": (_i, [_vp, _vp, _vp, _l, _i, _i, _vp, _vp]),
    "flite_gemm_fp8": (_i, [_vp, _i, _i, _i, _vp, _l, _vp, _l, _vp, _l, _vp, _l, _vp, _i, _vp, _l, _vp, _l, _vp, _l,
                            _i]),
    "flite_gemm_fp8_ws": (_i, [_vp, _i, _i, _i, _vp, _l, _vp, _l, _vp, _l, _vp, _l, _vp, _i, _vp, _l, _vp, _l, _vp,
                               _l, _i, _vp]),
    "flite_rmsnorm_modulate_fp8": (_i, [_vp, _vp, _l, _vp, _l, _vp, _l, _vp, _vp, _vp, _l, _l, _l, _i, _f]),
    "flite_dit_enable_fp8": (_i, [_vp, _vp, _i]),
    "flite_dit_set_fp8_bf16_blocks": (_i, [_vp, _vp, _i]),
    "flite_dit_set_fp8_gemm_classes": (_i, [_vp, _i]),
    "flite_dit_set_fp8_block_classes": (_i, [_vp, _vp, _i]),
    "flite_dit_set_residual_bf16": (_i, [_vp, _i]),
    "flite_dit_residual_bf16": (_i, [_vp]),
    "flite_dit_weights_updated": (_i, [_vp, _vp]),
    "flite_vae_weights_updated": (_i, [_vp]),
    "flite_dit_set_sequence_parallel": (_i, [_vp, _i, _i, _vp, _vp]),
    "flite_dit_sp_buffer_bytes": (_i, [_vp, ctypes.POINTER(_l), ctypes.POINTER(_l)]),
    "flite_dit_sp_bind_buffers": (_i, [_vp, _vp, _vp, _vp, _vp]),
    "flite_dit_sp_set_ring": (_i, [_vp, _i]),
    "flite_dit_set_probe": (_i, [_vp, _i, _i]),
    "flite_dit_read_probe": (_i, [_vp, ctypes.POINTER(_f), _i, ctypes.POINTER(_i)]),
}

EPI8_STORE_BF16 = 0
EPI8_RESID_F32 = 2
EPI8_RESID_BF16 = 7
EPI8_SWIGLU_FP8 = 4
EPI8_SWIGLU_BF16 = 6

PROBE_GEMM_GATEUP = 0
PROBE_ATTN_SELF = 1
PROBE_GEMM_DOWN = 2
PROBE_GEMM_QKV = 3
PROBE_STEP = 4


class FliteError(RuntimeError):
    pass


def lib_path() -> Path:
    return Path(os.environ.get("FLITE_LIB", str(_LIB_PATH)))


def load():
    """Load libflite_hip.so and bind every exported entry point. Raises if the library is absent."""
    global _lib
    if _lib is not None:
        return _lib
    path = lib_path()
    if not path.exists():
        raise FliteError(
            f"libflite_hip.so not found at {path}; build it with `python f-lite_amd/build_native.py` "
            "(there is no CPU fallback)"
        )
    lib = ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(status: int, what: str):
    if status != 0:
        msg = load().flite_last_error().decode(errors="replace")
        raise FliteError(f"{what} failed ({status}): {msg}")


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_gpu(t: torch.Tensor, name: str, dtype=None, contiguous=True):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        dev = t.device if isinstance(t, torch.Tensor) else type(t)
        raise FliteError(f"{name}: tensor must live on a ROCm device (got {dev}); there is no CPU fallback")
    if dtype is not None and t.dtype != dtype:
        raise FliteError(f"{name}: expected {dtype}, got {t.dtype}")
    if contiguous and not t.is_contiguous():
        raise FliteError(f"{name}: tensor must be contiguous")
    return t.data_ptr()


def _ptr(t):
    return None if t is None else t.data_ptr()


# ------------------------------------------------------------------------------------------------
# kernel-level operators
# ------------------------------------------------------------------------------------------------
def gemm_workspace(device) -> torch.Tensor:
    """Zero-filled stream-K workspace for gemm(..., workspace=) on `device` (flite_gemm_workspace_bytes)."""
    n = int(load().flite_gemm_workspace_bytes())
    return torch.zeros(max(n, 16), dtype=torch.uint8, device=device)


def gemm(a: torch.Tensor, w: torch.Tensor, bias=None, *, out=None, epilogue=EPI_STORE_BF16, w2=None,
         gate=None, gate_seg_stride=0, rows_per_seg=1, workspace=None) -> torch.Tensor:
    """C = a . w^T (+bias) with the selected fused epilogue. a:[M,K] bf16, w:[N,K] bf16 (nn.Linear layout).
    `workspace` (gemm_workspace) enables the stream-K split of a partial last wave of tiles."""
    lib = load()
    M, K = a.shape
    N = w.shape[0]
    if a.stride(1) != 1 or w.stride(1) != 1:
        raise FliteError("gemm: operands must be K-contiguous")
    if epilogue in (EPI_SWIGLU_BF16, EPI_GEGLU_BF16):
        if w2 is None or w2.shape != w.shape:
            raise FliteError("gemm(swiglu/geglu): w2 must match w")
        Nv = 2 * N
        if out is None:
            out = torch.empty(M, N, device=a.device, dtype=torch.bfloat16)
    else:
        Nv = N
        if out is None:
            dt = torch.bfloat16 if epilogue == EPI_STORE_BF16 else torch.float32
            out = torch.empty(M, N, device=a.device, dtype=dt)
    require_gpu(a, "a", torch.bfloat16, contiguous=False)
    require_gpu(w, "w", torch.bfloat16, contiguous=False)
    require_gpu(out, "out", contiguous=False)
    if bias is not None:
        require_gpu(bias, "bias", torch.bfloat16)
    args = (stream_ptr(a.device), M, Nv, K, a.data_ptr(), a.stride(0), w.data_ptr(), w.stride(0), _ptr(w2),
            _ptr(bias), epilogue, out.data_ptr(), out.stride(0), _ptr(gate), gate_seg_stride, rows_per_seg)
    if workspace is not None:
        require_gpu(workspace, "workspace", contiguous=True)
        check(lib.flite_gemm_bf16_ws(*args, workspace.data_ptr()), "flite_gemm_bf16_ws")
    else:
        check(lib.flite_gemm_bf16(*args), "flite_gemm_bf16")
    return out


# GEMM classes of the fp8 policy (include/flite.h FLITE_FP8_*)
FP8_CLASSES = {"qkv": 1, "proj": 2, "cross_q": 4, "cross_proj": 8, "gate_up": 16, "down": 32}


def fp8_class_mask(classes) -> int:
    """An int mask, or an iterable of FP8_CLASSES names ("all" = every class). A bool is refused (True is not a
    class set), and so is an empty name list: it would run every fp8 block in bf16 while the caller asked for fp8
    (pass the int 0 to mean exactly that)."""
    if classes is None:
        return 63
    if isinstance(classes, bool):
        raise FliteError("fp8 GEMM classes: pass class names or an int mask, not a bool")
    if isinstance(classes, int):
        if not 0 <= classes <= 63:
            raise FliteError(f"fp8 GEMM class mask {classes} outside 0..63")
        return classes
    if isinstance(classes, str):
        classes = [c for c in classes.split(",") if c.strip()]
    m = 0
    for c in classes:
        c = c.strip()
        if c == "all":
            m |= 63
        elif c in FP8_CLASSES:
            m |= FP8_CLASSES[c]
        else:
            raise FliteError(f"unknown fp8 GEMM class {c!r} (one of {sorted(FP8_CLASSES)} or 'all')")
    if m == 0:
        raise FliteError("fp8 GEMM classes: empty class set (every fp8 block would run bf16); pass 0 to mean that")
    return m


def fp8_block_masks(spec: str, depth: int, default=63) -> "list[int]":
    """Per-block class masks from a policy string (bench.py --fp8-block-classes): ';'-separated "LO-HI:CLASSES" or
    "I:CLASSES" items, CLASSES = '+'-separated FP8_CLASSES names, 'all', 'none' or an int mask; blocks no item
    names get `default`. E.g. "0-3:none;4-7:gate_up+qkv" keeps blocks 0-3 bf16 and runs only gate/up and qkv
    MXFP8 in blocks 4-7."""
    masks = [int(default)] * depth
    for item in (x.strip() for x in spec.split(";")):
        if not item:
            continue
        rng, _, cls = item.partition(":")
        if not cls:
            raise FliteError(f"fp8 block policy item {item!r}: expected BLOCKS:CLASSES")
        lo, _, hi = rng.partition("-")
        lo, hi = int(lo), int(hi or lo)
        if not 0 <= lo <= hi < depth:
            raise FliteError(f"fp8 block policy item {item!r}: blocks outside 0..{depth - 1}")
        cls = cls.strip()
        m = 0 if cls == "none" else int(cls) if cls.isdigit() else fp8_class_mask(cls.split("+"))
        if not 0 <= m <= 63:
            raise FliteError(f"fp8 block policy item {item!r}: mask outside 0..63")
        masks[lo:hi + 1] = [m] * (hi - lo + 1)
    return masks


def attn_workspace(device, batch, num_heads, max_q=0, max_k=0):
    """Zero-filled split workspace for attn_varlen(..., workspace=) (flite_attn_workspace_bytes); None when a
    (batch, num_heads) launch gains nothing from it. With max_q / max_k (flite_attn_workspace_bytes_for) it also
    holds the 256-row kernel's split plan, which launches given max_k >= 1024 then take."""
    if max_q or max_k:
        n = int(load().flite_attn_workspace_bytes_for(batch, num_heads, max_q, max_k))
    else:
        n = int(load().flite_attn_workspace_bytes(batch, num_heads))
    return torch.zeros(n, dtype=torch.uint8, device=device) if n > 0 else None


def attn_set_q256(mode):
    """Route policy for long bounded launches (process-wide; include/flite.h flite_attn_set_q256): True / 1 always
    the 256-query-row kernel, False / 0 never, 2 (the default) where its plan is predicted faster."""
    check(load().flite_attn_set_q256(int(mode)), "flite_attn_set_q256")


def attn_varlen(q, k, v, cu_q, cu_k, max_q, scale, out=None, max_score=0.0, workspace=None, max_k=0):
    """flash_attn_varlen_func replacement: q [Lq, h, 256], k/v [Lk, h, 256] (row-major, any row stride).
    `workspace` (attn_workspace) lets a bounded (max_score > 0) launch split its partial q-tiles by keys."""
    lib = load()
    Lq, H, D = q.shape
    if out is None:
        out = torch.empty(Lq, H, D, device=q.device, dtype=torch.bfloat16)
    for t, n in ((q, "q"), (k, "k"), (v, "v"), (out, "out")):
        require_gpu(t, n, torch.bfloat16, contiguous=False)
        if t.stride(2) != 1 or t.stride(1) != D:
            raise FliteError(f"attn: {n} must be [L, h, d] with contiguous heads")
    require_gpu(cu_q, "cu_q", torch.int32)
    require_gpu(cu_k, "cu_k", torch.int32)
    args = (stream_ptr(q.device), q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), q.stride(0),
            k.stride(0), v.stride(0), out.stride(0), D, cu_q.data_ptr(), cu_k.data_ptr(), cu_q.numel() - 1, H, D,
            max_q)
    if workspace is not None:
        require_gpu(workspace, "workspace", contiguous=True)
        check(lib.flite_attn_varlen_fwd_ws(*args, max_k, scale, max_score, workspace.data_ptr(), workspace.numel()),
              "flite_attn_varlen_fwd_ws")
    else:
        check(lib.flite_attn_varlen_fwd(*args, scale, max_score), "flite_attn_varlen_fwd")
    return out


def rmsnorm_modulate(x, w=None, shift=None, scale=None, seg_rows=0, eps=1e-6, out=None):
    lib = load()
    rows, dim = x.shape
    if out is None:
        out = torch.empty(rows, dim, device=x.device, dtype=torch.bfloat16)
    require_gpu(x, "x", contiguous=False)
    st = lib.flite_rmsnorm_modulate(stream_ptr(x.device), x.data_ptr(), int(x.dtype == torch.bfloat16), x.stride(0),
                                    out.data_ptr(), out.stride(0), _ptr(w), _ptr(shift), _ptr(scale),
                                    shift.stride(0) if shift is not None and shift.dim() == 2 else 0, seg_rows, rows,
                                    dim, eps)
    check(st, "flite_rmsnorm_modulate")
    return out


def rope_qknorm_(x, heads, rope_heads, cos=None, sin=None, tokens_per_seq=0, eps=1e-6):
    lib = load()
    require_gpu(x, "x", torch.bfloat16, contiguous=False)
    st = lib.flite_rope_qknorm(stream_ptr(x.device), x.data_ptr(), x.stride(0), x.shape[0], heads, rope_heads,
                               _ptr(cos), _ptr(sin), tokens_per_seq, eps)
    check(st, "flite_rope_qknorm")
    return x


def rope_tables(h, w, n_reg=16, base=10000.0, round_bf16=True, device="cuda"):
    lib = load()
    cos = torch.empty(n_reg + h * w, 128, device=device, dtype=torch.float32)
    sin = torch.empty_like(cos)
    check(lib.flite_rope_tables(stream_ptr(cos.device), cos.data_ptr(), sin.data_ptr(), h, w, n_reg, base,
                                int(round_bf16)), "flite_rope_tables")
    return cos, sin


def timestep_embedding(t, dim, quantize):
    lib = load()
    require_gpu(t, "t", torch.float32)
    emb = torch.empty(t.numel(), dim, device=t.device, dtype=torch.bfloat16)
    check(lib.flite_timestep_embedding(stream_ptr(t.device), t.data_ptr(), emb.data_ptr(), t.numel(), dim,
                                       int(quantize)), "flite_timestep_embedding")
    return emb


def init_param_(t: torch.Tensor, name: str, seed: int = 0, std: float = 0.02, ones: bool = False):
    """Fill t in place with the deterministic generator (bit-identical to oracle/weights.py)."""
    lib = load()
    require_gpu(t, name)
    if t.dtype not in (torch.bfloat16, torch.float32):
        raise FliteError("init_param: bf16 or fp32 only")
    check(lib.flite_init_param(stream_ptr(t.device), t.data_ptr(), int(t.dtype == torch.bfloat16), t.numel(),
                               name.encode(), seed, std, int(ones)), "flite_init_param")
    return t


def cfg_euler_(acc, uncond, cond, guidance, dt, use_cfg=True):
    """acc += dt * (u + g (c - u)) in place on fp32 NCHW tensors (pipeline.py:290,296-297); cond only when
    use_cfg is False."""
    require_gpu(acc, "acc", torch.float32)
    require_gpu(cond, "cond", torch.float32)
    if cond.shape != acc.shape:
        raise FliteError(f"cfg_euler: cond {tuple(cond.shape)} does not match acc {tuple(acc.shape)}")
    u_ptr = None
    if use_cfg:
        require_gpu(uncond, "uncond", torch.float32)
        if uncond.shape != acc.shape:
            raise FliteError(f"cfg_euler: uncond {tuple(uncond.shape)} does not match acc {tuple(acc.shape)}")
        u_ptr = uncond.data_ptr()
    check(load().flite_cfg_euler(stream_ptr(acc.device), u_ptr, cond.data_ptr(), acc.data_ptr(), acc.numel(),
                                 float(guidance), float(dt), int(use_cfg)), "flite_cfg_euler")
    return acc


def apg_sums(uncond, cond, k=0.0, phase=0, out=None):
    """APG's batch-global reductions on fp32 NCHW branch outputs (include/flite.h flite_apg_sums): phase 0 ->
    [sum c (c - u), sum c^2], phase 1 -> [sum o, sum o^2] with o = (c - u) - k c. A 2-float device tensor."""
    require_gpu(uncond, "uncond", torch.float32)
    require_gpu(cond, "cond", torch.float32)
    if uncond.shape != cond.shape:
        raise FliteError(f"apg_sums: uncond {tuple(uncond.shape)} and cond {tuple(cond.shape)} differ")
    out = torch.empty(2, device=cond.device, dtype=torch.float32) if out is None else out
    check(load().flite_apg_sums(stream_ptr(cond.device), uncond.data_ptr(), cond.data_ptr(), cond.numel(), float(k),
                                int(phase), out.data_ptr()), "flite_apg_sums")
    return out


def apg_euler_(acc, uncond, cond, guidance, k, orth_scale, dt):
    """acc += dt * (c + (g - 1) * orth_scale * ((c - u) - k c)) in place (pipeline.py:285-286,296)."""
    for t, n in ((acc, "acc"), (uncond, "uncond"), (cond, "cond")):
        require_gpu(t, n, torch.float32)
        if t.shape != acc.shape:
            raise FliteError(f"apg_euler: {n} {tuple(t.shape)} does not match acc {tuple(acc.shape)}")
    check(load().flite_apg_euler(stream_ptr(acc.device), uncond.data_ptr(), cond.data_ptr(), acc.data_ptr(),
                                 acc.numel(), float(guidance), float(k), float(orth_scale), float(dt)),
          "flite_apg_euler")
    return acc


def apg_sums_dev(uncond, cond, phase, ws):
    """flite_apg_sums_dev: phase 0 -> ws[0:2] = [sum c (c - u), sum c^2]; phase 1 (k from ws[0:2], on the device) ->
    ws[2:4] = [sum o, sum o^2]. `ws` is a 4-float device tensor; nothing returns to the host."""
    require_gpu(uncond, "uncond", torch.float32)
    require_gpu(cond, "cond", torch.float32)
    require_gpu(ws, "ws", torch.float32)
    if uncond.shape != cond.shape or ws.numel() < 4:
        raise FliteError("apg_sums_dev: uncond / cond shapes differ, or ws has fewer than 4 floats")
    check(load().flite_apg_sums_dev(stream_ptr(cond.device), uncond.data_ptr(), cond.data_ptr(), cond.numel(),
                                    int(phase), ws.data_ptr()), "flite_apg_sums_dev")
    return ws


def apg_euler_dev_(acc, uncond, cond, guidance, threshold, n_total, ws, dt):
    """flite_apg_euler_dev: the APG + Euler update with k and the orthogonal scale derived from ws on the device."""
    for t, n in ((acc, "acc"), (uncond, "uncond"), (cond, "cond")):
        require_gpu(t, n, torch.float32)
        if t.shape != acc.shape:
            raise FliteError(f"apg_euler_dev: {n} {tuple(t.shape)} does not match acc {tuple(acc.shape)}")
    require_gpu(ws, "ws", torch.float32)
    check(load().flite_apg_euler_dev(stream_ptr(acc.device), uncond.data_ptr(), cond.data_ptr(), acc.data_ptr(),
                                     acc.numel(), float(guidance), float(threshold), int(n_total), ws.data_ptr(),
                                     float(dt)), "flite_apg_euler_dev")
    return acc


# ------------------------------------------------------------------------------------------------
# MXFP8 (include/flite.h: e4m3 elements, one E8M0 scale per 32 K elements, scales [K/128][rows_pad][4])
# ------------------------------------------------------------------------------------------------
def mx_rows_pad(rows: int) -> int:
    return (rows + 255) // 256 * 256


def quant_fp8_rows(x: torch.Tensor, rows_pad=None):
    """bf16 [rows, K] -> (fp8 bytes uint8 [rows, K], scales uint8 [K/128, rows_pad, 4])."""
    require_gpu(x, "x", torch.bfloat16, contiguous=False)
    rows, K = x.shape
    rp = rows_pad or mx_rows_pad(rows)
    q = torch.empty(rows, K, device=x.device, dtype=torch.uint8)
    sc = torch.zeros(K // 128, rp, 4, device=x.device, dtype=torch.uint8)
    check(load().flite_quant_fp8_rows(stream_ptr(x.device), x.data_ptr(), x.stride(0), rows, K, q.data_ptr(), K,
                                      sc.data_ptr(), rp), "flite_quant_fp8_rows")
    return q, sc


def quant_fp8_gateup(gate: torch.Tensor, up: torch.Tensor):
    """gate/up [F, K] bf16 -> (fp8 [2F, K] interleaved in 16-row sub-tiles, scales [K/128, 2F, 4])."""
    F, K = gate.shape
    q = torch.empty(2 * F, K, device=gate.device, dtype=torch.uint8)
    sc = torch.zeros(K // 128, 2 * F, 4, device=gate.device, dtype=torch.uint8)
    check(load().flite_quant_fp8_gateup(stream_ptr(gate.device), gate.data_ptr(), up.data_ptr(), gate.stride(0), F, K,
                                        q.data_ptr(), sc.data_ptr()), "flite_quant_fp8_gateup")
    return q, sc


def gemm_fp8(a8, a_sc, w8, w_sc, bias=None, *, out=None, epilogue=EPI8_STORE_BF16, out_sc=None, gate=None,
             gate_seg_stride=0, rows_per_seg=1, workspace=None):
    """C = dequant(a8) . dequant(w8)^T on the MXFP8 MFMA. a8 [M, K] / w8 [N, K] uint8 with scales from
    quant_fp8_rows (w8/w_sc of the SwiGLU epilogue from quant_fp8_gateup, N = 2F). `workspace` (gemm_workspace)
    enables the stream-K split of a partial last wave of tiles."""
    lib = load()
    M, K = a8.shape
    N = w8.shape[0]
    if epilogue == EPI8_SWIGLU_BF16:
        if out is None:
            out = torch.empty(M, N // 2, device=a8.device, dtype=torch.bfloat16)
    elif epilogue == EPI8_SWIGLU_FP8:
        if out is None:
            out = torch.empty(M, N // 2, device=a8.device, dtype=torch.uint8)
        if out_sc is None:
            out_sc = torch.zeros(N // 2 // 128, mx_rows_pad(M), 4, device=a8.device, dtype=torch.uint8)
    elif out is None:
        out = torch.empty(M, N, device=a8.device, dtype=torch.bfloat16 if epilogue == EPI8_STORE_BF16 else torch.float32)
    for t, n in ((a8, "a8"), (a_sc, "a_scales"), (w8, "w8"), (w_sc, "w_scales"), (out, "out")):
        require_gpu(t, n, contiguous=False)
    if workspace is not None:
        require_gpu(workspace, "workspace", contiguous=True)
    check(lib.flite_gemm_fp8_ws(stream_ptr(a8.device), M, N, K, a8.data_ptr(), a8.stride(0), a_sc.data_ptr(),
                                a_sc.shape[1], w8.data_ptr(), w8.stride(0), w_sc.data_ptr(), w_sc.shape[1],
                                _ptr(bias), epilogue, out.data_ptr(), out.stride(0), _ptr(out_sc),
                                out_sc.shape[1] if out_sc is not None else 0, _ptr(gate), gate_seg_stride,
                                rows_per_seg, _ptr(workspace)),
          "flite_gemm_fp8_ws")
    return (out, out_sc) if epilogue == EPI8_SWIGLU_FP8 else out


def rmsnorm_modulate_fp8(x, w=None, shift=None, scale=None, seg_rows=0, eps=1e-6):
    """RMSNorm + modulate of fp32 rows to MXFP8: (y8 uint8 [rows, D], scales [D/128, rows_pad, 4])."""
    require_gpu(x, "x", torch.float32, contiguous=False)
    rows, D = x.shape
    rp = mx_rows_pad(rows)
    y8 = torch.empty(rows, D, device=x.device, dtype=torch.uint8)
    sc = torch.zeros(D // 128, rp, 4, device=x.device, dtype=torch.uint8)
    check(load().flite_rmsnorm_modulate_fp8(stream_ptr(x.device), x.data_ptr(), x.stride(0), y8.data_ptr(), D,
                                            sc.data_ptr(), rp, _ptr(w), _ptr(shift), _ptr(scale),
                                            shift.stride(0) if shift is not None and shift.dim() == 2 else 0,
                                            seg_rows, rows, D, eps), "flite_rmsnorm_modulate_fp8")
    return y8, sc


def gather_rows(src, idx, out=None):
    lib = load()
    n = idx.numel()
    if out is None:
        out = torch.empty(n, src.shape[1], device=src.device, dtype=src.dtype)
    require_gpu(src, "src", torch.bfloat16)
    require_gpu(idx, "idx", torch.int32)
    check(lib.flite_gather_rows(stream_ptr(src.device), src.data_ptr(), out.data_ptr(), idx.data_ptr(), n,
                                src.shape[1]), "flite_gather_rows")
    return out


SP_ALLGATHER_FN = ctypes.CFUNCTYPE(_i, _vp, _i, _vp)  # flite_sp_allgather_fn


class DitEngine:
    """Owner of a native flite_dit handle (the DiT forward and the denoise loop in C++)."""

    def __init__(self, cfg: DitConfig):
        self.lib = load()
        self.h = _vp()
        check(self.lib.flite_dit_create(ctypes.byref(cfg), ctypes.byref(self.h)), "flite_dit_create")
        self.cfg = cfg
        self._sp = None  # (rank, nranks, allgather) with sequence parallelism
        self._sp_cb = None
        self._sp_bufs = None
        self._sp_error = None
        self._device = None

    def set_sequence_parallel(self, rank: int = 0, nranks: int = 1, allgather=None, ring_shift=None):
        """flite_dit_set_sequence_parallel: this engine computes rows [rank*Tl, (rank+1)*Tl) of every sequence.
        allgather(send, recv) must all-gather the uint8 device tensor `send` into `recv` (nranks x, rank order)
        on the current stream (the engine makes its exchange stream current around the call). With
        ring_shift(send, recv) given, the self-attention's keys travel as a ring instead (flite_dit_sp_set_ring):
        ring_shift must send `send` to rank + 1 and receive rank - 1's block into `recv` (same size).
        nranks = 1 switches back to the whole sequence. Call prepare() afterwards."""
        if nranks > 1:
            if allgather is None:
                raise FliteError("sequence parallelism needs an allgather(send, recv) exchange")

            def bufs(which):
                if which < 2:
                    return self._sp_bufs[which], allgather
                k = which - 1  # ring shift k = 1 .. N-1 (flite.h: flite_dit_sp_set_ring)
                (ks, kr), _ = self._sp_bufs
                n = ks.numel()
                slot = lambda i: kr[i * n:(i + 1) * n]  # noqa: E731
                return (ks if k == 1 else slot((k - 2) & 1), slot((k - 1) & 1)), ring_shift

            def cb(user, which, stream):
                try:
                    (send, recv), fn = bufs(which)
                    # the engine names the stream the exchange belongs on (a side stream for the K/V rows,
                    # overlapped with the attention over the rank's own keys)
                    if stream:
                        with torch.cuda.stream(torch.cuda.ExternalStream(stream, device=send.device)):
                            fn(send, recv)
                    else:  # the null stream
                        fn(send, recv)
                    return 0
                except Exception as e:  # reported by the failing flite call
                    self._sp_error = e
                    return 1

            self._sp_cb = SP_ALLGATHER_FN(cb)
            fn = self._sp_cb
            self._sp = (rank, nranks, allgather)
        else:
            fn = ctypes.cast(None, SP_ALLGATHER_FN)
            self._sp, self._sp_cb = None, None
        self._sp_bufs = None
        check(self.lib.flite_dit_set_sequence_parallel(self.h, rank, nranks, fn, None),
              "flite_dit_set_sequence_parallel")
        check(self.lib.flite_dit_sp_set_ring(self.h, int(nranks > 1 and ring_shift is not None)),
              "flite_dit_sp_set_ring")

    def __del__(self):
        try:
            if self.h:
                self.lib.flite_dit_destroy(self.h)
        except Exception:
            pass

    def bind(self, name: str, t: torch.Tensor):
        require_gpu(t, name, torch.bfloat16)
        check(self.lib.flite_dit_bind(self.h, name.encode(), t.data_ptr(), t.numel()), f"bind({name})")

    def prepare(self, batch, lat_h, lat_w, n_ctx, n_t, device=None):
        check(self.lib.flite_dit_prepare(self.h, batch, lat_h, lat_w, n_ctx, n_t), "flite_dit_prepare")
        if self._sp is not None:  # (re)bind the exchange buffers for this shape
            kv, out = _l(0), _l(0)
            check(self.lib.flite_dit_sp_buffer_bytes(self.h, ctypes.byref(kv), ctypes.byref(out)),
                  "flite_dit_sp_buffer_bytes")
            n = self._sp[1]
            dev = device or torch.device("cuda", torch.cuda.current_device())
            mk = lambda b: torch.empty(b, dtype=torch.uint8, device=dev)  # noqa: E731
            self._sp_bufs = ((mk(kv.value), mk(n * kv.value)), (mk(out.value), mk(n * out.value)))
            (ks, kr), (os_, or_) = self._sp_bufs
            check(self.lib.flite_dit_sp_bind_buffers(self.h, ks.data_ptr(), kr.data_ptr(), os_.data_ptr(),
                                                     or_.data_ptr()), "flite_dit_sp_bind_buffers")

    def set_context(self, ctx_packed: torch.Tensor, cu_host):
        require_gpu(ctx_packed, "context", torch.bfloat16)
        arr = (_i * len(cu_host))(*cu_host)
        check(self.lib.flite_dit_set_context(self.h, stream_ptr(ctx_packed.device), ctx_packed.data_ptr(), arr,
                                             len(cu_host) - 1), "flite_dit_set_context")

    def set_timesteps(self, t: torch.Tensor, quantize: bool):
        require_gpu(t, "timesteps", torch.float32)
        check(self.lib.flite_dit_set_timesteps(self.h, stream_ptr(t.device), t.data_ptr(), t.numel(), int(quantize)),
              "flite_dit_set_timesteps")

    def _check_sp(self, status, what):
        """check(), re-raising the exception of a failed sequence-parallel exchange callback if there was one."""
        err, self._sp_error = self._sp_error, None
        if status != 0 and err is not None:
            raise FliteError(f"{what}: sequence-parallel exchange failed: {err!r}") from err
        check(status, what)

    def forward(self, x: torch.Tensor, out: torch.Tensor, t_row0=0, t_row_step=1):
        require_gpu(x, "x")
        require_gpu(out, "out")
        self._check_sp(self.lib.flite_dit_forward(self.h, stream_ptr(x.device), x.data_ptr(),
                                                  int(x.dtype == torch.bfloat16), x.shape[0], t_row0, t_row_step,
                                                  out.data_ptr(), int(out.dtype == torch.bfloat16)),
                       "flite_dit_forward")
        return out

    def enable_fp8(self, on: bool = True, device=None):
        check(self.lib.flite_dit_enable_fp8(self.h, stream_ptr(device), int(bool(on))), "flite_dit_enable_fp8")

    def set_fp8_bf16_blocks(self, blocks=()):
        """Blocks that keep bf16 GEMMs while fp8 mode is on (include/flite.h flite_dit_set_fp8_bf16_blocks)."""
        blocks = [int(b) for b in blocks]
        arr = (ctypes.c_int * max(len(blocks), 1))(*blocks)
        check(self.lib.flite_dit_set_fp8_bf16_blocks(self.h, arr, len(blocks)), "flite_dit_set_fp8_bf16_blocks")

    def set_fp8_gemm_classes(self, mask: int = 63):
        """GEMM classes on MXFP8 in the fp8 blocks (include/flite.h flite_dit_set_fp8_gemm_classes)."""
        check(self.lib.flite_dit_set_fp8_gemm_classes(self.h, int(mask)), "flite_dit_set_fp8_gemm_classes")

    def set_fp8_block_classes(self, masks=()):
        """Per-block MXFP8 class masks (include/flite.h flite_dit_set_fp8_block_classes): one int per block, or
        () to return to set_fp8_gemm_classes' single mask."""
        masks = [int(m) for m in masks]
        arr = (ctypes.c_int * max(len(masks), 1))(*masks)
        check(self.lib.flite_dit_set_fp8_block_classes(self.h, arr, len(masks)), "flite_dit_set_fp8_block_classes")

    def set_residual_bf16(self, on: bool = True):
        """Residual-stream storage bf16 (on) or fp32 (include/flite.h flite_dit_set_residual_bf16)."""
        check(self.lib.flite_dit_set_residual_bf16(self.h, int(bool(on))), "flite_dit_set_residual_bf16")

    def residual_bf16(self) -> bool:
        """True when the residual stream is held in bf16 (include/flite.h flite_dit_residual_bf16)."""
        r = self.lib.flite_dit_residual_bf16(self.h)
        if r < 0:
            check(1, "flite_dit_residual_bf16")
        return bool(r)

    def weights_updated(self, device=None):
        """The bound weights changed in place: remake the engine's derived copies (fp8: requantise)."""
        check(self.lib.flite_dit_weights_updated(self.h, stream_ptr(device)), "flite_dit_weights_updated")

    def set_probe(self, kind: int, max_pairs: int = 4096):
        check(self.lib.flite_dit_set_probe(self.h, kind, max_pairs), "flite_dit_set_probe")

    def read_probe(self, cap: int = 4096):
        buf = (_f * cap)()
        n = _i(0)
        check(self.lib.flite_dit_read_probe(self.h, buf, cap, ctypes.byref(n)), "flite_dit_read_probe")
        return list(buf[: n.value])

    def sample(self, acc: torch.Tensor, n_img, t_list, dt_list, guidance, use_cfg, apg=False, apg_thr=0.03,
               use_graph=True):
        require_gpu(acc, "latents", torch.float32)
        n = len(t_list)
        ta = (_f * n)(*t_list)
        da = (_f * n)(*dt_list)
        self._check_sp(self.lib.flite_dit_sample(self.h, stream_ptr(acc.device), acc.data_ptr(), n_img, n, ta, da,
                                                 float(guidance), int(use_cfg), int(apg), float(apg_thr),
                                                 int(use_graph)), "flite_dit_sample")
        return acc


class VaeConfig(ctypes.Structure):
    """flite_vae_config (include/flite.h)."""

    _fields_ = [
        ("latent_channels", _i),
        ("n_blocks", _i),
        ("block_out_channels", _i * 4),
        ("layers_per_block", _i),
        ("norm_groups", _i),
        ("mid_attention", _i),
    ]


class VaeEngine:
    """Owner of a native flite_vae handle (the Flux VAE decoder + uint8 post-processing)."""

    def __init__(self, config):
        self.lib = load()
        c = VaeConfig()
        c.latent_channels = config.latent_channels
        boc = list(config.block_out_channels)
        c.n_blocks = len(boc)
        if len(boc) != 4:
            raise FliteError("VAE: 4 decoder blocks expected")
        for i, v in enumerate(boc):
            c.block_out_channels[i] = v
        c.layers_per_block = config.layers_per_block
        c.norm_groups = config.norm_num_groups
        c.mid_attention = int(bool(config.mid_block_add_attention))
        self.h = _vp()
        check(self.lib.flite_vae_create(ctypes.byref(c), ctypes.byref(self.h)), "flite_vae_create")

    def __del__(self):
        try:
            if self.h:
                self.lib.flite_vae_destroy(self.h)
        except Exception:
            pass

    def bind(self, name, t):
        require_gpu(t, name, torch.bfloat16)
        check(self.lib.flite_vae_bind(self.h, name.encode(), t.data_ptr(), t.numel()), f"vae bind({name})")

    def prepare(self, h, w):
        check(self.lib.flite_vae_prepare(self.h, h, w), "flite_vae_prepare")

    def enable_fp8_weights(self, on: bool = True):
        """MXFP8 storage of the packed conv weights (expanded to bf16 per conv); takes effect at the next prepare."""
        check(self.lib.flite_vae_enable_fp8_weights(self.h, int(bool(on))), "flite_vae_enable_fp8_weights")

    def weights_updated(self):
        """The bound weights changed in place: re-pack (and, with fp8 storage, requantise) the conv weights."""
        check(self.lib.flite_vae_weights_updated(self.h), "flite_vae_weights_updated")

    def decode_uint8(self, z, img, scaling, shift):
        require_gpu(z, "latents", torch.float32)
        require_gpu(img, "images", torch.uint8)
        check(self.lib.flite_vae_decode_uint8(self.h, stream_ptr(z.device), z.data_ptr(), z.shape[0], img.data_ptr(),
                                              float(scaling), float(shift)), "flite_vae_decode_uint8")
        return img

    def prepare_tiled(self, h, w, tile_latent, tile_sample, overlap):
        check(self.lib.flite_vae_prepare_tiled(self.h, h, w, int(tile_latent), int(tile_sample), float(overlap)),
              "flite_vae_prepare_tiled")

    def decode_tiled_uint8(self, z, img, scaling, shift):
        require_gpu(z, "latents", torch.float32)
        require_gpu(img, "images", torch.uint8)
        check(self.lib.flite_vae_decode_tiled_uint8(self.h, stream_ptr(z.device), z.data_ptr(), z.shape[0],
                                                    img.data_ptr(), float(scaling), float(shift)),
              "flite_vae_decode_tiled_uint8")
        return img


def conv3x3(x_nhwc, weight, bias=None, upsample=False, resid=None, out_f32=False):
    """nn.Conv2d(k=3, pad=1) (+ nearest-2x upsample first) on NHWC bf16 [h, w, cin]; weight [cout, cin, 3, 3]."""
    lib = load()
    h, w, cin = x_nhwc.shape
    cout = weight.shape[0]
    cpad = (weight.shape[1] + 63) // 64 * 64
    if cin != cpad:
        raise FliteError("conv3x3: input channels must be zero-padded to a multiple of 64")
    packed = torch.empty(cout, 9, cpad, device=x_nhwc.device, dtype=torch.bfloat16)
    s = stream_ptr(x_nhwc.device)
    check(lib.flite_conv3x3_pack_weight(s, weight.data_ptr(), packed.data_ptr(), cout, weight.shape[1], cpad),
          "flite_conv3x3_pack_weight")
    H, W = (2 * h, 2 * w) if upsample else (h, w)
    out = torch.empty(H, W, cout, device=x_nhwc.device, dtype=torch.float32 if out_f32 else torch.bfloat16)
    check(lib.flite_conv3x3_bf16(s, x_nhwc.data_ptr(), 1, h, w, cin, int(upsample), packed.data_ptr(), _ptr(bias),
                                 cout, out.data_ptr(), _ptr(resid), int(out_f32)), "flite_conv3x3_bf16")
    return out


GROUP_NORM_WS_DOUBLES = 2 * 64 + 1024 * 64  # include/flite.h FLITE_GROUP_NORM_WS_DOUBLES


def group_norm(x, groups, gamma, beta, eps=1e-6, silu=False):
    lib = load()
    rows, C = x.shape
    y = torch.empty_like(x)
    stats = torch.empty(GROUP_NORM_WS_DOUBLES, device=x.device, dtype=torch.float64)
    check(lib.flite_group_norm(stream_ptr(x.device), x.data_ptr(), y.data_ptr(), rows, C, groups, gamma.data_ptr(),
                               beta.data_ptr(), eps, int(silu), stats.data_ptr()), "flite_group_norm")
    return y
