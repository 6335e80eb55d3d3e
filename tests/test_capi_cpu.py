"""CPU: the C-ABI library builds for gfx950, loads, and exports every entry point include/flite.h declares
(no compute calls: there is no GPU in the build container)."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "flite.h"


def declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(flite_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    import sys

    sys.path.insert(0, str(ROOT / "f-lite_amd"))
    import build_native

    path = build_native.build(verbose=False)
    return ctypes.CDLL(str(path))


def test_header_declares_the_path():
    fns = declared_functions()
    for must in ("flite_gemm_bf16", "flite_attn_varlen_fwd", "flite_rmsnorm_modulate", "flite_rope_qknorm",
                 "flite_dit_forward", "flite_dit_sample", "flite_vae_decode_uint8", "flite_conv3x3_bf16"):
        assert must in fns


def test_every_declared_symbol_is_exported(lib):
    for name in declared_functions():
        assert hasattr(lib, name), name


def test_python_binding_covers_header():
    from f_lite import _native

    assert set(declared_functions()) == set(_native.SIGNATURES)


def test_version_and_error_without_gpu(lib):
    from f_lite import _native

    l = _native.load()
    assert l.flite_version() == 1
    # a call that fails argument validation before touching the device returns an error, never throws
    st = l.flite_dit_create(None, None)
    assert st != 0
    assert b"null" in l.flite_last_error()
