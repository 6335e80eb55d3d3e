"""Build libflite_hip.so (all HIP kernels + the C ABI) for gfx950, in-tree.

hipcc cross-compiles for gfx950 without a GPU, so this runs in the CPU container as well as on the box.
Objects go to f-lite_amd/build/, the library to f-lite_amd/f_lite/libflite_hip.so (git-ignored, but it
travels to the GPU box with the gpurun snapshot).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build"
LIB = ROOT / "f_lite" / "libflite_hip.so"
INCLUDE = ROOT.parent / "include"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

CFLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-Wall",
    "-Wno-unused-function",
    "-Wno-unused-variable",
    "-Wno-unused-but-set-variable",
    f"-I{INCLUDE}",
    f"-I{CSRC}",
]


# Per-file extra flags. gemm.hip: no SLP vectorisation -- it packs the fp32 epilogue math (RoPE rotation pairs)
# into v_pk_*_f32 with op_sel shuffles, which needs extra register pairs and spilled 262 VGPRs in the fused qkv
# epilogue (packed f32 beside MFMAs is an anti-lever anyway: MI355X guide, per-instruction costs).
# attention_q256.hip: the same, for the softmax row sums of its two query blocks, which SLP paired into one
# v_pk_add_f32 chain inside the PV phase (16 per key tile, each ~13 cycles dearer than a v_add_f32 there).
FILE_FLAGS = {"gemm.hip": ["-fno-slp-vectorize"], "gemm_fp8.hip": ["-fno-slp-vectorize"],
              "attention_q256.hip": ["-fno-slp-vectorize"]}


def _sources():
    return sorted([p for p in CSRC.iterdir() if p.suffix in (".hip", ".cpp")])


def _headers_mtime() -> float:
    hs = list(CSRC.glob("*.h")) + list(INCLUDE.glob("*.h"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


def _compile(src: Path, force: bool) -> Path:
    obj = BUILD / (src.stem + ".o")
    if not force and obj.exists():
        if obj.stat().st_mtime >= max(src.stat().st_mtime, _headers_mtime()):
            return obj
    cmd = [HIPCC, *CFLAGS, *FILE_FLAGS.get(src.name, []), "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, verbose: bool = True) -> Path:
    BUILD.mkdir(exist_ok=True)
    srcs = _sources()
    jobs = min(len(srcs), int(os.environ.get("MAX_JOBS", "8")), 16)
    with cf.ThreadPoolExecutor(max_workers=max(jobs, 1)) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    newest = max(o.stat().st_mtime for o in objs)
    if force or not LIB.exists() or LIB.stat().st_mtime < newest:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(LIB), *map(str, objs),
               "-L/opt/rocm/lib", "-lrocprofiler-sdk-roctx", "-Wl,-rpath,/opt/rocm/lib"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"[flite] built {LIB} ({len(objs)} objects)")
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
