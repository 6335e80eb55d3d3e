"""F-Lite sampling path on MI355X (gfx950): drop-in for the reference `f_lite` package
(/root/reference/f_lite/__init__.py:1-5 exports FLitePipeline, FLitePipelineOutput, APGConfig, DiT).

The compute runs in libflite_hip.so (hand-written HIP kernels for gfx950 behind the C ABI of
include/flite.h); this package is the host side mirroring the reference's Python interface.
"""
from .model import DiT
from .pipeline import APGConfig, FLitePipeline, FLitePipelineOutput

__all__ = ["FLitePipeline", "FLitePipelineOutput", "APGConfig", "DiT"]
