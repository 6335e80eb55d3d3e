"""TEST INFRASTRUCTURE ONLY -- the CPU oracle for the F-Lite sampling path.

This package restates, on the CPU in PyTorch/numpy, the algorithm of the reference
(sippycoder/f-lite: f_lite/model.py, f_lite/model_v2.py, f_lite/pipeline.py and the diffusers Flux VAE
decoder it calls) so that the MI355X-native path can be checked against it. It is pinned against golden
vectors produced by importing the reference itself in the build container (tests/golden/make_golden.py).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it. The product
(f-lite_amd/f_lite) never imports, calls or links anything from here.
"""
