import sys
sys.path.insert(0, "f-lite_amd/tools")
from kbench_attn import run
for lk in (64, 128, 256, 512, 1024, 2048, 4096):
    run(4096, lk, iters=30, split=False)
