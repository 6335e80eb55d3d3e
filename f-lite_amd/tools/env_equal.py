"""Bit-equality of the sampling loop under an environment switch (diagnostic; run on the GPU box):

    python f-lite_amd/tools/env_equal.py VAR=VALUE [--preset 10b --depth 2 --size 256]

runs the same CFG-6 4-step loop (zero negative prompt, hipGraph and eager) in two child processes, with and without
VAR, and reports whether the final latents are bit-identical (e.g. FLITE_CTX_OVERLAP=1: the collapsed rows'
update on a side stream must not change a bit)."""
import argparse
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
CHILD = """
import sys, torch
sys.path[:0] = [{pkg!r}]
from f_lite import DiT, FLitePipeline
from f_lite.model import PRESETS
cfg = dict(PRESETS[{preset!r}], depth={depth})
m = DiT.random(seed=0, device="cuda", **cfg)
if {fp8}:
    m.enable_fp8(True)
g = torch.Generator().manual_seed(6)
hw = {size}
lat = torch.randn(2, 16, hw // 8, hw // 8, generator=g).bfloat16().cuda()
pos = torch.randn(2, 24, cfg["cross_attn_input_size"], generator=g).bfloat16().cuda()
out = {{}}
for graph in (False, True):
    out[graph] = FLitePipeline(m)(prompt_embeds=pos, latents=lat, height=hw, width=hw, num_inference_steps=4,
                                  guidance_scale=6.0, output_type="latent", use_graph=graph).images.float().cpu()
torch.save(out, sys.argv[1])
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("var")
    ap.add_argument("--preset", default="10b")
    ap.add_argument("--depth", type=int, default=2)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--fp8", action="store_true", help="the MXFP8 blocks (DiT.enable_fp8)")
    a = ap.parse_args()
    import torch

    key, val = a.var.split("=", 1)
    script = Path("/tmp/env_equal_child.py")
    script.write_text(CHILD.format(pkg=str(ROOT / "f-lite_amd"), preset=a.preset, depth=a.depth, size=a.size,
                                        fp8=bool(a.fp8)))
    outs = []
    for i, extra in enumerate(({}, {key: val})):
        env = dict(os.environ)
        env.pop(key, None)
        env.update(extra)
        f = Path(f"/tmp/env_equal_{i}.pt")
        r = subprocess.run([sys.executable, str(script), str(f)], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(r.stderr[-2000:])
            sys.exit(1)
        outs.append(torch.load(f, weights_only=True))
    for graph in (False, True):
        eq = torch.equal(outs[0][graph], outs[1][graph])
        print(f"{a.var} {'graph' if graph else 'eager'}: {'bit-identical' if eq else 'DIFFERENT'} "
              f"(max |diff| {(outs[0][graph] - outs[1][graph]).abs().max().item():.3e})", flush=True)
        if not eq:
            sys.exit(2)


if __name__ == "__main__":
    main()
