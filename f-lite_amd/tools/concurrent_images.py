"""Two images in flight on one GPU: two engines over the SAME weights (each with its own activations, K/V cache
and hipGraph stream), each image's whole 30-step loop + VAE decode on its own stream, so the tail rounds of one
image's kernels overlap the other's. Prints images/s sequential vs concurrent.
Usage: python f-lite_amd/tools/concurrent_images.py [--images 4] [--fp8] [--height 1024 --width 1024]"""
import argparse
import copy
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from f_lite import DiT, FLitePipeline  # noqa: E402
from f_lite import _native as nat  # noqa: E402
from f_lite.model import PRESETS  # noqa: E402
from f_lite.vae import AutoencoderKL  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--images", type=int, default=4)
ap.add_argument("--height", type=int, default=1024)
ap.add_argument("--width", type=int, default=1024)
ap.add_argument("--fp8", action="store_true")
ap.add_argument("--tiling", action="store_true")
args = ap.parse_args()

dev = torch.device("cuda", 0)
cfg = dict(PRESETS["10b"])
model = DiT.random(seed=0, device=dev, **cfg)
vae = AutoencoderKL.random(seed=0, device=dev)
m2, v2 = copy.copy(model), copy.copy(vae)  # same parameter tensors, separate native engines
m2._engine = None
v2._engine = None
if args.fp8:
    model.enable_fp8(True)
    m2.enable_fp8(True)
pipes = [FLitePipeline(model, vae), FLitePipeline(m2, v2)]
if args.tiling:
    for p in pipes:
        p.enable_vae_tiling()
ctx = nat.init_param_(torch.empty(1, 512, 4096, device=dev, dtype=torch.bfloat16), "synthetic.t5_context", seed=1,
                      std=1.0)
lh, lw = args.height // 8, args.width // 8


def lat(i):
    return nat.init_param_(torch.empty(1, 16, lh, lw, device=dev, dtype=torch.bfloat16), f"synthetic.latents.{i}",
                           seed=2, std=1.0)


def run(p, i):
    return p(prompt_embeds=ctx, latents=lat(i), height=args.height, width=args.width, num_inference_steps=30,
             guidance_scale=6.0, output_type="uint8").images


streams = [torch.cuda.Stream(), torch.cuda.Stream()]
for k in range(2):  # warm both engines (graph capture, VAE prepare)
    with torch.cuda.stream(streams[k]):
        ref = run(pipes[k], 100 + k)
torch.cuda.synchronize()

t0 = time.perf_counter()
for i in range(args.images):
    a = run(pipes[0], i)
torch.cuda.synchronize()
seq = args.images / (time.perf_counter() - t0)

outs = {}
t0 = time.perf_counter()
for i in range(0, args.images, 2):
    for k in range(2):
        with torch.cuda.stream(streams[k]):
            outs[i + k] = run(pipes[k], i + k)
torch.cuda.synchronize()
conc = args.images / (time.perf_counter() - t0)
same = torch.equal(outs[args.images - 2], run(pipes[0], args.images - 2))
torch.cuda.synchronize()
print(f"{args.height}x{args.width} {'fp8' if args.fp8 else 'bf16'}: sequential {seq:.4f} img/s, two streams "
      f"{conc:.4f} img/s ({100 * (conc / seq - 1):+.1f} %); concurrent image == sequential image: {same}",
      flush=True)
