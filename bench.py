#!/usr/bin/env python
"""F-Lite sampling-path benchmark on MI355X (BASELINE.json metric).

Metric: images/sec @1024x1024, 30 steps, F-Lite-10B bf16 (model_v2 layout), CFG 6, random-init weights and
synthetic T5 context, including the VAE decode to uint8. One "step" of this benchmark = one image generated
per GPU (30 CFG-batched DiT steps + VAE decode), inputs already resident in HBM.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Multi-GPU: one process per GPU, images sharded one per GPU (weak scaling); RCCL is used only to broadcast the
shared text embedding from rank 0 before the loop (no per-step collective). Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "f-lite_amd"))
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

PEAK_BF16 = 256 * 4 * 1024 * 2.4e9  # 2.5166 PF/s dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_FP8 = 2 * PEAK_BF16  # dense fp8 (block-scaled MFMA: 2x the bf16 rate per clock, MI355X_MICROARCH.md)
PEAK_HBM = 8.0e12


def dit_flops(cfg: dict, H: int, W: int, steps: int, ctx_len: int = 512):
    """Algorithmic FLOPs: per sample per step F_step, once per image F_once (context K/V +
    context_proj); 2 FLOP per MAC, GEMM + attention, eltwise excluded."""
    D = cfg["hidden_size"]
    F = int(D * cfg["mlp_ratio"])
    p = cfg["patch_size"]
    C = cfg["in_channels"]
    T = 16 + (H // 8 // p) * (W // 8 // p)
    depth = cfg["depth"]
    cross = [True if cfg["per_block_adaln"] else (i % 4 == 0 or i < 8) for i in range(depth)]
    nc = sum(cross)
    f_step = depth * (2 * T * D * 3 * D + 2 * T * D * D + 2 * T * D * 2 * F + 2 * T * F * D + 4 * T * T * D)
    f_step += nc * (2 * T * D * D + 2 * T * D * D + 4 * T * ctx_len * D)
    f_step += 2 * (T - 16) * C * p * p * D * 2
    f_once = nc * 2 * ctx_len * D * 2 * D + 2 * ctx_len * cfg["cross_attn_input_size"] * D
    return f_step, f_once


def vae_flops(H: int, W: int):
    """Flux VAE decoder conv/attention FLOPs at H x W output (2 FLOP/MAC)."""
    from f_lite.vae import decoder_flops

    return decoder_flops(H, W)


def host_info():
    """nproc, the cores this process may use, the lscpu model name and the NUMA node count."""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity_cores"] = len(os.sched_getaffinity(0))
    except AttributeError:
        info["affinity_cores"] = os.cpu_count()
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                info["cpu_model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        info["numa_nodes"] = len([p for p in Path("/sys/devices/system/node").glob("node[0-9]*")])
    except OSError:
        pass
    info.update(cgroup_cpu_quota())
    info["omp_num_threads"] = os.environ.get("OMP_NUM_THREADS")
    return info


def cgroup_cpu_quota() -> dict:
    """The CPU bandwidth quota of this process's cgroup: v2 `cpu.max` ("<quota> <period>" or "max <period>") or
    v1 `cpu.cfs_quota_us` / `cpu.cfs_period_us`. Returns the raw text and the granted CPUs (None when unlimited)."""
    out = {"cgroup_cpu_max": None, "cgroup_cpus": None}
    try:
        rel = ""
        for line in Path("/proc/self/cgroup").read_text().splitlines():
            if line.startswith("0::"):
                rel = line[3:].strip()
        for f in (Path("/sys/fs/cgroup") / rel.lstrip("/") / "cpu.max", Path("/sys/fs/cgroup/cpu.max")):
            if f.exists():
                raw = f.read_text().strip()
                out["cgroup_cpu_max"] = f"{f}: {raw}"
                q, per = raw.split()[:2]
                if q != "max":
                    out["cgroup_cpus"] = int(q) / int(per)
                return out
        q = Path("/sys/fs/cgroup/cpu/cpu.cfs_quota_us")
        if q.exists():
            quota = int(q.read_text())
            per = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read_text())
            out["cgroup_cpu_max"] = f"cgroup v1 cfs_quota_us {quota} cfs_period_us {per}"
            if quota > 0:
                out["cgroup_cpus"] = quota / per
    except (OSError, ValueError):
        pass
    return out


def cpu_threads() -> "tuple[int, str]":
    """torch threads for the CPU baseline and why: every CPU the cgroup quota grants (capped by the affinity set);
    without a quota, every core of the affinity set capped by OMP_NUM_THREADS when the host sets it (the GPU box
    asks each job to keep to a 16-CPU share of a larger machine)."""
    info = host_info()
    n = info["affinity_cores"]
    if info.get("cgroup_cpus"):
        q = max(1, int(info["cgroup_cpus"]))
        return max(1, min(n, q)), f"cgroup quota grants {info['cgroup_cpus']:g} CPUs ({info['cgroup_cpu_max']})"
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0 and int(omp) < n:
        return int(omp), (f"no cgroup CPU quota ({info['cgroup_cpu_max']}); OMP_NUM_THREADS={omp} of "
                          f"{n} affinity cores (the box's per-job CPU share)")
    return max(1, n), f"no cgroup CPU quota ({info['cgroup_cpu_max']}); all {n} affinity cores"


def cpu_baseline_sample(model, vae, cfg: dict, H: int, W: int, steps: int, n_blocks: int = 3, vae_s=None):
    """The fp32 CPU port of the path (oracle/flite_ref.py + oracle/vae_ref.py, checked against the stub-loaded
    reference's golden fixtures) timed on this node's host cores, on the same bf16 weights copied to the host.

    The component sample (the cross-check of cpu_baseline_full's whole step since round 6; `--cpu-baseline-full 0`
    makes it the value): measures every DIFFERENT piece of one image once and extrapolates: (a) the per-call DiT
    work outside the blocks (context_proj + norm, patch embed, time embed / adaLN, final stage; RefDiT at depth 0)
    at the CFG batch of 2, (b) `n_blocks` DiT blocks at full size (every block of a layout has the same shapes),
    (c) one full VAE decode to uint8 when a VAE is present (or `vae_s`, a decode already timed). Per image =
    steps x (a + depth x b / n_blocks) + c, labelled as extrapolated."""
    import dataclasses

    from oracle import flite_ref as R
    from oracle import vae_ref as VR

    threads, why = cpu_threads()
    prev_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    D = cfg["hidden_size"]
    nh = cfg["num_heads"]
    p = cfg["patch_size"]
    hp, wp = H // 8 // p, W // 8 // p
    T = 16 + hp * wp
    B = 2
    rcfg = R.DiTConfig(**{k: cfg[k] for k in ("in_channels", "patch_size", "hidden_size", "depth", "num_heads",
                                                 "mlp_ratio", "cross_attn_input_size", "train_bias_and_rms",
                                                 "per_block_adaln")})
    n_blocks = min(n_blocks, cfg["depth"])
    params = {n: t.detach().float().cpu() for n, t in model.named_parameters()
              if not n.startswith("blocks.") or int(n.split(".")[1]) < n_blocks}
    g = torch.Generator().manual_seed(0)
    res = {}
    with torch.no_grad():
        # (a) everything outside the blocks, one CFG-batched call
        top = R.RefDiT(dataclasses.replace(rcfg, depth=0), params, dtype=torch.float32)
        x_lat = torch.randn(B, cfg["in_channels"], H // 8, W // 8, generator=g)
        ctx_in = torch.randn(B, 512, cfg["cross_attn_input_size"], generator=g)
        t_in = torch.tensor([0.75, 0.75], dtype=torch.bfloat16)
        t0 = time.perf_counter()
        top(x_lat, ctx_in, None, t_in)
        res["top_s"] = time.perf_counter() - t0
        # (b) n_blocks full-size blocks
        ref = R.RefDiT(rcfg, params, dtype=torch.float32)
        x = torch.randn(B * T, D, generator=g)
        ctx = torch.randn(B * 512, D, generator=g)
        cu = torch.tensor([0, T, 2 * T], dtype=torch.int32)
        ccu = torch.tensor([0, 512, 1024], dtype=torch.int32)
        mod = tuple(0.02 * torch.randn(B * T, D, generator=g) for _ in range(9))
        cos, sin = R.rope_tables(hp, wp, D // (2 * nh), 10000.0, 16, torch.bfloat16)
        cos, sin = cos[None].repeat(1, B, 1), sin[None].repeat(1, B, 1)
        t0 = time.perf_counter()
        for i in range(n_blocks):
            x = ref.block(i, x, cu, T, ctx, ccu, mod, cos, sin)
        res["block_s"] = (time.perf_counter() - t0) / n_blocks
        # (c) one VAE decode to uint8
        res["vae_s"] = 0.0 if vae_s is None else float(vae_s)
        if vae is not None and vae_s is None:
            vparams = {n: t.detach().float().cpu() for n, t in vae.named_parameters()}
            dec = VR.RefVAEDecoder(vparams)
            z = torch.randn(1, 16, H // 8, W // 8, generator=g)
            t0 = time.perf_counter()
            VR.decode_to_uint8(dec, z)
            res["vae_s"] = time.perf_counter() - t0
    torch.set_num_threads(prev_threads)
    per_image = steps * (res["top_s"] + cfg["depth"] * res["block_s"]) + res["vae_s"]
    out = {
        "value": 1.0 / per_image,
        "unit": "images/s",
        "cores": threads,
        "cores_reason": why,
        "kind": "port",
        "extrapolated": True,
        "sample": (f"fp32 CPU port (oracle/flite_ref.py, oracle/vae_ref.py) at {H}x{W}, CFG batch 2 (T={T}): "
                   f"per-call non-block DiT work {res['top_s']:.2f} s, {n_blocks} of {cfg['depth']} blocks "
                   f"{res['block_s']:.2f} s each, VAE decode {res['vae_s']:.2f} s; per image = {steps} x "
                   f"({res['top_s']:.2f} + {cfg['depth']} x {res['block_s']:.2f}) + {res['vae_s']:.2f} = "
                   f"{per_image:.0f} s (EXTRAPOLATED from the measured components)"),
        "host": host_info(),
        "components_s": {k: round(v, 3) for k, v in res.items()},
    }
    return out


def cpu_baseline_full(model, vae, cfg: dict, H: int, W: int, steps: int, k_steps: int = 1):
    """BASELINE.md §4's plan and the default `cpu_baseline` since round 6: K whole CFG-batched denoise steps of the
    fp32 CPU port (every block, the CFG combine and Euler update) + one VAE decode, per image = (steps / K) x the K
    steps + the decode, labelled extrapolated. K = 1 at 10B 1024^2 is ~2.5 min of CPU on the box's 16-core
    share: one measured step of the 30, each of which does the same work (the schedule changes only t)."""
    from oracle import flite_ref as R
    from oracle import vae_ref as VR

    threads, why = cpu_threads()
    prev_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    rcfg = R.DiTConfig(**{k: cfg[k] for k in ("in_channels", "patch_size", "hidden_size", "depth", "num_heads",
                                                 "mlp_ratio", "cross_attn_input_size", "train_bias_and_rms",
                                                 "per_block_adaln")})
    import threading

    stop = threading.Event()

    def heartbeat():  # minutes of silent CPU work: keep the log moving
        t0 = time.time()
        while not stop.wait(30.0):
            print(f"[cpu baseline] {time.time() - t0:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    params = {n: t.detach().float().cpu() for n, t in model.named_parameters()}
    ref = R.RefDiT(rcfg, params, dtype=torch.float32)
    g = torch.Generator().manual_seed(0)
    lat = torch.randn(1, cfg["in_channels"], H // 8, W // 8, generator=g)
    pos = torch.randn(1, 512, cfg["cross_attn_input_size"], generator=g)
    res = {}
    with torch.no_grad():
        t0 = time.perf_counter()
        R.sample(ref, lat, pos, torch.zeros_like(pos), num_steps=steps, guidance_scale=6.0, height=H, width=W,
                 t_dtype=torch.bfloat16, acc_dtype=torch.float32, max_steps=k_steps)
        res["dit_steps_s"] = time.perf_counter() - t0
        res["vae_s"] = 0.0
        if vae is not None:
            dec = VR.RefVAEDecoder({n: t.detach().float().cpu() for n, t in vae.named_parameters()})
            t0 = time.perf_counter()
            VR.decode_to_uint8(dec, lat)
            res["vae_s"] = time.perf_counter() - t0
    stop.set()
    torch.set_num_threads(prev_threads)
    per_image = res["dit_steps_s"] * steps / k_steps + res["vae_s"]
    return {
        "value": 1.0 / per_image, "unit": "images/s", "cores": threads, "cores_reason": why, "kind": "port",
        "extrapolated": True,
        "sample": (f"fp32 CPU port (oracle/flite_ref.py sample loop + oracle/vae_ref.py) at {H}x{W}: {k_steps} whole "
                   f"CFG-6 steps of the {steps}-step schedule {res['dit_steps_s']:.1f} s, VAE decode "
                   f"{res['vae_s']:.1f} s; per image = {steps}/{k_steps} x {res['dit_steps_s']:.1f} + "
                   f"{res['vae_s']:.1f} = {per_image:.0f} s (EXTRAPOLATED x{steps / k_steps:g}, BASELINE.md §4)"),
        "host": host_info(), "components_s": {k: round(v, 3) for k, v in res.items()},
    }


def relaunch_distributed(n: int) -> int:
    """`bench.py --gpus N` run without torchrun: start the N ranks as a child torch.distributed.run (one process
    per GPU, 127.0.0.1 rendezvous) and return its exit code. Called before anything touches the GPU."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(Path(__file__).resolve())] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3, help="timed images per GPU")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="10b", choices=["7b", "10b"])
    ap.add_argument("--height", type=int, default=1024)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--sample-steps", type=int, default=30)
    ap.add_argument("--guidance", type=float, default=6.0)
    ap.add_argument("--no-vae", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--vae-tiling", action="store_true",
                    help="pipe.enable_vae_tiling() as generate.py:77-78 does (tiled decode above 1024 px)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline-full", type=int, default=1, metavar="K",
                    help="CPU baseline from K whole CFG steps + VAE, x steps/K (BASELINE.md §4; ~2.5 min of CPU per "
                         "step at 10B 1024^2 on 16 cores), with the per-component sample beside it as a cross-check; "
                         "0: the per-component sample alone")
    ap.add_argument("--images-per-gpu", type=int, default=1,
                    help="images per bench step and GPU, sampled as ONE batch (num_images_per_prompt; M = 2 x B x T)")
    ap.add_argument("--fp8", action="store_true",
                    help="BASELINE configs[4]: block GEMMs on MXFP8 weights + activations (block-scaled fp8 MFMA)")
    ap.add_argument("--fp8-bf16-blocks", default="",
                    help="with --fp8: comma-separated block indices that keep bf16 GEMMs (precision policy)")
    ap.add_argument("--negative-images", type=int, default=5, metavar="K",
                    help="after the metric's timed images, time min(K, --steps) more with a random (non-uniform) "
                         "negative context, as generate.py:17,84 passes a user's negative prompt: the uniform-context "
                         "collapse is then off (value_with_negative_prompt); 0 skips it")
    ap.add_argument("--fp8-classes", default="all",
                    help="with --fp8: GEMM classes on MXFP8 (comma-separated _native.FP8_CLASSES names: qkv, proj, "
                         "cross_q, cross_proj, gate_up, down; 'all'), the others bf16 (precision policy)")
    ap.add_argument("--fp8-block-classes", default="",
                    help="with --fp8: per-block class policy, _native.fp8_block_masks syntax (e.g. "
                         "'0-3:none;4-7:gate_up+qkv'); overrides --fp8-classes for the blocks it names")
    ap.add_argument("--residual", default=None, choices=["fp32", "bf16"],
                    help="residual-stream storage (DiT.set_residual_dtype); default: the engine's (bf16 unless "
                         "FLITE_RESID_BF16=0)")
    ap.add_argument("--probe", default="gateup", choices=["gateup", "attn", "down", "qkv", "step", "none"])
    ap.add_argument("--mode", default="replica", choices=["replica", "cfg-parallel", "sp", "sp-ring"],
                    help="replica: image i on GPU i mod N (the metric line); cfg-parallel: the two CFG branches of an "
                         "image on a pair of GPUs; sp / sp-ring: one image over all N GPUs, token rows split, K/V "
                         "all-gathered per block (sp) or shifted round a ring (sp-ring). The latency modes are "
                         "single-image lines (SURVEY §8f rank 1), not the metric")
    args = ap.parse_args()

    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no torchrun around us: launch the N ranks ourselves (nothing has touched the GPU yet)
        raise SystemExit(relaunch_distributed(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU is required")
    if args.mode == "cfg-parallel" and world % 2:
        raise SystemExit("--mode cfg-parallel pairs the ranks: --gpus must be even")
    if args.mode in ("sp", "sp-ring") and world < 2:
        raise SystemExit(f"--mode {args.mode} splits one image over the ranks: --gpus must be >= 2")
    if args.mode != "replica" and (args.images_per_gpu != 1 or args.guidance < 1.0):
        raise SystemExit("the latency modes run one CFG image per group (--images-per-gpu 1, --guidance >= 1)")
    # FLITE_BENCH_REHEARSAL=1: rehearse the N-rank path on a box with fewer GPUs (ranks share GPUs round-robin,
    # gloo instead of RCCL, which refuses two ranks on one device). Never the measured configuration: the line
    # says so in "distributed".
    rehearsal = world > 1 and os.environ.get("FLITE_BENCH_REHEARSAL") == "1"
    if rehearsal:
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    # FLITE_BENCH_PG=1 at N = 1: run the line through a one-rank RCCL process group anyway, so the multi-GPU code path
    # (communicator set-up, the timed context broadcast, max over ranks) executes on the one GPU
    single_pg = world == 1 and os.environ.get("FLITE_BENCH_PG") == "1"
    if world > 1 or single_pg:
        import torch.distributed as dist

        if single_pg:
            import socket

            with socket.socket() as so:
                so.bind(("127.0.0.1", 0))
                free_port = so.getsockname()[1]
            for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", str(free_port)), ("RANK", "0"),
                         ("WORLD_SIZE", "1")):
                os.environ.setdefault(k, v)

        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")

    from f_lite import DiT, FLitePipeline
    from f_lite import _native as nat
    from f_lite.distributed import (broadcast_context, image_indices, max_over_ranks, process_group_info,
                                    timed_broadcast_context)
    from f_lite.model import PRESETS

    cfg = dict(PRESETS[args.model])
    model = DiT.random(seed=0, device=dev, **cfg)
    if args.residual is not None:
        model.set_residual_dtype(torch.bfloat16 if args.residual == "bf16" else torch.float32)
    keep16 = [int(b) for b in args.fp8_bf16_blocks.split(",") if b.strip()]
    fp8_mask = nat.fp8_class_mask(args.fp8_classes) if args.fp8 else None
    blk_masks = (nat.fp8_block_masks(args.fp8_block_classes, cfg["depth"], fp8_mask)
                 if args.fp8 and args.fp8_block_classes else None)
    if args.fp8:
        model.enable_fp8(True, bf16_blocks=keep16, gemm_classes=fp8_mask, block_classes=blk_masks)
    vae = None
    if not args.no_vae:
        from f_lite.vae import AutoencoderKL

        vae = AutoencoderKL.random(seed=0, device=dev)
    pipe = FLitePipeline(model, vae)
    if args.vae_tiling:
        pipe.enable_vae_tiling()

    # synthetic T5 context [1, 512, 4096] (uniform, std 1), generated on rank 0 and broadcast over RCCL/xGMI
    ctx = torch.empty(1, 512, cfg["cross_attn_input_size"], device=dev, dtype=torch.bfloat16)
    if rank == 0:
        nat.init_param_(ctx, "synthetic.t5_context", seed=1, std=1.0)
    # the context broadcast is the replica mode's one collective: timed, so a multi-GPU line says what it cost
    bcast_ms = timed_broadcast_context(ctx, src=0)
    # a negative prompt's embedding (generate.py:17,84 -> pipeline.py:163-168): not a context of equal rows
    neg_ctx = None
    if args.negative_images > 0 and args.mode == "replica":
        neg_ctx = torch.empty_like(ctx)
        if rank == 0:
            nat.init_param_(neg_ctx, "synthetic.t5_negative_context", seed=3, std=1.0)
        broadcast_context(neg_ctx, src=0)

    lh, lw = args.height // 8, args.width // 8

    BI = args.images_per_gpu
    # work units: replica = one rank; cfg-parallel = a pair of ranks (uncond, cond); sp = all ranks
    if args.mode == "cfg-parallel":
        pairs = [dist.new_group([2 * i, 2 * i + 1]) for i in range(world // 2)]  # every rank creates every group
        pipe.enable_cfg_parallel(pairs[rank // 2])
        n_units, unit = world // 2, rank // 2
    elif args.mode in ("sp", "sp-ring"):
        pipe.enable_sequence_parallel(None, ring=args.mode == "sp-ring")
        n_units, unit = 1, 0
    else:
        n_units, unit = world, rank
    if args.mode != "replica":
        args.probe = "none"  # the per-launch probe shapes assume whole CFG batches on one GPU

    def latents_for(i):  # step i of this rank: images i * BI .. i * BI + BI - 1
        lats = []
        for j in range(i * BI, i * BI + BI):
            lat = torch.empty(1, 16, lh, lw, device=dev, dtype=torch.bfloat16)
            lats.append(nat.init_param_(lat, f"synthetic.latents.{j}", seed=2, std=1.0))
        return torch.cat(lats)

    out_type = "latent" if vae is None else "uint8"

    def one_image(i, negative=None):
        return pipe(prompt_embeds=ctx, negative_prompt_embeds=negative, latents=latents_for(i), height=args.height,
                    width=args.width, num_inference_steps=args.sample_steps, guidance_scale=args.guidance,
                    output_type=out_type, num_images_per_prompt=BI, use_graph=not args.no_graph).images

    def timed(n, negative=None):
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k in range(n):
            one_image(mine[k], negative)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        return time.perf_counter() - t

    mine = image_indices(n_units * (args.steps + args.warmup), unit, n_units)  # image i -> unit i mod n_units
    for w in range(args.warmup):
        one_image(mine[args.steps + w])
    kinds = {"gateup": nat.PROBE_GEMM_GATEUP, "attn": nat.PROBE_ATTN_SELF, "down": nat.PROBE_GEMM_DOWN,
             "qkv": nat.PROBE_GEMM_QKV, "step": nat.PROBE_STEP, "none": -1}
    eng = model.engine()
    elapsed = timed(args.steps)
    # the same workload with a user's negative prompt (no uniform-context collapse): one untimed image for the new
    # context's set-up and graph capture, then min(K, steps) timed; reported beside the metric, never as `value`
    neg_images, elapsed_neg = 0, None
    if neg_ctx is not None:
        neg_images = min(args.negative_images, args.steps)
        one_image(mine[0], neg_ctx)
        elapsed_neg = timed(neg_images, neg_ctx)
    # Per-launch timing of the dominant kernel: HIP event pairs on the engine stream around every launch of
    # that kernel during one more image (the same launch sequence, run eagerly: event timestamps are not
    # readable from a replayed hipGraph on ROCm 7.2).
    probe_ms = []
    if args.probe != "none":
        eng.set_probe(kinds[args.probe], 4 * cfg["depth"] * args.sample_steps)
        pipe(prompt_embeds=ctx, latents=latents_for(unit), height=args.height, width=args.width,
             num_inference_steps=args.sample_steps, guidance_scale=args.guidance, output_type=out_type,
             num_images_per_prompt=BI, use_graph=False)
        torch.cuda.synchronize()
        probe_ms = eng.read_probe(8192)
        eng.set_probe(-1, 0)
    elapsed = max_over_ranks(elapsed, device=dev)
    if elapsed_neg is not None:
        elapsed_neg = max_over_ranks(elapsed_neg, device=dev)
    bcast_ms_max = max_over_ranks(bcast_ms, device=dev) if dist is not None else bcast_ms
    pg = process_group_info()
    if rank != 0:
        dist.destroy_process_group()
        return

    ms_per_step = elapsed / args.steps * 1000.0
    value = n_units * args.steps * BI / elapsed
    f_step, f_once = dit_flops(cfg, args.height, args.width, args.sample_steps)
    f_vae = vae_flops(args.height, args.width) if vae is not None else 0.0
    D = cfg["hidden_size"]
    F = int(D * cfg["mlp_ratio"])
    T = 16 + (args.height // 16) * (args.width // 16)
    # the reference's work per image, and what this path skips: in the replica mode the two CFG copies of an image
    # share block 0's self-attention sub-block (qkv GEMM, attention, proj GEMM: identical inputs until block 0's
    # cross-attention, dit.cpp forward), computed once per step instead of twice
    f_ref_image = args.sample_steps * 2 * f_step + 2 * f_once + f_vae
    dedup = args.mode == "replica" and args.guidance >= 1.0 and os.environ.get("FLITE_NO_CFG_DEDUP") is None
    f_dedup = args.sample_steps * (2 * T * D * 3 * D + 4 * T * T * D + 2 * T * D * D) if dedup else 0.0
    # uniform-context collapse (dit.cpp set_context): the uncond copy's context is the pipeline's zero negative prompt
    # (pipeline.py:160-161), so its cross-attention keys/values are all equal and its cross-attention sub-block is
    # the step-invariant x += gate * (V . Wproj^T): no cross-q GEMM, attention or cross-proj GEMM for those rows
    cross_blocks = sum(1 for i in range(cfg["depth"]) if cfg["per_block_adaln"] or i % 4 == 0 or i < 8)
    # (fp8 blocks: where the collapsed rows end on a 4-row boundary, dit.cpp uni_fp8)
    collapse = (args.mode != "sp" and args.mode != "sp-ring" and args.guidance >= 1.0 and (not args.fp8 or T % 4 == 0)
                and os.environ.get("FLITE_NO_CTX_COLLAPSE") is None)
    f_collapse = (args.sample_steps * cross_blocks * (2 * T * D * D + 4 * T * 512 * D + 2 * T * D * D)
                  if collapse else 0.0)
    f_image = f_ref_image - f_dedup - f_collapse
    neg = None
    if elapsed_neg is not None:
        v_neg = n_units * neg_images * BI / elapsed_neg
        neg = {"value": round(v_neg, 5), "images_per_gpu": neg_images, "ms_per_image": round(elapsed_neg / neg_images
                                                                                           * 1000.0 / BI, 2),
               "algorithmic_flops_per_image": f_ref_image - f_dedup,
               "mfma_util_image": round((f_ref_image - f_dedup) * v_neg / world / PEAK_BF16, 4),
               "context": "random [1,512,4096] negative context (not uniform): the uncond copy runs its own "
                          "cross-attention, as with any user negative prompt (generate.py:17,84)"}
    M = 2 * BI * T
    per_launch = {
        "gateup": (2.0 * M * 2 * F * D, "SwiGLU gate/up GEMM (M=%d, N=%d, K=%d)" % (M, 2 * F, D)),
        "down": (2.0 * M * D * F, "down GEMM + gated residual (M=%d, N=%d, K=%d)" % (M, D, F)),
        "qkv": (2.0 * M * 3 * D * D, "qkv GEMM (M=%d, N=%d, K=%d)" % (M, 3 * D, D)),
        "attn": (2 * BI * 4.0 * T * T * D, "self-attention (B=%d, H=%d, T=%d, hd=256)" % (2 * BI, cfg["num_heads"], T)),
        "step": (2.0 * BI * f_step, "one CFG-batched denoise step"),
    }
    roofline = None
    if probe_ms:
        avg_ms = sum(probe_ms) / len(probe_ms)
        flops, what = per_launch[args.probe]
        achieved = flops / (avg_ms * 1e-3) / 1e12
        cls = {"gateup": "gate_up", "down": "down", "qkv": "qkv"}.get(args.probe)
        fp8_kernel = args.fp8 and cls is not None and bool(nat.fp8_class_mask(args.fp8_classes) & nat.FP8_CLASSES[cls])
        peak = PEAK_FP8 if fp8_kernel else PEAK_BF16
        roofline = {"bound": "mfma", "achieved": round(achieved, 1), "peak": round(peak / 1e12, 1),
                    "unit": "TFLOP/s", "frac": round(achieved * 1e12 / peak, 4), "traffic": None,
                    "kernel": what, "launches": len(probe_ms), "avg_ms": round(avg_ms, 4),
                    "algorithmic_flops_per_launch": flops}
        pmc = ROOT / "profiles" / "pmc_traffic.json"
        if pmc.exists() and not args.fp8:
            try:
                tr = json.loads(pmc.read_text()).get(args.probe)
                if tr:
                    roofline["traffic"] = tr["hbm_bytes_per_launch"]
                    roofline["traffic_source"] = ("rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE passes over "
                                                  "f-lite_amd/tools/pmc_gemm.py (same kernel and shape), "
                                                  "profiles/pmc_traffic.json; L2->fabric bytes incl. "
                                                  "Infinity-Cache hits")
                    roofline["algorithmic_bytes_per_launch"] = 2.0 * (M * D + 2 * F * D + M * F)
                    if "mfma_busy_frac" in tr:
                        roofline["pmc_mfma_busy_frac"] = round(tr["mfma_busy_frac"], 4)
            except Exception:
                pass
    cpu = None
    if not args.no_cpu_baseline and world == 1:  # at N = 1 only (rank 0)
        if args.cpu_baseline_full > 0:
            # the value: whole measured CFG step(s) + VAE; the component sample beside it as the cross-check
            cpu = cpu_baseline_full(model, vae, cfg, args.height, args.width, args.sample_steps,
                                    args.cpu_baseline_full)
            chk = cpu_baseline_sample(model, vae, cfg, args.height, args.width, args.sample_steps, n_blocks=1,
                                      vae_s=cpu["components_s"]["vae_s"])
            cpu["components_check"] = {"per_image_s": round(1.0 / chk["value"], 1), "sample": chk["sample"],
                                       "components_s": chk["components_s"],
                                       "ratio_to_value": round(cpu["value"] / chk["value"], 4)}
        else:
            cpu = cpu_baseline_sample(model, vae, cfg, args.height, args.width, args.sample_steps)

    metric = "images/sec @%dx%d, %d steps, F-Lite-%s %s" % (args.width, args.height, args.sample_steps,
                                                            args.model.upper(), "fp8" if args.fp8 else "bf16")
    if (args.model, args.height, args.width, args.sample_steps, args.fp8) == ("10b", 1024, 1024, 30, False):
        metric += "; 1/8 GPU + MFMA util%"  # BASELINE.json's metric string (util in mfma_util_image)
    if args.mode != "replica":
        metric += " [single-image latency mode: %s]" % args.mode
    line = {
        "metric": metric,
        "value": round(value, 5),
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 2),
        "higher_is_better": True,
        "scaling": "strong" if args.mode in ("sp", "sp-ring") else "weak",
        "vs_baseline": None,
        "dtype": ("fp8 (MXFP8: OCP e4m3 weights+activations, E8M0 scale per 32; block GEMMs) + bf16 attention"
                  if args.fp8 else "bf16"),
        "data": "synthetic (random-init weights from the deterministic generator; synthetic T5 context "
                "[1,512,4096]; seeded latents)",
        "config": {"workload": "F-Lite-%s %s, %dx%d, %d steps, CFG %.1f, %s" % (
            args.model.upper(), "model_v2 layout" if cfg["per_block_adaln"] else "model.py layout",
            args.width, args.height, args.sample_steps, args.guidance,
            "VAE decode to uint8" if vae is not None else "latents only (no VAE)"),
                   "images_per_gpu_per_step": BI, "cfg_batch": 2,
                   "parallelism": {"replica": "replica dp%d" % world, "cfg-parallel": "cfg-parallel %d pair(s)" % n_units,
                                   "sp": "sequence parallel sp%d (K/V all-gather per block)" % world,
                                   "sp-ring": "sequence parallel sp%d (ring K/V shifts)" % world}[args.mode],
                   "hipgraph": not args.no_graph, "vae_tiling": bool(args.vae_tiling),
                   "fp8_bf16_blocks": keep16 if args.fp8 else None,
                   "fp8_classes": args.fp8_classes if args.fp8 else None,
                   "fp8_class_mask": fp8_mask,
                   "fp8_block_classes": (args.fp8_block_classes or None) if args.fp8 else None,
                   "residual_dtype": "bf16" if model.engine().residual_bf16() else "fp32"},
        "distributed": {"world_size": world,
                        "backend": ("gloo REHEARSAL (ranks share %d GPU(s); not a measurement)"
                                    % torch.cuda.device_count() if rehearsal else
                                    "nccl (RCCL over xGMI)" if dist is not None else "none"),
                        "collectives": {
                            "replica": "one broadcast of the [1,512,4096] context from rank 0 before the loop",
                            "cfg-parallel": "context broadcast + per step one all-gather of the two fp32 branch outputs",
                            "sp": "context broadcast + per block an all-gather of the K/V rows, per step the output rows",
                            "sp-ring": "context broadcast + per block N-1 ring shifts of K/V rows, per step the output "
                                       "rows"}[args.mode],
                        "images_per_unit": args.steps, "units": n_units,
                        "process_group": pg,
                        "context_broadcast_ms": round(bcast_ms_max, 3),
                        "context_broadcast_note": "wall time of the [1,512,4096] bf16 context broadcast incl. the "
                                                  "first collective's communicator set-up (max over ranks)"},
        "value_with_negative_prompt": None if neg is None else neg["value"],
        "negative_prompt": neg,
        "mode": args.mode,
        "latency_ms_per_image": round(elapsed / args.steps * 1000.0 / BI, 2),
        "mfma_util_image": round(f_image * value / world / PEAK_BF16, 4),
        "mfma_util_image_peak": "bf16 dense (2.5166 PF) for both dtypes" if args.fp8 else "bf16 dense",
        "algorithmic_flops_per_image": f_image,
        "reference_flops_per_image": f_ref_image,
        "cfg_dedup_flops_per_image": f_dedup,
        "uniform_ctx_collapse_flops_per_image": f_collapse,
        "roofline": roofline,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
