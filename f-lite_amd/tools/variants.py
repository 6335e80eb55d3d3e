"""A/B builds of one kernel source with compile-time knobs (diagnostic; not part of the product library).

build (CPU container):  python tools/variants.py build gemm NAME -DKNOB=1 ...
    compiles csrc/<src>.hip with the knobs and links it with the product objects of every other source into
    tools/variants/NAME/libflite_hip.so (git-ignored).
run (GPU box):          python tools/variants.py run gemm NAME1 NAME2 ... [--rounds R]
    times the DiT GEMM (or attention) shapes under each variant, alternating variants per round, one
    subprocess per (variant, round) with FLITE_LIB pointing at the variant library.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
PKG = HERE.parent
sys.path.insert(0, str(PKG))

GEMM_SHAPES = [  # name, M, N, K, epilogue
    ("cube8k", 8192, 8192, 8192, "store"),
    ("gateup", 8224, 24576, 3072, "swiglu"),
    ("qkv", 8224, 9216, 3072, "store"),
    ("cross_q", 8224, 3072, 3072, "store"),
    ("proj", 8224, 3072, 3072, "resid"),
    ("down", 8224, 3072, 12288, "resid"),
]


def build(src, name, args):
    """args: -D knobs, and --sub OLD==>NEW textual substitutions applied to a temporary copy of the source
    (ablation builds: the product source never carries them)."""
    import build_native as bn

    bn.build(verbose=False)
    out = HERE / "variants" / name
    out.mkdir(parents=True, exist_ok=True)
    defines, subs = [], []
    text = (bn.CSRC / f"{src}.hip").read_text()
    it = iter(args)
    for a in it:
        if a == "--sub":
            old, new = next(it).split("==>")
            subs.append((old, new))
        elif a == "--from":  # another version of the source (e.g. `git show HEAD~1:...` saved to a file)
            text = Path(next(it)).read_text()
        else:
            defines.append(a)
    for old, new in subs:
        if old not in text:
            raise SystemExit(f"substitution target not found: {old!r}")
        text = text.replace(old, new)
    tmp = out / f"{src}.hip"
    tmp.write_text(text)
    obj = out / f"{src}.o"
    cmd = [bn.HIPCC, *bn.CFLAGS, *bn.FILE_FLAGS.get(f"{src}.hip", []), *defines, "-c", str(tmp), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stderr[-4000:])
    objs = [str(obj)] + [str(bn.BUILD / (p.stem + ".o")) for p in bn._sources() if p.stem != src]
    subprocess.run([bn.HIPCC, f"--offload-arch={bn.ARCH}", "-shared", "-fPIC", "-o", str(out / "libflite_hip.so"),
                    *objs, "-L/opt/rocm/lib", "-lrocprofiler-sdk-roctx", "-Wl,-rpath,/opt/rocm/lib"], check=True)
    (out / "defines.json").write_text(json.dumps({"defines": defines, "subs": subs}))
    print(f"built variant {name}: {defines} {len(subs)} substitution(s)")


def time_gemms(iters=20):
    import torch
    from f_lite import _native as nat

    torch.manual_seed(0)
    ws = nat.gemm_workspace("cuda")
    res = {}
    for name, M, N, K, epi in GEMM_SHAPES:
        a = torch.randn(M, K, device="cuda").bfloat16()
        if epi == "swiglu":
            w = (torch.randn(N // 2, K, device="cuda") * 0.05).bfloat16()
            w2 = (torch.randn(N // 2, K, device="cuda") * 0.05).bfloat16()
            out = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
            kw = dict(epilogue=nat.EPI_SWIGLU_BF16, w2=w2)
        elif epi == "resid":
            w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
            out = torch.zeros(M, N, device="cuda")
            kw = dict(epilogue=nat.EPI_RESID_F32, gate=torch.randn(2, N, device="cuda"), gate_seg_stride=N,
                      rows_per_seg=M // 2)
        else:
            w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            kw = dict(epilogue=nat.EPI_STORE_BF16)
        for _ in range(3):
            nat.gemm(a, w, out=out, workspace=ws, **kw)
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(iters):
            nat.gemm(a, w, out=out, workspace=ws, **kw)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / iters
        err = None
        if os.environ.get("VARIANTS_CHECK"):  # one launch against torch's fp32 product of the same operands
            af = a.float()
            if epi == "swiglu":
                ref = torch.nn.functional.silu(af @ w.float().t()) * (af @ w2.float().t())
                o = torch.empty_like(out)
                nat.gemm(a, w, out=o, workspace=ws, **kw)
            elif epi == "resid":
                x0 = torch.randn(M, N, device="cuda")
                g = kw["gate"]
                seg = (torch.arange(M, device="cuda") // (M // 2)).clamp(max=1)
                ref = x0 + (af @ w.float().t()) * g[seg]
                o = x0.clone()
                nat.gemm(a, w, out=o, workspace=ws, **kw)
            else:
                ref = af @ w.float().t()
                o = torch.empty_like(out)
                nat.gemm(a, w, out=o, workspace=ws, **kw)
            torch.cuda.synchronize()
            err = ((o.float() - ref).norm() / ref.norm()).item()
            del ref, o
        res[name] = (ms, 2.0 * M * N * K / ms / 1e9, err)
    return res


def time_attn(iters=30):
    import torch
    from f_lite import _native as nat

    torch.manual_seed(0)
    res = {}
    B, H, D = 2, 12, 256
    for name, T, Lk in (("self", 4112, 4112), ("cross", 4112, 512), ("cross_notail", 4096, 512),
                        ("cross_4720", 4720, 512)):
        q = torch.nn.functional.normalize(torch.randn(B * T, H, D, device="cuda"), dim=-1).mul(16).bfloat16()
        k = torch.nn.functional.normalize(torch.randn(B * Lk, H, D, device="cuda"), dim=-1).mul(16).bfloat16()
        v = torch.randn(B * Lk, H, D, device="cuda").bfloat16()
        cu_q = torch.tensor([0, T, 2 * T], dtype=torch.int32, device="cuda")
        cu_k = torch.tensor([0, Lk, 2 * Lk], dtype=torch.int32, device="cuda")
        out = torch.empty_like(q)
        ws = nat.attn_workspace("cuda", B, H)
        run = lambda: nat.attn_varlen(q, k, v, cu_q, cu_k, T, D ** -0.5, out=out, max_score=16.5,  # noqa: E731
                                      workspace=ws, max_k=Lk)
        for _ in range(3):
            run()
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(iters):
            run()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / iters
        err = None
        if os.environ.get("VARIANTS_CHECK"):  # one launch against torch's fp32 softmax attention, 4 heads per sequence
            o = torch.zeros_like(out)
            nat.attn_varlen(q, k, v, cu_q, cu_k, T, D ** -0.5, out=o, max_score=16.5, workspace=ws, max_k=Lk)
            num = den = 0.0
            for b in range(B):
                for h in (0, 5, 7, 11):
                    qs, ks = q[b * T:(b + 1) * T, h].float(), k[b * Lk:(b + 1) * Lk, h].float()
                    ref = torch.softmax(qs @ ks.t() * D ** -0.5, dim=-1) @ v[b * Lk:(b + 1) * Lk, h].float()
                    num += (o[b * T:(b + 1) * T, h].float() - ref).norm().item() ** 2
                    den += ref.norm().item() ** 2
            err = (num / den) ** 0.5
        res[name] = (ms, 4.0 * B * H * T * Lk * D / ms / 1e9, err)
    return res


def main():
    mode, src = sys.argv[1], sys.argv[2]
    if mode == "build":
        build(src, sys.argv[3], sys.argv[4:])
        return
    if mode == "child":
        print("RESULT " + json.dumps(time_attn() if src == "attention" else time_gemms()), flush=True)
        return
    args = sys.argv[3:]
    rounds = 3
    if "--rounds" in args:
        i = args.index("--rounds")
        rounds = int(args[i + 1])
        del args[i:i + 2]
    names = args
    table = {n: [] for n in names}
    for r in range(rounds):
        for n in names:  # NAME or NAME:VAR=VALUE (the variant's library under an extra environment variable)
            lib = HERE / "variants" / n.split(":")[0] / "libflite_hip.so"
            env = dict(os.environ, FLITE_LIB=str(lib))
            if ":" in n:
                key, val = n.split(":", 1)[1].split("=", 1)
                env[key] = val
            p = subprocess.run([sys.executable, __file__, "child", src], env=env, capture_output=True, text=True,
                               timeout=300)
            line = [l for l in p.stdout.splitlines() if l.startswith("RESULT ")]
            if p.returncode != 0 or not line:
                print(p.stdout[-2000:], p.stderr[-2000:])
                sys.exit(1)
            table[n].append(json.loads(line[0][7:]))
            print(f"round {r} {n}: " + " ".join(f"{k} {v[0]*1e3:.1f}us/{v[1]:.0f}TF" +
                                                 (f"/err {v[2]:.1e}" if len(v) > 2 and v[2] is not None else "")
                                                 for k, v in table[n][-1].items()), flush=True)
    print("== median us per shape")
    for n in names:
        shapes = table[n][0].keys()
        med = {k: sorted(t[k][0] for t in table[n])[len(table[n]) // 2] * 1e3 for k in shapes}
        print(n, " ".join(f"{k} {v:.1f}" for k, v in med.items()), f"sum {sum(med.values()):.1f}")


if __name__ == "__main__":
    main()
