"""Find the lane maps of v_mfma_scale_f32_16x16x128_f8f6f4 (fp8 e4m3 operands, E8M0 block scales) on the GPU.

    python f-lite_amd/tools/mfma_fp8_probe.py        (build mfma_fp8_probe.so here first: --build)

Operands are exact small integers (representable in e4m3), so every hypothesis is checked bit-exactly against
the hardware result (guide: "check the map with exact integer data before relying on it"). Prints which A/B
k-map and which scale map hold; the fp8 GEMM (gemm.hip, EPI with FP8 operands) is written to the winner.
"""
import ctypes
import json
import subprocess
import sys
from pathlib import Path

import torch

HERE = Path(__file__).resolve().parent
SO = HERE / "mfma_fp8_probe.so"


def build():
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                           str(HERE / "mfma_fp8_probe.hip"), "-o", str(SO)])


# lane l (0..63), byte j (0..31) -> k (0..127); the row (A) / column (B) is l & 15 in every hypothesis
HYP = {
    "contig32": lambda l, j: 32 * (l >> 4) + j,
    "two16": lambda l, j: 16 * (l >> 4) + j if j < 16 else 64 + 16 * (l >> 4) + (j - 16),
    "four8": lambda l, j: 8 * (l >> 4) + (j & 7) + 32 * (j >> 3),
    "contig32_rev": lambda l, j: 32 * (3 - (l >> 4)) + j,
}


def fp8_bytes(vals):
    return torch.tensor(vals, dtype=torch.float32).to(torch.float8_e4m3fn).view(torch.uint8)


def run(lib, a_bytes, b_bytes, sa, sb):
    dev = "cuda"
    a = a_bytes.reshape(64, 32).contiguous().view(torch.int32).to(dev)
    b = b_bytes.reshape(64, 32).contiguous().view(torch.int32).to(dev)
    sa_t = torch.tensor(sa, dtype=torch.int32, device=dev)
    sb_t = torch.tensor(sb, dtype=torch.int32, device=dev)
    d = torch.zeros(64 * 4, dtype=torch.float32, device=dev)
    rc = lib.mfma_fp8_probe(*(ctypes.c_void_p(t.data_ptr()) for t in (a, b, sa_t, sb_t, d)))
    assert rc == 0
    out = torch.zeros(16, 16)
    dc = d.cpu().view(64, 4)
    for l in range(64):
        for r in range(4):
            out[(l >> 4) * 4 + r, l & 15] = dc[l, r]
    return out


def expected(A, B, hyp_a, hyp_b, sa_of=None, sb_of=None):
    """A[m][k], B[k][n] logical; scales: sa_of(m, kblock) multiplier."""
    D = torch.zeros(16, 16, dtype=torch.float64)
    for m in range(16):
        for n in range(16):
            s = 0.0
            for k in range(128):
                fa = sa_of(m, k // 32) if sa_of else 1.0
                fb = sb_of(n, k // 32) if sb_of else 1.0
                s += float(A[m, k]) * float(B[k, n]) * fa * fb
            D[m, n] = s
    return D


def main():
    if "--build" in sys.argv:
        build()
        return
    lib = ctypes.CDLL(str(SO))
    g = torch.Generator().manual_seed(0)
    A = torch.randint(-3, 4, (16, 128), generator=g).float()
    B = torch.randint(-3, 4, (128, 16), generator=g).float()
    res = {}
    for name, f in HYP.items():
        ab = torch.zeros(64, 32, dtype=torch.uint8)
        bb = torch.zeros(64, 32, dtype=torch.uint8)
        for l in range(64):
            ab[l] = fp8_bytes([A[l & 15, f(l, j)].item() for j in range(32)])
            bb[l] = fp8_bytes([B[f(l, j), l & 15].item() for j in range(32)])
        one = [127] * 64
        D = run(lib, ab, bb, one, one)
        ok = torch.equal(D.double(), expected(A, B, f, f))
        res[name] = ok
        print(f"k-map {name}: {'MATCH' if ok else 'no'}", flush=True)
        if ok:
            # scales: lane l's E8M0 byte (opsel 0) = 127 + t(l): does it scale (row l & 15, k-block l >> 4)?
            sa = [127 + ((l >> 4) + (l & 3)) % 3 for l in range(64)]
            sb = [127 + (l >> 4) % 2 for l in range(64)]
            D2 = run(lib, ab, bb, sa, sb)
            e2 = expected(A, B, f, f, sa_of=lambda m, kb: 2.0 ** ((kb + (m & 3)) % 3),
                          sb_of=lambda n, kb: 2.0 ** (kb % 2))
            ok2 = torch.equal(D2.double(), e2)
            res[name + ".scale_per_lane_block"] = ok2
            print(f"  scale map (lane l -> row l&15, k-block l>>4): {'MATCH' if ok2 else 'no'}", flush=True)
            if not ok2:
                e3 = expected(A, B, f, f, sa_of=lambda m, kb: 2.0 ** ((kb + (m & 3)) % 3), sb_of=None)
                print("   (diff vs A-only hypothesis)", float((D2.double() - e3).abs().max()))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
