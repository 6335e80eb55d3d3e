"""Cycle anatomy of the 256-row attention key loop (attention_q256.hip; diagnostic, never in the product library).

patch (CPU container): python f-lite_amd/tools/attn_stamps_q256.py patch
    writes tools/variants/_src/attention_q256_stamps.hip with s_memtime stamps around phase A, phase B and the
    end-of-tile wait + barrier of every key-loop iteration (live waves), then builds tools/variants/q256stamps.
run (GPU box):       FLITE_LIB=f-lite_amd/tools/variants/q256stamps/libflite_hip.so python f-lite_amd/tools/attn_stamps_q256.py run
    prints the mean cycles per iteration of each phase for whole tiles, key halves and tail chunks.
"""
import ctypes
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
NV = 14


def patch():
    src = (HERE.parent / "csrc" / "attention_q256.hip").read_text()

    def sub(old, new, count=1):
        nonlocal src
        if src.count(old) != count:
            raise SystemExit(f"patch target found {src.count(old)} times (want {count}): {old!r}")
        src = src.replace(old, new)

    sub('#include "kernels.h"\n',
        '#include "kernels.h"\n__device__ unsigned long long g_q256_stamps[16384 * 4 * 14];\n'
        'struct StampAtExit {\n  unsigned long long* d = nullptr;\n'
        '  __device__ ~StampAtExit() { if (d) { d[0] = __builtin_amdgcn_s_memtime(); d[3] = __builtin_amdgcn_s_memrealtime(); } }\n};\n'
        'extern "C" int flite_q256_read_stamps(void* dst, long bytes) {\n'
        '  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_q256_stamps), bytes, 0, hipMemcpyDeviceToHost) != hipSuccess;\n'
        '}\n')
    sub('  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);\n',
        '  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);\n'
        '  const unsigned long long st_k0 = __builtin_amdgcn_s_memtime();\n'
        '  const unsigned long long rt_k0 = __builtin_amdgcn_s_memrealtime();\n'
        '  unsigned long long st_a = 0, st_b = 0, st_s = 0, st_l0 = 0, st_l1 = 0;\n  unsigned st_n = 0;\n')
    sub('''    const bool next = j + 1 < nt;  // the tile whose S phase A computes exists
''', '''    const bool next = j + 1 < nt;  // the tile whose S phase A computes exists
    const unsigned long long st0 = __builtin_amdgcn_s_memtime();
''')
    sub('''    if constexpr (LIVE) {
      const float l0 = l_run[0], l1 = l_run[1];''', '''    const unsigned long long st1 = __builtin_amdgcn_s_memtime();
    if constexpr (LIVE) {
      const float l0 = l_run[0], l1 = l_run[1];''')
    sub('''      l_run[1] = next ? l_run[1] : l1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };''', '''      l_run[1] = next ? l_run[1] : l1;
    }
    const unsigned long long st2 = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const unsigned long long st3 = __builtin_amdgcn_s_memtime();
    st_a += st1 - st0;
    st_b += st2 - st1;
    st_s += st3 - st2;
    ++st_n;
  };''')
    sub('''    __syncthreads();  // every wave's K_0 reads are done before iteration 0 refills Kbuf 0
''', '''    __syncthreads();  // every wave's K_0 reads are done before iteration 0 refills Kbuf 0
    st_l0 = __builtin_amdgcn_s_memtime();
''')
    sub('''  o_fence16<0>(o_acc);
  o_fence16<1>(o_acc);
''', '''  o_fence16<0>(o_acc);
  o_fence16<1>(o_acc);
  st_l1 = __builtin_amdgcn_s_memtime();
  if (lane == 0 && live && blockIdx.x < 16384) {
    unsigned long long* d = g_q256_stamps + ((size_t)blockIdx.x * 4 + wave) * 14;
    d[0] = (unsigned long long)nchunk;
    d[1] = st_l0 ? st_l0 - st_k0 : 0;
    d[2] = st_a;
    d[3] = st_b;
    d[4] = st_s;
    d[5] = st_n;
    d[6] = st_l0 ? st_l1 - st_l0 : 0;
    d[7] = 1;
    d[9] = st_k0;
    d[10] = rt_k0;
    d[12] = (unsigned long long)__builtin_amdgcn_s_getreg(0xF804);  // HW_ID: wave, SIMD, CU, SH, SE
    d[13] = (unsigned long long)__builtin_amdgcn_s_getreg(0xF814);  // XCC_ID
  }
  StampAtExit st_exit;  // every return below stamps the exit time into d[8]
  if (lane == 0 && live && blockIdx.x < 16384) st_exit.d = g_q256_stamps + ((size_t)blockIdx.x * 4 + wave) * 14 + 8;
''')
    out = HERE / "variants" / "_src"
    out.mkdir(parents=True, exist_ok=True)
    f = out / "attention_q256_stamps.hip"
    f.write_text(src)
    subprocess.run([sys.executable, str(HERE / "variants.py"), "build", "attention_q256", "q256stamps", "--from",
                    str(f)], check=True)


def run():
    import torch
    from f_lite import _native as nat

    nat.attn_set_q256(True)
    lib = nat.load()
    read = lib.flite_q256_read_stamps
    read.argtypes = [ctypes.c_void_p, ctypes.c_long]
    D = 256
    for name, lens, H in (("self 2x4112 H12", [4112, 4112], 12), ("one round 2x4096 H8", [4096, 4096], 8)):
        B, T = len(lens), lens[0]
        q = torch.nn.functional.normalize(torch.randn(B * T, H, D, device="cuda"), dim=-1).mul(16).bfloat16()
        k = torch.nn.functional.normalize(torch.randn(B * T, H, D, device="cuda"), dim=-1).mul(16).bfloat16()
        v = torch.randn(B * T, H, D, device="cuda").bfloat16()
        cu = torch.tensor([0, T, 2 * T], dtype=torch.int32, device="cuda")
        ws = nat.attn_workspace("cuda", B, H, T, T)
        for _ in range(5):
            nat.attn_varlen(q, k, v, cu, cu, T, D ** -0.5, max_score=16.5, workspace=ws, max_k=T)
        torch.cuda.synchronize()
        z = torch.zeros(16384 * 4 * NV, dtype=torch.int64)
        buf = (ctypes.c_ulonglong * z.numel())()
        nat.attn_varlen(q, k, v, cu, cu, T, D ** -0.5, max_score=16.5, workspace=ws, max_k=T)
        torch.cuda.synchronize()
        assert read(buf, ctypes.sizeof(buf)) == 0
        t = torch.tensor(list(buf), dtype=torch.float64).view(-1, NV)
        t = t[t[:, 7] == 1]
        r0, r1 = t[:, 10].min(), t[:, 11].max()
        print(f"{name}: realtime span {(r1 - r0) / 100:.1f} us (100 MHz s_memrealtime, first wave start -> last exit)",
              flush=True)
        hw = t[:, 12].long()
        cu = (t[:, 13].long() & 15) * 4096 + ((hw >> 13) & 7) * 512 + ((hw >> 12) & 1) * 256 + ((hw >> 8) & 15)
        w0 = (hw & 15) == (hw & 15).min()  # one record per workgroup: its first live wave's slot
        items = {}
        for c_, a_, b_ in zip(cu.tolist(), t[:, 10].tolist(), t[:, 11].tolist()):
            items.setdefault(c_, set()).add((a_, b_))
        counts = torch.tensor([len(v) for v in items.values()], dtype=torch.float64)
        print(f"  CUs used {len(items)}; items per CU min {counts.min():.0f} median {counts.median():.0f} max "
              f"{counts.max():.0f}", flush=True)
        busy = torch.tensor([sum(b_ - a_ for a_, b_ in v) for v in items.values()], dtype=torch.float64) / 100
        print(f"  per-CU busy us: min {busy.min():.1f} median {busy.median():.1f} max {busy.max():.1f}", flush=True)
        for label, sel in (("whole tiles", t[:, 0] == 1), ("key halves", t[:, 0] == 2), ("tail chunks", t[:, 0] > 2)):
            s = t[sel]
            if len(s):
                st_ = (s[:, 10] - r0) / 100
                print(f"  {label} start times (us after the first): " +
                      " ".join(f"{v:.1f}" for v in torch.quantile(st_, torch.tensor([0, .1, .25, .5, .75, .9, 1.],
                                                                                     dtype=torch.float64)).tolist()),
                      flush=True)
        for label, sel in (("whole tiles", t[:, 0] == 1), ("key halves", t[:, 0] == 2), ("tail chunks", t[:, 0] > 2)):
            s = t[sel]
            if not len(s):
                continue
            it = s[:, 5].clamp(min=1)
            tail = s[:, 8] - (s[:, 9] + s[:, 1] + s[:, 6])
            print(f"{name} {label}: {len(s)} waves, {s[:, 5].mean():.1f} iterations; per iteration: phase A "
                  f"{(s[:, 2] / it).mean():.0f} cyc, phase B {(s[:, 3] / it).mean():.0f}, wait+barrier "
                  f"{(s[:, 4] / it).mean():.0f} (ideal MFMA 1024 + 1024); prologue {s[:, 1].mean():.0f} cyc, loop "
                  f"{s[:, 6].mean():.0f} cyc, after the loop {tail.mean():.0f} cyc (max {tail.max():.0f}), wave "
                  f"lifetime {(s[:, 8] - s[:, 9]).mean():.0f} cyc", flush=True)


if __name__ == "__main__":
    patch() if sys.argv[1] == "patch" else run()
