"""Cycle anatomy of the bounded attention key loop (diagnostic; never part of the product library).

patch (CPU container): python f-lite_amd/tools/attn_stamps.py patch
    writes tools/variants/_src/attention_stamps.hip: csrc/attention.hip with s_memtime stamps around phase A,
    phase B and the end-of-tile wait + barrier of every key-loop iteration, the prologue (kernel entry -> loop) and
    the loop end; each wave's sums go to a device array (vector stores from lane 0) read back by
    flite_attn_read_stamps. Then: python f-lite_amd/tools/variants.py build attention stamps --from <that file>
run (GPU box):       FLITE_LIB=f-lite_amd/tools/variants/stamps/libflite_hip.so python f-lite_amd/tools/attn_stamps.py run
    self- and cross-attention at the 10B 1024^2 shapes; prints the mean cycles per iteration of each phase for the
    full q-tiles (and the tail chunks), the prologue and the loop, over all waves.
The stamps themselves cost cycles (an s_memtime + its lgkmcnt wait per segment): compare phases, not the total.
"""
import ctypes
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
NV = 8  # values per wave


def patch(src_path=None, name="stamps"):
    src = Path(src_path or (HERE.parent / "csrc" / "attention.hip")).read_text()

    def sub(old, new, count=1):
        nonlocal src
        if src.count(old) != count:
            raise SystemExit(f"patch target found {src.count(old)} times (want {count}): {old!r}")
        src = src.replace(old, new)

    sub('#include "kernels.h"\n',
        '#include "kernels.h"\n__device__ unsigned long long g_attn_stamps[16384 * 4 * 8];\n'
        'extern "C" int flite_attn_read_stamps(void* dst, long bytes) {\n'
        '  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_attn_stamps), bytes, 0, hipMemcpyDeviceToHost) != hipSuccess;\n'
        '}\n'
        'extern "C" int flite_attn_clear_stamps() {\n'
        '  static unsigned long long z[16384 * 4 * 8];\n'
        '  return hipMemcpyToSymbol(HIP_SYMBOL(g_attn_stamps), z, sizeof(z), 0, hipMemcpyHostToDevice) != hipSuccess;\n'
        '}\n')
    sub('  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);\n',
        '  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);\n'
        '  const unsigned long long st_k0 = __builtin_amdgcn_s_memtime();\n'
        '  unsigned long long st_a = 0, st_b = 0, st_s = 0, st_l0 = 0, st_l1 = 0;\n  unsigned st_n = 0;\n')
    sub('''      if constexpr (HS) {
        if constexpr (P == 0)''', '''      const unsigned long long st0 = __builtin_amdgcn_s_memtime();
      if constexpr (HS) {
        if constexpr (P == 0)''')
    sub('''      if constexpr (P == 0)
        phase_b(I0{}, hs_, pa, pb);
      else
        phase_b(I1{}, hs_, pb, pa);
      ATTN_TILE_SYNC();
''', '''      const unsigned long long st1 = __builtin_amdgcn_s_memtime();
      if constexpr (P == 0)
        phase_b(I0{}, hs_, pa, pb);
      else
        phase_b(I1{}, hs_, pb, pa);
      const unsigned long long st2 = __builtin_amdgcn_s_memtime();
      ATTN_TILE_SYNC();
      const unsigned long long st3 = __builtin_amdgcn_s_memtime();
      st_a += st1 - st0;
      st_b += st2 - st1;
      st_s += st3 - st2;
      ++st_n;
''')
    sub('''      __syncthreads();  // every wave's K_0 reads are done before iteration 0 refills Kbuf 0
      int j = 0;''', '''      __syncthreads();  // every wave's K_0 reads are done before iteration 0 refills Kbuf 0
      st_l0 = __builtin_amdgcn_s_memtime();
      int j = 0;''')
    sub('''  if constexpr (BOUNDED) o_acc_fence(o_acc);
''', '''  if constexpr (BOUNDED) o_acc_fence(o_acc);
  st_l1 = __builtin_amdgcn_s_memtime();
  if (lane == 0 && blockIdx.x < 16384) {
    unsigned long long* d = g_attn_stamps + ((size_t)blockIdx.x * 4 + wave) * 8;
    d[0] = (unsigned long long)(chunk + 1);
    d[1] = st_l0 ? st_l0 - st_k0 : 0;
    d[2] = st_a;
    d[3] = st_b;
    d[4] = st_s;
    d[5] = st_n;
    d[6] = st_l0 ? st_l1 - st_l0 : 0;
    d[7] = 1;
  }
''')
    out = HERE / "variants" / "_src"
    out.mkdir(parents=True, exist_ok=True)
    (out / f"attention_{name}.hip").write_text(src)
    print(f"wrote {out / f'attention_{name}.hip'}")


def run():
    import torch
    from f_lite import _native as nat

    lib = nat.load()
    read = lib.flite_attn_read_stamps
    read.argtypes = [ctypes.c_void_p, ctypes.c_long]
    clear = lib.flite_attn_clear_stamps
    B, H, D = 2, 12, 256
    for name, T, Lk in (("self", 4112, 4112), ("cross", 4112, 512)):
        q = torch.nn.functional.normalize(torch.randn(B * T, H, D, device="cuda"), dim=-1).mul(16).bfloat16()
        k = torch.nn.functional.normalize(torch.randn(B * Lk, H, D, device="cuda"), dim=-1).mul(16).bfloat16()
        v = torch.randn(B * Lk, H, D, device="cuda").bfloat16()
        cu_q = torch.tensor([0, T, 2 * T], dtype=torch.int32, device="cuda")
        cu_k = torch.tensor([0, Lk, 2 * Lk], dtype=torch.int32, device="cuda")
        ws = nat.attn_workspace("cuda", B, H)
        for _ in range(5):
            nat.attn_varlen(q, k, v, cu_q, cu_k, T, D ** -0.5, max_score=16.5, workspace=ws, max_k=Lk)
        torch.cuda.synchronize()
        clear()
        nat.attn_varlen(q, k, v, cu_q, cu_k, T, D ** -0.5, max_score=16.5, workspace=ws, max_k=Lk)
        torch.cuda.synchronize()
        n = 16384 * 4 * NV
        buf = (ctypes.c_ulonglong * n)()
        assert read(buf, ctypes.sizeof(buf)) == 0
        t = torch.tensor(list(buf), dtype=torch.float64).view(-1, NV)
        t = t[t[:, 7] == 1]
        for label, sel in (("full q-tiles", t[:, 0] == 0), ("tail chunks", t[:, 0] > 0)):
            s = t[sel]
            if not len(s):
                continue
            it = s[:, 5].clamp(min=1)
            print(f"{name} {label}: {len(s)} waves, {s[:, 5].mean():.1f} iterations; per iteration: phase A "
                  f"{(s[:, 2] / it).mean():.0f} cyc, phase B {(s[:, 3] / it).mean():.0f}, wait+barrier "
                  f"{(s[:, 4] / it).mean():.0f} (ideal MFMA: 1024 + 1024); prologue {s[:, 1].mean():.0f} cyc, "
                  f"loop {s[:, 6].mean():.0f} cyc", flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "patch":  # patch [SOURCE NAME]: stamp another variant's source
        patch(*sys.argv[2:4])
    else:
        run()
