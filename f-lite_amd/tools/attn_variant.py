"""Schedule variants of the bounded attention key loop (diagnostic A/B builds; the product source carries no knobs).

    python f-lite_amd/tools/attn_variant.py NAME [--kspread] [--vdma-b PHASE]
        writes tools/variants/_src/attention_NAME.hip from csrc/attention.hip and builds tools/variants/NAME with
        tools/variants.py (--from). Then on the GPU box:
    python f-lite_amd/tools/variants.py run attention base NAME ... [--rounds R]

--kspread      the 8 K_{j+2} LDS-DMA pieces of phase A go one per second MFMA pair (s even) instead of pairs 0-7
--vdma-b P     the 8 V_{j+1} pieces leave phase A for phase B, one after every 4th PV MFMA (m % 4 == P): phase A then
               carries K reads + K pieces, phase B V reads + V pieces + the softmax, so neither phase alone saturates
               the CU's texture path (64 KiB of pieces per 64-key tile at 64 B/clk = 1024 of the tile's 2048 MFMA
               cycles). V_{j+1} lands in the V buffer phase B of iteration j does NOT read (last read in j - 1,
               before its barrier), and the end-of-iteration vmcnt(0) + barrier publishes it as before.

The round-4 --qscale (pre-scaled Q^T, no shift) and --ldelay (row sum one score late) variants are in the product
source since round 4 (profiles/r04b), so they are no longer patches; profiles/r04b's baseline is that commit's parent.
"""
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent


def make(name, kspread=False, vdma_b=None, qlate=False, packdelay=False, split=None):
    src = (HERE.parent / "csrc" / "attention.hip").read_text()

    def sub(old, new, count=1):
        nonlocal src
        if src.count(old) != count:
            raise SystemExit(f"patch target found {src.count(old)} times (want {count}): {old!r}")
        src = src.replace(old, new)

    dma_a_old = '''        if constexpr (DMA) {  // K pieces first (needed first), then V
          if (s < 8)
            blds16(krs, k_src[s], lds0 + DKB * TILE + (wave * 8 + s) * 1024 + K_OFF);
          else
            blds16(vrs, v_src[s - 8], lds0 + DVB * TILE + (wave * 8 + s - 8) * 1024 + V_OFF);
        }'''
    k_cond = "(s & 1) == 0" if kspread else "s < 8"
    k_idx = "(s >> 1)" if kspread else "s"
    if vdma_b is None:
        v_part = '''
          else if (!(''' + k_cond + '''))
            blds16(vrs, v_src[s - 8], lds0 + DVB * TILE + (wave * 8 + s - 8) * 1024 + V_OFF);''' if not kspread else '''
          else
            blds16(vrs, v_src[s >> 1], lds0 + DVB * TILE + (wave * 8 + (s >> 1)) * 1024 + V_OFF);'''
    else:
        v_part = ""
    sub(dma_a_old, '''        if constexpr (DMA) {
          if (''' + k_cond + ''')
            blds16(krs, k_src[''' + k_idx + '''], lds0 + DKB * TILE + (wave * 8 + ''' + k_idx + ''') * 1024 + K_OFF);''' +
        v_part + '''
        }''')
    if qlate:  # Q^T moves to AGPRs (which waits for its loads) only AFTER the K_0 / V_0 / K_1 copies are issued,
        # so the prologue pays max(Q latency, K/V latency) instead of their sum
        pin = ("    if constexpr (BOUNDED) {  // move Q^T into AGPRs here, then clear the write -> MFMA-read hazard\n"
               "#pragma unroll\n"
               "      for (int s = 0; s < 16; ++s) asm volatile(\"\" : \"+a\"(qf[s]));\n"
               "      asm volatile(\"s_nop 4\" ::: \"memory\");\n"
               "    }\n")
        sub(pin, "")
        sub("        for (int i = 0; i < 8; ++i) blds16(krs, k_src[i], lds0 + TILE + (wave * 8 + i) * 1024 + K_OFF);\n"
            "      }\n",
            "        for (int i = 0; i < 8; ++i) blds16(krs, k_src[i], lds0 + TILE + (wave * 8 + i) * 1024 + K_OFF);\n"
            "      }\n" + pin.replace("    if constexpr", "      if constexpr").replace("#pragma", "#pragma")
            .replace("\n      for", "\n        for").replace("\n      asm", "\n        asm").replace("\n    }\n", "\n      }\n"))
    if packdelay:  # (product source: delayed row sum already in) the bf16 pair of scores (e-2, e-1) is packed at
        # element e, so the v_cvt_pk never waits on the v_exp just issued; the last pair after the loop
        sub("""      l_run += e_prev;
      if (e & 1) {
        const bf16x2 pr = {(__bf16)e_prev, (__bf16)v};
        pn[(e >> 4) * 2 + (r >> 3)][(r & 7) >> 1] = __builtin_bit_cast(unsigned, pr);
      }
      e_prev = v;
    };""", """      l_run += e_prev;
      if (!(e & 1) && e >= 2) pack_pair(pn, e - 2, e_prev2, e_prev);
      e_prev2 = e_prev;
      e_prev = v;
    };""")
        sub("    auto softmax_elem = [&](u32x4 (&pn)[4], int e, float& e_prev) {",
            """    auto pack_pair = [&](u32x4 (&pn)[4], int e, float a, float b) {  // scores e, e + 1 (e even)
      const int r = e & 15;
      const bf16x2 pr = {(__bf16)a, (__bf16)b};
      pn[(e >> 4) * 2 + (r >> 3)][(r & 7) >> 1] = __builtin_bit_cast(unsigned, pr);
    };
    float e_prev2 = 0.f;
    auto softmax_elem = [&](u32x4 (&pn)[4], int e, float& e_prev) {""")
        sub("      if constexpr (EX) l_run += e_prev;\n",
            "      if constexpr (EX) {\n        l_run += e_prev;\n        pack_pair(pn, 30, e_prev2, e_prev);\n      }\n")
        sub("        for (int e = 0; e < 32; ++e) softmax_elem(pa, e, e_prev);\n        l_run += e_prev;\n",
            "        for (int e = 0; e < 32; ++e) softmax_elem(pa, e, e_prev);\n        l_run += e_prev;\n"
            "        pack_pair(pa, 30, e_prev2, e_prev);\n")

    if split is not None:  # (product source) phase A runs S half 0 then S half 1; the softmax of half 0 moves into
        # phase A beside the half-1 MFMAs, so phase B carries only half 1's softmax (one score per two PV MFMAs).
        # split == "spread": the 16 LDS-DMA pieces one per two S MFMAs; "first": one per MFMA of half 0.
        start = src.index("    auto phase_a = [&](auto kb_, auto dkb_, auto dvb_, auto dma_, int tk, bool k_live, int tv, bool v_live) {")
        end = src.index("    // softmax of key e (0..31")
        dma_at = ("(i & 1) == 0" if split == "spread" else "i < 16")
        dma_idx = ("(i >> 1)" if split == "spread" else "i")
        new_a = """    float e_carry = 0.f;  // p of the last softmax score: the row sum adds it one score late (same adds, same order)
    auto softmax_elem2 = [&](u32x4 (&pn)[4], int e) {  // score e (0..31: half e >> 4, row e & 15) into P^T pn
      const f32x16& sacc = e < 16 ? s0 : s1;
      const int r = e & 15;
      const float v = __builtin_amdgcn_exp2f(sacc[r]);
      l_run += e_carry;
      if (e & 1) {
        const bf16x2 pr = {(__bf16)e_carry, (__bf16)v};
        pn[(e >> 4) * 2 + (r >> 3)][(r & 7) >> 1] = __builtin_bit_cast(unsigned, pr);
      }
      e_carry = v;
    };
    auto phase_a = [&](auto kb_, auto dkb_, auto dvb_, auto dma_, u32x4 (&pn)[4], int tk, bool k_live, int tv,
                       bool v_live) {
      constexpr int KB = decltype(kb_)::value, DKB = decltype(dkb_)::value, DVB = decltype(dvb_)::value;
      constexpr bool DMA = decltype(dma_)::value;
      const char* Kb = kbase + KB * TILE;
      i32x4 krs = {0, 0, 0, 0}, vrs = {0, 0, 0, 0};
      if constexpr (DMA) {
        krs = rsrc_tile(k_ptr0, k_tile_b, k_total_b, tk, k_live);
        vrs = rsrc_tile(v_ptr0, v_tile_b, v_total_b, tv, v_live);
      }
      bf16x8 kf[32];  // step i: S half i >> 4, k-step i & 15
      auto rdk = [&](int i) { kf[i] = *(const bf16x8*)(Kb + (i >> 4) * 32 * 512 + k_off[i & 15]); };
#pragma unroll
      for (int i = 0; i < KAHEAD; ++i) rdk(i);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        if (i + KAHEAD < 32) rdk(i + KAHEAD);
        __builtin_amdgcn_sched_barrier(0);
        if (i == 0)
          mfma_s_first(s0, kf[0], qf[0]);
        else if (i == 16)
          mfma_s_first(s1, kf[16], qf[0]);
        else if (i < 16)
          mfma_s(s0, kf[i], qf[i]);
        else
          mfma_s(s1, kf[i], qf[i - 16]);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (DMA) {
          if (""" + dma_at + """) {
            const int q = """ + dma_idx + """;
            if (q < 8)
              blds16(krs, k_src[q], lds0 + DKB * TILE + (wave * 8 + q) * 1024 + K_OFF);
            else
              blds16(vrs, v_src[q - 8], lds0 + DVB * TILE + (wave * 8 + q - 8) * 1024 + V_OFF);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        if (i == 16) mfma_read_fence1(s0);  // the last half-0 MFMA -> its VALU readers below
        if (i >= 16) softmax_elem2(pn, i - 16);
        __builtin_amdgcn_sched_barrier(0);
      }
      mfma_read_fence1(s1);  // MFMA write of S half 1 -> VALU read (softmax in the next phase B)
    };
"""
        src = src[:start] + new_a + src[end:]
        sub("""__device__ __forceinline__ void o_acc_fence(""", """__device__ __forceinline__ void mfma_read_fence1(f32x16& a) {
  asm volatile("s_nop 7\\n\\ts_nop 7\\n\\ts_nop 3" : "+v"(a));
}
__device__ __forceinline__ void o_acc_fence(""")
        # phase B: only half 1's scores, one per two PV MFMAs
        sub("        if constexpr (EX) softmax_elem(pn, m, e_prev);\n", "        if constexpr (EX) {\n          if ((m & 1) == 0) softmax_elem2(pn, 16 + (m >> 1));\n        }\n")
        sub("      if constexpr (EX) l_run += e_prev;\n", "")
        sub("          phase_a(I1{}, I0{}, I1{}, BT{}, t_begin + j + 2, j + 2 < nt, t_begin + j + 1, true);",
            "          phase_a(I1{}, I0{}, I1{}, BT{}, pb, t_begin + j + 2, j + 2 < nt, t_begin + j + 1, true);")
        sub("          phase_a(I0{}, I1{}, I0{}, BT{}, t_begin + j + 2, j + 2 < nt, t_begin + j + 1, true);",
            "          phase_a(I0{}, I1{}, I0{}, BT{}, pa, t_begin + j + 2, j + 2 < nt, t_begin + j + 1, true);")
        sub("""      phase_a(I0{}, I0{}, I0{}, BF{}, 0, false, 0, false);
      {
        float e_prev = 0.f;
#pragma unroll
        for (int e = 0; e < 32; ++e) softmax_elem(pa, e, e_prev);
        l_run += e_prev;
      }""", """      phase_a(I0{}, I0{}, I0{}, BF{}, pa, 0, false, 0, false);
#pragma unroll
      for (int e = 16; e < 32; ++e) softmax_elem2(pa, e);""")
        sub("  } else if (nt > 0) {\n    stage(t_begin, 0);", "    l_run += e_carry;\n  } else if (nt > 0) {\n    stage(t_begin, 0);")
    if vdma_b is not None:
        sub('''    auto phase_b = [&](auto vb_, auto ex_, u32x4 (&pc)[4], u32x4 (&pn)[4]) {
      constexpr int VB = decltype(vb_)::value;
      constexpr bool EX = decltype(ex_)::value;''', '''    auto phase_b = [&](auto vb_, auto ex_, u32x4 (&pc)[4], u32x4 (&pn)[4], int tv) {
      constexpr int VB = decltype(vb_)::value;
      constexpr bool EX = decltype(ex_)::value;
      i32x4 vrs2 = {0, 0, 0, 0};
      if constexpr (EX) vrs2 = ''' + ("rsrc_tile(v_ptr0, v_tile_b, v_total_b, tv, true);" if "v_ptr0" in src else
                                   "rsrc_tile(p.v, v_base, p.v_row_stride, tv, true);"))
        sub('''        if (dt == 0)
          mfma_o<true>(o_acc[dt], vf, pk);
        else
          mfma_o<false>(o_acc[dt], vf, pk);
        __builtin_amdgcn_sched_barrier(0);''', '''        if (dt == 0)
          mfma_o<true>(o_acc[dt], vf, pk);
        else
          mfma_o<false>(o_acc[dt], vf, pk);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (EX) {
          if ((m & 3) == ''' + str(int(vdma_b)) + ''')
            blds16(vrs2, v_src[m >> 2], lds0 + (VB ^ 1) * TILE + (wave * 8 + (m >> 2)) * 1024 + V_OFF);
        }
        __builtin_amdgcn_sched_barrier(0);''')
        sub("        phase_b(I0{}, hs_, pa, pb);", "        phase_b(I0{}, hs_, pa, pb, t_begin + j + 1);")
        sub("        phase_b(I1{}, hs_, pb, pa);", "        phase_b(I1{}, hs_, pb, pa, t_begin + j + 1);")
    out = HERE / "variants" / "_src"
    out.mkdir(parents=True, exist_ok=True)
    f = out / f"attention_{name}.hip"
    f.write_text(src)
    subprocess.run([sys.executable, str(HERE / "variants.py"), "build", "attention", name, "--from", str(f)],
                   check=True)


if __name__ == "__main__":
    a = sys.argv[1:]
    name = a[0]
    vb = None
    if "--vdma-b" in a:
        vb = int(a[a.index("--vdma-b") + 1])
    make(name, kspread="--kspread" in a, vdma_b=vb, qlate="--qlate" in a, packdelay="--packdelay" in a,
         split=a[a.index("--split") + 1] if "--split" in a else None)
