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
"""
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent


def make(name, kspread=False, vdma_b=None, qscale=False, ldelay=False, qlate=False, packdelay=False):
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
    if qscale:  # bounded path: Q^T pre-scaled by scale*log2(e) at load (one bf16 rounding, as q's own), no shift:
        # p = exp2(s'), one v_exp per score instead of v_fma + v_exp (|s'| <= 23.8: p in [2^-23.8, 2^23.8])
        sub("    for (int s = 0; s < 16; ++s) qf[s] = *(const bf16x8*)(qp + 16 * s);\n",
            "    for (int s = 0; s < 16; ++s) qf[s] = *(const bf16x8*)(qp + 16 * s);\n"
            "    if constexpr (BOUNDED) {\n"
            "      const float qs = p.scale * 1.4426950408889634f;\n"
            "#pragma unroll\n"
            "      for (int s = 0; s < 16; ++s)\n"
            "#pragma unroll\n"
            "        for (int j = 0; j < 8; ++j) qf[s][j] = (__bf16)((float)qf[s][j] * qs);\n"
            "    }\n")
        sub("  float m_run = BOUNDED ? p.max_score * 1.4426950408889634f : -1e30f;",
            "  float m_run = BOUNDED ? 0.f : -1e30f;")
        sub("      const float v = __builtin_amdgcn_exp2f(sacc[r] * sl2 - m_run);",
            "      const float v = __builtin_amdgcn_exp2f(sacc[r]);")
    if ldelay:  # row sum: add the PREVIOUS element's p (same adds, same order: bit-identical), so the v_add no
        # longer waits on the v_exp just issued (the trans -> VALU forwarding hazard cost an s_nop per element)
        sub("      l_run += v;\n      if (e & 1) {", "      l_run += e_prev;\n      if (e & 1) {")
        sub("        if constexpr (EX) softmax_elem(pn, m, e_prev);\n        __builtin_amdgcn_sched_barrier(0);\n      }\n",
            "        if constexpr (EX) softmax_elem(pn, m, e_prev);\n        __builtin_amdgcn_sched_barrier(0);\n      }\n"
            "      if constexpr (EX) l_run += e_prev;\n")
        sub("        for (int e = 0; e < 32; ++e) softmax_elem(pa, e, e_prev);\n",
            "        for (int e = 0; e < 32; ++e) softmax_elem(pa, e, e_prev);\n        l_run += e_prev;\n")
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
    make(name, kspread="--kspread" in a, vdma_b=vb, qscale="--qscale" in a, ldelay="--ldelay" in a,
         qlate="--qlate" in a, packdelay="--packdelay" in a)
