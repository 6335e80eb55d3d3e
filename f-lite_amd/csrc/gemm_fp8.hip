// MXFP8 GEMM for gfx950: e4m3 operands with E8M0 block scales on v_mfma_scale_f32_16x16x128_f8f6f4
// (twice the bf16 MFMA rate). The fp8 counterpart of gemm.hip for BASELINE.json configs[4] (fp8 weights and
// activations): qkv / cross-q / proj / cross-proj / SwiGLU gate-up / down of every DiTBlock (model.py:151-156,
// 261-267).
//
//   C[M,N] = dequant(A8)[M,K] . dequant(W8)[N,K]^T
//
// Same tile as the bf16 kernel: 256 (or 224) x 256 outputs, 512 threads = 8 waves as 2(M) x 4(N), W the MFMA A
// operand (so a lane's accumulator is 4 consecutive output columns of one row, as in gemm.hip's epilogues).
// A k-tile is 128 fp8 = 128 bytes per row: the LDS image, the swizzle and the LDS-DMA staging are byte for byte
// those of the bf16 kernel's 64-deep k-tile, and each (mi, ni) pair takes ONE 16x16x128 MFMA per k-tile (32
// cycles) where bf16 takes two 16x16x32 (16 cycles each): the same MFMA cycles per k-tile for twice the depth.
// Per k-tile the 4 block scales of 256 rows (one 32-bit word per row, "k-tile major" scale arrays, fp8.hip) come
// in with ONE extra 1-KiB LDS-DMA piece per operand.
//
// Operand lane maps, measured on MI355X with exact integer data (tools/mfma_fp8_probe.py): lane l holds row
// (l & 15) and K bytes [16 (l >> 4), +16) in its bytes 0-15 and [64 + 16 (l >> 4), +16) in bytes 16-31 -- i.e.
// 16-B chunks (l >> 4) and 4 + (l >> 4) of the 128-B row, the two chunks the bf16 kernel reads for its two
// k-steps -- and its scale operand (byte 0, op_sel 0) is the scale of the row's 32-block (l >> 4).
#include <cstdlib>

#include "fp8.h"
#include "kernels.h"
#include "stream_k.h"

namespace flite {

namespace {

constexpr int BN = 256;
constexpr int NT = 512;
constexpr int TILE_BYTES = 256 * 128;        // one operand k-tile (256 rows x 128 B)
constexpr int W_REGION = 2 * TILE_BYTES;
constexpr int SC_REGION = 4 * TILE_BYTES;    // [As buf0 | As buf1 | Ws buf0 | Ws buf1], 1 KiB each
constexpr int LDS_BYTES = 4 * TILE_BYTES + 4 * 1024;  // 132 KiB

typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((ext_vector_type(8))) int i32x8;

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ i32x4 make_rsrc(const void* base, unsigned bytes) {
  const unsigned long long a = (unsigned long long)base;
  i32x4 r;
  r.x = __builtin_amdgcn_readfirstlane((int)(a & 0xffffffffu));
  r.y = __builtin_amdgcn_readfirstlane((int)(a >> 32));
  r.z = __builtin_amdgcn_readfirstlane((int)bytes);
  r.w = 0x00020000;
  return r;
}

__device__ __forceinline__ unsigned lds_addr_of(const void* p) {
  return (unsigned)(unsigned long long)(const LDS_AS char*)p;
}

// One k-tile of LDS-DMA for this wave (as gemm.hip stage_dma): 4 A + 4 W pieces of 1 KiB, plus `sc` (0/1) scale
// pieces: wave 0 copies the A scales, wave 1 the W scales. One asm block (hipcc would otherwise wait vmcnt(0)
// before every LDS read); `skip` (uniform) makes it a no-op.
__device__ __forceinline__ void stage_dma8(const i32x4& ra, unsigned sa, unsigned va0, unsigned va1, unsigned va2,
                                           unsigned va3, const i32x4& rw, unsigned sw, unsigned vw0, unsigned vw1,
                                           unsigned vw2, unsigned vw3, unsigned lds_a, unsigned lds_w,
                                           const i32x4& rs, unsigned ss, unsigned vs, unsigned lds_s, unsigned has_s,
                                           unsigned skip) {
  unsigned keep;
  asm volatile(
      "s_cmp_eq_u32 %[skip], 0\n\t"
      "s_cbranch_scc0 .Lskip_dma8_%=\n\t"
      "s_mov_b32 %[keep], m0\n\t"
      "s_mov_b32 m0, %[la]\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[va0], %[ra], %[sa] offen lds\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[va1], %[ra], %[sa] offen lds\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[va2], %[ra], %[sa] offen lds\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[va3], %[ra], %[sa] offen lds\n\t"
      "s_mov_b32 m0, %[lw]\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[vw0], %[rw], %[sw] offen lds\n\t"
      "s_add_u32 m0, m0, 0x2000\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[vw1], %[rw], %[sw] offen lds\n\t"
      "s_add_u32 m0, m0, 0x2000\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[vw2], %[rw], %[sw] offen lds\n\t"
      "s_add_u32 m0, m0, 0x2000\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[vw3], %[rw], %[sw] offen lds\n\t"
      "s_cmp_eq_u32 %[hs], 0\n\t"
      "s_cbranch_scc1 .Lno_sc8_%=\n\t"
      "s_mov_b32 m0, %[ls]\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[vs], %[rs], %[ss] offen lds\n"
      ".Lno_sc8_%=:\n\t"
      "s_mov_b32 m0, %[keep]\n"
      ".Lskip_dma8_%=:"
      : [keep] "=&s"(keep)
      : [skip] "s"(skip), [la] "s"(lds_a), [lw] "s"(lds_w), [ra] "s"(ra), [sa] "s"(sa), [rw] "s"(rw), [sw] "s"(sw),
        [va0] "v"(va0), [va1] "v"(va1), [va2] "v"(va2), [va3] "v"(va3), [vw0] "v"(vw0), [vw1] "v"(vw1),
        [vw2] "v"(vw2), [vw3] "v"(vw3), [rs] "s"(rs), [ss] "s"(ss), [vs] "v"(vs), [ls] "s"(lds_s), [hs] "s"(has_s)
      : "memory", "scc");
}

template <int EPI, int MI>
struct Fp8Cta {
  static constexpr int WM = MI * 16;
  const GemmFp8Params& p;
  int tid, lane, wave, wave_m, wave_n, lr, lk;
  unsigned lds0;
  i32x4 a_rsrc, w_rsrc, s_rsrc;
  unsigned ab, wb;        // per-lane LDS byte address of this lane's row base + chunk lk (buffer 0)
  unsigned ab2, wb2;      // ... chunk 4 + lk
  unsigned asb, wsb;      // per-lane scale byte address (buffer 0): row * 4 + lk
  unsigned a_off[4], w_off[4], s_off;
  unsigned s_stride;      // bytes between consecutive k-tiles of this wave's scale array
  int ke;

  __device__ __forceinline__ Fp8Cta(const GemmFp8Params& p_, char* smem) : p(p_) {
    tid = threadIdx.x;
    lane = tid & 63;
    wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    wave_m = wave >> 2;
    wave_n = wave & 3;
    lr = lane & 15;
    lk = lane >> 4;
    lds0 = (unsigned)__builtin_amdgcn_readfirstlane((int)lds_addr_of(smem));
    a_rsrc = make_rsrc(p.A, (unsigned)((long)p.M * p.lda));
    w_rsrc = make_rsrc(p.W, (unsigned)((long)p.N * p.ldw));
    const int nkt = p.K / 128;
    // wave 0 stages A scales, wave 1 W scales (uniform choice)
    if (wave == 0) {
      s_rsrc = make_rsrc(p.As, (unsigned)((long)nkt * p.a_rows_pad * 4));
      s_stride = (unsigned)(p.a_rows_pad * 4);
    } else {
      s_rsrc = make_rsrc(p.Ws, (unsigned)((long)nkt * p.w_rows_pad * 4));
      s_stride = (unsigned)(p.w_rows_pad * 4);
    }
    const unsigned c0 = ((lk) ^ swz(lr)) << 4, c1 = ((4 + lk) ^ swz(lr)) << 4;
    ab = lds0 + (wave_m * WM + lr) * 128 + c0;
    ab2 = lds0 + (wave_m * WM + lr) * 128 + c1;
    wb = lds0 + W_REGION + (wave_n * 64 + lr) * 128 + c0;
    wb2 = lds0 + W_REGION + (wave_n * 64 + lr) * 128 + c1;
    asb = lds0 + SC_REGION + (wave_m * WM + lr) * 4 + lk;
    wsb = lds0 + SC_REGION + 2048 + (wave_n * 64 + lr) * 4 + lk;
  }

  __device__ __forceinline__ void setup_tile(int m0, int n0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      {
        const int row = (wave * 4 + i) * 8 + (lane >> 3);
        const int chunk = (lane & 7) ^ swz(row);
        const int am = min(m0 + row, p.M - 1);
        a_off[i] = (unsigned)((long)am * p.lda + chunk * 16);
        // 224-row tiles: rows 224-255 are never read; an out-of-range offset moves no bytes (gemm.hip setup_tile)
        if (MI == 7 && wave == 7 && (long)p.M * p.lda <= 0x7fffffffL) a_off[i] = 0x80000000u;
      }
      {
        const int row = (wave + 8 * i) * 8 + (lane >> 3);
        const int chunk = (lane & 7) ^ swz(row);
        const int wn = min(n0 + row, p.N - 1);
        w_off[i] = (unsigned)((long)wn * p.ldw + chunk * 16);
      }
    }
    // scale piece: rows r0 .. r0 + 255 of k-tile 0 (one 32-bit word per row, 16 B = 4 rows per lane)
    s_off = (unsigned)(((wave == 0 ? m0 : n0) + lane * 4) * 4);
  }

  __device__ __forceinline__ void stage(int kt, int buf) {
    const unsigned la = (unsigned)__builtin_amdgcn_readfirstlane((int)(lds0 + buf * TILE_BYTES + wave * 4096));
    const unsigned lw =
        (unsigned)__builtin_amdgcn_readfirstlane((int)(lds0 + W_REGION + buf * TILE_BYTES + wave * 1024));
    const unsigned ls = (unsigned)__builtin_amdgcn_readfirstlane(
        (int)(lds0 + SC_REGION + (wave == 0 ? 0 : 2048) + buf * 1024));
    const unsigned kb = (unsigned)(kt * 128);
    const unsigned sk = (unsigned)__builtin_amdgcn_readfirstlane((int)(kt * s_stride));
    stage_dma8(a_rsrc, kb, a_off[0], a_off[1], a_off[2], a_off[3], w_rsrc, kb, w_off[0], w_off[1], w_off[2],
               w_off[3], la, lw, s_rsrc, sk, s_off, ls, (unsigned)__builtin_amdgcn_readfirstlane(wave < 2 ? 1 : 0),
               (unsigned)__builtin_amdgcn_readfirstlane(kt >= ke ? 1 : 0));
  }

  template <int BUF>
  __device__ __forceinline__ i32x8 rd_w(int ni) const {
    const i32x4 lo = *(const LDS_AS i32x4*)(wb + BUF * TILE_BYTES + ni * 16 * 128);
    const i32x4 hi = *(const LDS_AS i32x4*)(wb2 + BUF * TILE_BYTES + ni * 16 * 128);
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  }
  template <int BUF>
  __device__ __forceinline__ i32x8 rd_a(int mi) const {
    const i32x4 lo = *(const LDS_AS i32x4*)(ab + BUF * TILE_BYTES + mi * 16 * 128);
    const i32x4 hi = *(const LDS_AS i32x4*)(ab2 + BUF * TILE_BYTES + mi * 16 * 128);
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  }
  template <int BUF>
  __device__ __forceinline__ int rd_ws(int ni) const {
    return (int)*(const LDS_AS unsigned char*)(wsb + BUF * 1024 + ni * 16 * 4);
  }
  template <int BUF>
  __device__ __forceinline__ int rd_as(int mi) const {
    return (int)*(const LDS_AS unsigned char*)(asb + BUF * 1024 + mi * 16 * 4);
  }

  __device__ __forceinline__ static void mfma2(f32x4 (&acc)[8][4], const i32x8 (&wf)[4], const int (&ws)[4],
                                               const i32x8& a0, int s0, const i32x8& a1, int s1, int mi0) {
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      if (mi0 < MI)
        acc[mi0][ni] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wf[ni], a0, acc[mi0][ni], 0, 0, 0, ws[ni],
                                                                         0, s0);
      if (mi0 + 1 < MI)
        acc[mi0 + 1][ni] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wf[ni], a1, acc[mi0 + 1][ni], 0, 0, 0,
                                                                             ws[ni], 0, s1);
    }
  }

  // One 128-deep k-tile from buffer BUF. On entry: wf/ws = W fragments and scales of this tile, a0/a1 (+scales)
  // = A fragments of mi 0, 1. Quarter q runs the MFMAs of mi 2q, 2q+1 while the next pair is read; after the
  // third quarter every read of BUF is done: wait for the next tile's copies, barrier, restage BUF with tile
  // kt + 2 (waves 0-3 here, 4-7 after the last quarter), and the last quarter reads the next tile's W and
  // A(0, 1) from BUF ^ 1.
  template <int BUF>
  __device__ __forceinline__ void ktile(f32x4 (&acc)[8][4], i32x8 (&wf)[4], int (&ws)[4], i32x8& a0, int& s0,
                                        i32x8& a1, int& s1, int kt) {
    i32x8 b0, b1;
    int t0, t1;
    // q0: mi 0,1 | read mi 2,3
    b0 = rd_a<BUF>(2);
    b1 = MI > 3 ? rd_a<BUF>(3) : b0;
    t0 = rd_as<BUF>(2);
    t1 = MI > 3 ? rd_as<BUF>(3) : t0;
    mfma2(acc, wf, ws, a0, s0, a1, s1, 0);
    // q1: mi 2,3 | read mi 4,5
    a0 = rd_a<BUF>(4);
    a1 = MI > 5 ? rd_a<BUF>(5) : a0;
    s0 = rd_as<BUF>(4);
    s1 = MI > 5 ? rd_as<BUF>(5) : s0;
    mfma2(acc, wf, ws, b0, t0, b1, t1, 2);
    // q2: mi 4,5 | read mi 6,7
    b0 = rd_a<BUF>(6);
    b1 = MI > 7 ? rd_a<BUF>(7) : b0;
    t0 = rd_as<BUF>(6);
    t1 = MI > 7 ? rd_as<BUF>(7) : t0;
    mfma2(acc, wf, ws, a0, s0, a1, s1, 4);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    stage(wave_m == 0 ? kt + 2 : ke, BUF);
    // q3: mi 6,7 | read the next tile's W (+scales) and A(0, 1) from BUF ^ 1
    {
      i32x8 wn[4];
      int wsn[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        wn[ni] = rd_w<BUF ^ 1>(ni);
        wsn[ni] = rd_ws<BUF ^ 1>(ni);
      }
      a0 = rd_a<BUF ^ 1>(0);
      a1 = rd_a<BUF ^ 1>(1);
      s0 = rd_as<BUF ^ 1>(0);
      s1 = rd_as<BUF ^ 1>(1);
      mfma2(acc, wf, ws, b0, t0, b1, t1, 6);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        wf[ni] = wn[ni];
        ws[ni] = wsn[ni];
      }
    }
    stage(wave_m == 1 ? kt + 2 : ke, BUF);
  }

  // acc = the k-tiles [kb, kend) of the tile set up by setup_tile
  __device__ __forceinline__ void mainloop(f32x4 (&acc)[8][4], int kb, int kend) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    ke = kend;
    // the previous tile's last reads / DMA of this workgroup must be done before the buffers are refilled
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    stage(kb, 0);
    stage(kb + 1, 1);
    // this wave's copies of tile kb are the oldest: leave kb+1's (8, +1 scale piece for waves 0, 1) in flight
    if (kend - kb <= 1)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (wave < 2)
      asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    i32x8 wf[4], a0, a1;
    int ws[4], s0, s1;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      wf[ni] = rd_w<0>(ni);
      ws[ni] = rd_ws<0>(ni);
    }
    a0 = rd_a<0>(0);
    a1 = rd_a<0>(1);
    s0 = rd_as<0>(0);
    s1 = rd_as<0>(1);
    int kt = kb;
    for (; kt + 1 < kend; kt += 2) {
      ktile<0>(acc, wf, ws, a0, s0, a1, s1, kt);
      ktile<1>(acc, wf, ws, a0, s0, a1, s1, kt + 1);
    }
    if (kt < kend) ktile<0>(acc, wf, ws, a0, s0, a1, s1, kt);
  }

  // RoPE + QK-norm, as gemm.hip's qkv_norm_epilogue: RoPE tiles (n0 < rope_cols) hold the q/k heads in rope_perm
  // column order (the fp8 weight rows were quantised in that order), so each lane rotates its pairs in registers;
  // the per-head RMSNorm sums squares over 4 lanes and the 4 wave_n waves (LDS partials); one bf16 rounding.
  __device__ __forceinline__ void qkv_norm_epilogue(f32x4 (&acc)[8][4], int n0, int m_base, int n_base) {
    const bool rope = n0 < p.rope_cols;  // tile-uniform
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n_base + ni * 16 + r;
        const float b = (p.bias != nullptr && n < p.N) ? bf2f(p.bias[rope ? rope_perm(n) : n]) : 0.f;
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) acc[mi][ni][r] += b;
      }
    if (n0 < p.norm_cols) {
      if (rope) rope_rotate<MI>(acc, p.rope, m_base, p.M, wave_n, lk);
      __syncthreads();  // every wave is done with the k-tile buffers
      const unsigned sums = lds0 + 65536;
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        float ss = 0.f;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
#pragma unroll
          for (int r = 0; r < 4; ++r) ss += acc[mi][ni][r] * acc[mi][ni][r];
        ss += __shfl_xor(ss, 16, 64);
        ss += __shfl_xor(ss, 32, 64);
        if (lk == 0) *(LDS_AS float*)(sums + (((wave_m * 8 + mi) * 16 + lr) * 4 + wave_n) * 4) = ss;
      }
      __syncthreads();
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        const f32x4 part = *(const LDS_AS f32x4*)(sums + ((wave_m * 8 + mi) * 16 + lr) * 16);
        const float rn = rsqrtf((part[0] + part[1] + part[2] + part[3]) * (1.f / 256.f) + p.norm_eps);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[mi][ni][r] *= rn;
      }
    }
    const bool wide = wide_ok();  // N % 256 == 0: no column tail
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const int m = m_base + mi * 16;
      u32x2 pk[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        pk[ni].x = pack2bf(acc[mi][ni][0], acc[mi][ni][1]);
        pk[ni].y = pack2bf(acc[mi][ni][2], acc[mi][ni][3]);
      }
      bf16_t* orow = (bf16_t*)p.out + (long)m * p.ldo;
      if (wide) {  // common.h deal8: 16-B pieces
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const u32x4 w = deal8(pk[2 * q], pk[2 * q + 1]);
          if (m < p.M) *(u32x4*)(orow + n_base - lk * 4 + 32 * q + deal8_col(lk)) = w;
        }
      } else if (m < p.M) {
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) *(u32x2*)(orow + n_base + ni * 16) = pk[ni];
      }
    }
  }
  // 16-B bf16 stores are legal when every row start is 16-B aligned
  __device__ __forceinline__ bool wide_ok() const { return (p.ldo & 7) == 0 && ((uintptr_t)p.out & 15) == 0; }

  // ---- epilogues: lane holds C[m][n..n+3], m = m_base + mi*16, n = n_base + ni*16 (gemm.hip layout) ----
  __device__ __forceinline__ void epilogue(f32x4 (&acc)[8][4], int m0, int n0) {
    const int m_base = m0 + wave_m * WM + lr;
    const int n_base = n0 + wave_n * 64 + lk * 4;
    if constexpr (EPI == EPI8_SWIGLU_FP8) {
      // gate (ni 0, 2) / up (ni 1, 3) pairs -> this wave's 32 output columns = ONE 32-block of h
      const int F = p.N >> 1;
      const int oc0 = (n0 >> 1) + wave_n * 32;  // first column of the block
      if (oc0 >= F) return;
      const int blk = oc0 >> 5;
      uint8_t* o8 = (uint8_t*)p.out;
      const bool wide = (p.ldo & 7) == 0 && ((uintptr_t)p.out & 7) == 0;
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        const int m = m_base + mi * 16;
        float h[8];
#pragma unroll
        for (int pr = 0; pr < 2; ++pr)
#pragma unroll
          for (int r = 0; r < 4; ++r) h[4 * pr + r] = silu_f(acc[mi][2 * pr][r]) * acc[mi][2 * pr + 1][r];
        float amax = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(h[j]));
        amax = fmaxf(amax, __shfl_xor(amax, 16, 64));
        amax = fmaxf(amax, __shfl_xor(amax, 32, 64));
        const int e = mx_exp(amax);
        const float inv = mx_inv(e);
        const unsigned lo = pack4_fp8(h, inv), hi = pack4_fp8(h + 4, inv);  // columns 4 lk .. and 16 + 4 lk ..
        if (wide) {  // common.h deal8: one 8-B piece per row instead of two 4-B pieces
          const u32x2 w = deal8(lo, hi);
          if (m < p.M) *(u32x2*)(o8 + (long)m * p.ldo + oc0 + deal8_col(lk)) = w;
        } else if (m < p.M) {
          uint8_t* orow = o8 + (long)m * p.ldo + oc0 + lk * 4;
          *(unsigned*)(orow) = lo;
          *(unsigned*)(orow + 16) = hi;
        }
        if (m < p.M && lk == 0) p.out_sc[((long)(blk >> 2) * p.out_rows_pad + m) * 4 + (blk & 3)] = (uint8_t)(e + 127);
      }
      return;
    } else if constexpr (EPI == EPI8_SWIGLU_BF16) {
      // the same gate/up pairs, h rounded to bf16: columns oc0 + 4 lk .. + 3 and oc0 + 16 + 4 lk .. + 3 of the row
      const int F = p.N >> 1;
      const int oc0 = (n0 >> 1) + wave_n * 32;
      if (oc0 >= F) return;
      bf16_t* ob = (bf16_t*)p.out;
      const bool wide = (F & 7) == 0 && wide_ok();  // an 8-column piece is inside or outside [0, F)
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        const int m = m_base + mi * 16;
        float h[8];
#pragma unroll
        for (int pr = 0; pr < 2; ++pr)
#pragma unroll
          for (int r = 0; r < 4; ++r) h[4 * pr + r] = silu_f(acc[mi][2 * pr][r]) * acc[mi][2 * pr + 1][r];
        const u32x2 lo = {pack2bf(h[0], h[1]), pack2bf(h[2], h[3])}, hi = {pack2bf(h[4], h[5]), pack2bf(h[6], h[7])};
        if (wide) {  // common.h deal8: one 16-B piece per row instead of two 8-B pieces
          const u32x4 w = deal8(lo, hi);
          const int oc = oc0 + deal8_col(lk);
          if (m < p.M && oc < F) *(u32x4*)(ob + (long)m * p.ldo + oc) = w;
        } else if (m < p.M) {
          bf16_t* orow = ob + (long)m * p.ldo + oc0 + lk * 4;
          *(u32x2*)(orow) = lo;
          *(u32x2*)(orow + 16) = hi;
        }
      }
      return;
    } else if constexpr (EPI == EPI8_RESID_F32 || EPI == EPI8_RESID_BF16) {
      constexpr bool X16 = EPI == EPI8_RESID_BF16;  // bf16 residual stream: one rounding at the store
      constexpr int XB = X16 ? 2 : 4;
      float bias[4][4];
      int nc[4];
      bool nok[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int n = n_base + ni * 16;
        nok[ni] = n < p.N;
        nc[ni] = nok[ni] ? n : 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) bias[ni][r] = (p.bias != nullptr && nok[ni]) ? bf2f(p.bias[nc[ni] + r]) : 0.f;
      }
      if constexpr (X16) {
        // 16-B lanes in the deal8 layout (gemm.hip resid_epilogue WIDE): same values, half the x instructions;
        // two rows' loads issued before their stores, as below
        if ((p.N & 7) == 0 && wide_ok() && !p.resid_narrow) {
#pragma unroll
          for (int mb = 0; mb < 8; mb += 2) {
            unsigned xw[2][2][4];  // [row][q][dword], accumulator layout after the inverse deal
            f32x4 gv[2][4];
            char* orow[2];
            bool mok[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
              const int m = m_base + (mb + i) * 16;
              mok[i] = mb + i < MI && m < p.M;
              const int mc = mok[i] ? m : p.M - 1;
              orow[i] = (char*)p.out + (long)mc * p.ldo * XB;
              const float* grow = p.gate + (long)(mc / p.rows_per_seg) * p.gate_seg_stride;
#pragma unroll
              for (int ni = 0; ni < 4; ++ni)
                gv[i][ni] = p.gate ? *(const f32x4*)(grow + nc[ni]) : f32x4{1.f, 1.f, 1.f, 1.f};
#pragma unroll
              for (int q = 0; q < 2; ++q) {
                const int pc = n_base - lk * 4 + 32 * q + deal8_col(lk);
                const u32x4 w = *(const u32x4*)(orow[i] + (pc < p.N ? pc : 0) * XB);
                const auto t = __builtin_amdgcn_permlane16_swap(w.x, w.z, false, false);  // deal8's inverse
                const auto u = __builtin_amdgcn_permlane16_swap(w.y, w.w, false, false);
                xw[i][q][0] = t[0], xw[i][q][1] = u[0], xw[i][q][2] = t[1], xw[i][q][3] = u[1];
              }
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
              for (int q = 0; q < 2; ++q) {
                u32x2 pk[2];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                  const int ni = 2 * q + h;
                  const unsigned lo = xw[i][q][2 * h], hi = xw[i][q][2 * h + 1];
                  f32x4 x = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                             __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
#pragma unroll
                  for (int r = 0; r < 4; ++r) x[r] += (acc[mb + i][ni][r] + bias[ni][r]) * gv[i][ni][r];
                  pk[h] = u32x2{pack2bf(x[0], x[1]), pack2bf(x[2], x[3])};
                }
                const u32x4 o = deal8(pk[0], pk[1]);  // every lane takes part; only the store is masked
                const int pc = n_base - lk * 4 + 32 * q + deal8_col(lk);
                if (mok[i] && pc < p.N) *(u32x4*)(orow[i] + pc * XB) = o;
              }
          }
          return;
        }
      }
#pragma unroll
      for (int mb = 0; mb < 8; mb += 2) {
        f32x4 xv[2][4], gv[2][4];
        char* orow[2];
        bool mok[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int m = m_base + (mb + i) * 16;
          mok[i] = mb + i < MI && m < p.M;
          const int mc = mok[i] ? m : p.M - 1;
          orow[i] = (char*)p.out + (long)mc * p.ldo * XB;
          const float* grow = p.gate + (long)(mc / p.rows_per_seg) * p.gate_seg_stride;
#pragma unroll
          for (int ni = 0; ni < 4; ++ni) {
            if constexpr (X16) {
              const u32x2 w = *(const u32x2*)(orow[i] + nc[ni] * XB);
              xv[i][ni] = f32x4{__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                                __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u)};
            } else {
              xv[i][ni] = *(const f32x4*)(orow[i] + nc[ni] * XB);
            }
            gv[i][ni] = p.gate ? *(const f32x4*)(grow + nc[ni]) : f32x4{1.f, 1.f, 1.f, 1.f};
          }
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int ni = 0; ni < 4; ++ni) {
            f32x4 x = xv[i][ni];
#pragma unroll
            for (int r = 0; r < 4; ++r) x[r] += (acc[mb + i][ni][r] + bias[ni][r]) * gv[i][ni][r];
            if constexpr (X16) {
              if (mok[i] && nok[ni]) *(u32x2*)(orow[i] + nc[ni] * XB) = u32x2{pack2bf(x[0], x[1]), pack2bf(x[2], x[3])};
            } else {
              if (mok[i] && nok[ni]) *(f32x4*)(orow[i] + nc[ni] * XB) = x;
            }
          }
      }
      return;
    } else if constexpr (EPI == EPI8_QKV_NORM_BF16) {
      qkv_norm_epilogue(acc, n0, m_base, n_base);
      return;
    } else {  // EPI8_STORE_BF16
      float bias[4][4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = n_base + ni * 16 + r;
          bias[ni][r] = (p.bias != nullptr && n < p.N) ? bf2f(p.bias[n]) : 0.f;
        }
      const bool wide = (p.N & 7) == 0 && wide_ok();  // an 8-column group of deal8 is inside or outside [0, N)
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        const int m = m_base + mi * 16;
        u32x2 pk[4];
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const f32x4 v = acc[mi][ni];
          pk[ni].x = pack2bf(v[0] + bias[ni][0], v[1] + bias[ni][1]);
          pk[ni].y = pack2bf(v[2] + bias[ni][2], v[3] + bias[ni][3]);
        }
        bf16_t* orow = (bf16_t*)p.out + (long)m * p.ldo;
        if (wide) {
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const u32x4 w = deal8(pk[2 * q], pk[2 * q + 1]);
            const int n = n_base - lk * 4 + 32 * q + deal8_col(lk);
            if (m < p.M && n < p.N) *(u32x4*)(orow + n) = w;
          }
        } else if (m < p.M) {
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
            if (n_base + ni * 16 < p.N) *(u32x2*)(orow + n_base + ni * 16) = pk[ni];
        }
      }
    }
  }
};

template <int EPI, int MI>
__global__ __launch_bounds__(NT, 2) void gemm_fp8_kernel(GemmFp8Params p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using Cta = Fp8Cta<EPI, MI>;
  Cta c(p, smem);
  const int num_m = (p.M + Cta::WM * 2 - 1) / (Cta::WM * 2);
  const int num_n = (p.N + BN - 1) / BN;
  const int nk = p.K / 128;
  const int wg = sk::xcd_remap(blockIdx.x, gridDim.x);
  f32x4 acc[8][4];
  if constexpr (MI == 8) {
    if (p.sk_tiles > 0) {  // persistent grid, one workgroup per CU (launch8)
      sk::stream_k_body<NT>(c, acc, num_m, num_n, nk, wg);
      return;
    }
  }
  int m0, n0;
  sk::tile_origin(wg, num_m, num_n, m0, n0, Cta::WM * 2, BN);
  c.setup_tile(m0, n0);
  c.mainloop(acc, 0, nk);
  c.epilogue(acc, m0, n0);
}

int g_cus = 0;
bool g_attrs = false;
bool g_sk_ok = false;  // every workgroup of a one-per-CU grid is resident at once (stream-K waits on peers)

template <int EPI>
hipError_t set_attrs8() {
  hipError_t e = hipFuncSetAttribute((const void*)gemm_fp8_kernel<EPI, 8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     LDS_BYTES);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute((const void*)gemm_fp8_kernel<EPI, 7>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             LDS_BYTES);
}

int init8() {
  if (g_attrs) return 0;
  FLITE_HIP_CHECK(set_attrs8<EPI8_STORE_BF16>());
  FLITE_HIP_CHECK(set_attrs8<EPI8_RESID_F32>());
  FLITE_HIP_CHECK(set_attrs8<EPI8_RESID_BF16>());
  FLITE_HIP_CHECK(set_attrs8<EPI8_SWIGLU_FP8>());
  FLITE_HIP_CHECK(set_attrs8<EPI8_QKV_NORM_BF16>());
  FLITE_HIP_CHECK(set_attrs8<EPI8_SWIGLU_BF16>());
  int dev = 0;
  FLITE_HIP_CHECK(hipGetDevice(&dev));
  FLITE_HIP_CHECK(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev));
  int per_cu = 0;
  FLITE_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gemm_fp8_kernel<EPI8_RESID_F32, 8>, NT,
                                                              LDS_BYTES));
  g_sk_ok = per_cu >= 1;
  g_attrs = true;
  return 0;
}

// 224-row tiles where they take a large share of a round fewer rounds x tile size on the chip (gemm.hip use_bm224:
// the 256-row tile's fewer LDS-DMA pieces and LDS bytes per FLOP win smaller margins in the power-limited loop)
bool bm224(const GemmFp8Params& p) {
  if (g_cus <= 0) return false;
  const int num_n = (p.N + BN - 1) / BN;
  const int t256 = (p.M + 255) / 256 * num_n, t224 = (p.M + 223) / 224 * num_n;
  const double r256 = (double)((t256 + g_cus - 1) / g_cus), r224 = (double)((t224 + g_cus - 1) / g_cus) * 0.875;
  return r224 < 0.93 * r256;
}

template <int EPI>
void launch8(GemmFp8Params p, hipStream_t s) {
  if constexpr (EPI == EPI8_RESID_BF16) {
    static const bool narrow = getenv("FLITE_GEMM_RESID_NARROW") != nullptr;  // A/B switch for measurements
    p.resid_narrow = narrow;
  }
  const int num_n = (p.N + BN - 1) / BN;
  const int T = (p.M + 255) / 256 * num_n;
  p.sk_tiles = (p.sk_ws != nullptr && p.sk_flags != nullptr && g_sk_ok)
                   ? sk::choose_sk_tiles(T, p.K / 128, g_cus, &p.sk_wgs)
                   : 0;
  static const bool sk_always = getenv("FLITE_FP8_SK_ALWAYS") != nullptr;  // A/B switch for measurements
  if (sk_always && p.sk_ws != nullptr && p.sk_flags != nullptr && g_sk_ok && T % g_cus != 0 &&
      (long)(T % g_cus) * (p.K / 128) >= 2L * g_cus) {
    p.sk_tiles = T % g_cus;
    p.sk_wgs = g_cus;
  }
  if (p.sk_tiles) {
    hipLaunchKernelGGL((gemm_fp8_kernel<EPI, 8>), dim3(g_cus), dim3(NT), LDS_BYTES, s, p);
  } else if (bm224(p)) {
    hipLaunchKernelGGL((gemm_fp8_kernel<EPI, 7>), dim3((p.M + 223) / 224 * num_n), dim3(NT), LDS_BYTES, s, p);
  } else {
    hipLaunchKernelGGL((gemm_fp8_kernel<EPI, 8>), dim3((p.M + 255) / 256 * num_n), dim3(NT), LDS_BYTES, s, p);
  }
}

}  // namespace

int gemm_fp8(const GemmFp8Params& p, int epi, hipStream_t s) {
  FLITE_REQUIRE(p.M > 0 && p.N > 0 && p.K > 0, "gemm_fp8: empty problem");
  FLITE_REQUIRE(p.K % 128 == 0, "gemm_fp8: K must be a multiple of 128");
  FLITE_REQUIRE(p.lda % 16 == 0 && p.ldw % 16 == 0, "gemm_fp8: row strides must be multiples of 16 bytes");
  FLITE_REQUIRE(((uintptr_t)p.A & 15) == 0 && ((uintptr_t)p.W & 15) == 0 && ((uintptr_t)p.As & 15) == 0 &&
                    ((uintptr_t)p.Ws & 15) == 0,
                "gemm_fp8: operands and scales must be 16-B aligned");
  FLITE_REQUIRE(p.a_rows_pad >= mx_rows_pad(p.M) && p.w_rows_pad >= p.N && p.w_rows_pad % 256 == 0 &&
                    p.a_rows_pad % 256 == 0,
                "gemm_fp8: scale arrays must cover 256-row tiles (rows_pad multiple of 256, >= rows)");
  FLITE_REQUIRE((long)p.M * p.lda < (1L << 32) && (long)p.N * p.ldw < (1L << 32) &&
                    (long)(p.K / 128) * p.a_rows_pad * 4 < (1L << 32),
                "gemm_fp8: operands must be < 4 GiB (32-bit buffer offsets)");
  if (init8()) return 1;
  switch (epi) {
    case EPI8_STORE_BF16:
      FLITE_REQUIRE(p.N % 4 == 0 && p.ldo % 4 == 0, "gemm_fp8(store): N, ldo multiples of 4");
      launch8<EPI8_STORE_BF16>(p, s);
      break;
    case EPI8_RESID_F32:
      FLITE_REQUIRE(p.N % 4 == 0 && p.ldo % 4 == 0 && p.rows_per_seg > 0, "gemm_fp8(resid): N, ldo, rows_per_seg");
      launch8<EPI8_RESID_F32>(p, s);
      break;
    case EPI8_RESID_BF16:
      FLITE_REQUIRE(p.N % 4 == 0 && p.ldo % 4 == 0 && p.rows_per_seg > 0 && ((uintptr_t)p.out & 7) == 0,
                    "gemm_fp8(resid bf16): N, ldo, rows_per_seg, 8-B aligned rows");
      launch8<EPI8_RESID_BF16>(p, s);
      break;
    case EPI8_SWIGLU_FP8:
      FLITE_REQUIRE(p.N % 256 == 0, "gemm_fp8(swiglu): 2F must be a multiple of 256");
      FLITE_REQUIRE(p.out_sc != nullptr && p.out_rows_pad >= mx_rows_pad(p.M) && p.ldo % 16 == 0,
                    "gemm_fp8(swiglu): output scales / stride");
      FLITE_REQUIRE(p.bias == nullptr, "gemm_fp8(swiglu): no bias");
      launch8<EPI8_SWIGLU_FP8>(p, s);
      break;
    case EPI8_SWIGLU_BF16:
      FLITE_REQUIRE(p.N % 256 == 0 && p.ldo % 4 == 0 && ((uintptr_t)p.out & 7) == 0,
                    "gemm_fp8(swiglu bf16): 2F a multiple of 256, 8-B aligned rows");
      FLITE_REQUIRE(p.bias == nullptr, "gemm_fp8(swiglu): no bias");
      launch8<EPI8_SWIGLU_BF16>(p, s);
      break;
    case EPI8_QKV_NORM_BF16:
      FLITE_REQUIRE(p.N % 256 == 0 && p.ldo % 4 == 0 && p.norm_cols % 256 == 0 && p.rope_cols % 256 == 0 &&
                        p.rope_cols <= p.norm_cols && p.norm_cols <= p.N,
                    "gemm_fp8(qkv_norm): heads of 256 columns");
      FLITE_REQUIRE(p.rope_cols == 0 || (p.rope.cs && p.rope.tokens > 0 && p.rope.h > 0 && p.rope.w > 0),
                    "gemm_fp8(qkv_norm): RoPE tables missing");
      launch8<EPI8_QKV_NORM_BF16>(p, s);
      break;
    default:
      FLITE_REQUIRE(false, "gemm_fp8: unknown epilogue");
  }
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace flite
