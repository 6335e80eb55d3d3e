// bf16 MFMA GEMM for gfx950 with fused epilogues.
//
//   C[M,N] = A[M,K] . W[N,K]^T (+ bias[N])           -- nn.Linear layout: both operands K-contiguous
//
// Replaces every nn.Linear on the DiT hot path (reference f_lite/model.py:151-156 qkv/q/context_kv/proj,
// model.py:261-267 LigerSwiGLUMLP gate/up/down, model.py:436 context_proj, model.py:448-456 time/adaLN,
// model.py:475 final_proj), the patch-embed Conv2d (model.py:321, k=s=2 == GEMM over 64-vectors) and, in the
// implicit-GEMM CONV mode, the 3x3 convolutions of the VAE decoder.
//
// Tile 256x256x64, 512 threads = 8 waves laid out 2(M) x 4(N); each wave owns 128x64 of C as 8x4 tiles of
// v_mfma_f32_16x16x32_bf16 (on random bf16 data the 16x16x32 shape holds a higher clock than 32x32x16:
// MI355X_MICROARCH.md, DVFS item 7). W is the MFMA "A" operand and the activations the "B" operand, so each
// lane's accumulator holds 4 consecutive output COLUMNS of one output row (8/16-B epilogue stores; row-wise
// fused epilogues need no shuffles).
// Operands stream HBM->LDS by LDS-DMA (16 B/lane, lane-linear image; the bank-conflict XOR swizzle is applied on
// the per-lane SOURCE offset and undone on the ds_read), two LDS buffers, one barrier per 64-deep k-tile.
// Fragments are register double-buffered at half-k-step granularity (W: two sets of 4; A: low/high halves of
// 8), so every ds_read overlaps MFMAs of the previous half-step, including across the k-tile barrier.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "kernels.h"
#include "stream_k.h"

namespace flite {

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int NT = 512;
constexpr int TILE_BYTES = BM * BK * 2;          // 32 KiB per operand tile
// LDS: [A buf0 | A buf1 | W buf0 | W buf1]: every fragment read is a per-lane base + 16-bit immediate
constexpr int W_REGION = 2 * TILE_BYTES;
constexpr int LDS_BYTES = 4 * TILE_BYTES;        // 128 KiB
// + 8 KiB that nothing reads: the landing area of the weight read-ahead (GemmCta::read_ahead)
constexpr int PF_LDS = 8192;
constexpr int LDS_ALLOC = LDS_BYTES + PF_LDS;

typedef __attribute__((ext_vector_type(4))) int i32x4;

// 128-B tile rows (64 bf16 of K) hold 8 16-B chunks; chunk c of row r is stored at c ^ swz(r). Any 16
// consecutive rows then cover all 16 bank slots of a 256-B bank row -> conflict-free ds_read_b128.
__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

// One k-tile of LDS-DMA for this wave: 4 A pieces (1 KiB apart in LDS) + 4 W pieces (8 KiB apart) of 1 KiB
// (64 lanes x 16 B) by buffer_load_dwordx4 ... lds (the range check returns 0 for out-of-range offsets: conv
// padding). A single asm block because hipcc tracks builtin LDS-DMA and then waits vmcnt(0) before every LDS
// read it cannot prove disjoint, serialising the prefetch with the MFMAs; the waits for these copies are
// placed by hand. `skip` (uniform) turns the block into a no-op without splitting the basic block.
__device__ __forceinline__ void stage_dma(const i32x4& ra, unsigned sa, unsigned va0, unsigned va1, unsigned va2,
                                          unsigned va3, const i32x4& rw, unsigned sw, unsigned vw0, unsigned vw1,
                                          unsigned vw2, unsigned vw3, unsigned lds_a, unsigned lds_w,
                                          unsigned skip) {
  unsigned keep;
  asm volatile(
      "s_cmp_eq_u32 %[skip], 0\n\t"
      "s_cbranch_scc0 .Lskip_dma_%=\n\t"
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
      "s_mov_b32 m0, %[keep]\n"
      ".Lskip_dma_%=:"
      : [keep] "=&s"(keep)
      : [skip] "s"(skip), [la] "s"(lds_a), [lw] "s"(lds_w), [ra] "s"(ra), [sa] "s"(sa), [rw] "s"(rw), [sw] "s"(sw),
        [va0] "v"(va0), [va1] "v"(va1), [va2] "v"(va2), [va3] "v"(va3), [vw0] "v"(vw0), [vw1] "v"(vw1),
        [vw2] "v"(vw2), [vw3] "v"(vw3)
      : "memory", "scc");
}

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

// sched_group_barrier masks
constexpr int SG_MFMA = 0x008, SG_DSR = 0x100;

// CONV = implicit-GEMM 3x3 convolution (pad 1) over an NHWC bf16 input: A row m = output pixel, k = (tap, c)
// with tap = ky*3+kx. Each 64-wide k-tile is one tap and 64 consecutive channels (128 contiguous bytes of
// one input pixel); the buffer range check returns 0 for the padding pixels.
// `upsample` folds nearest-2x interpolation into the addressing (Upsample2D + conv).
// MI = 16-row MFMA blocks per wave along M: 8 -> 256-row output tiles, 7 -> 224-row tiles (fewer, smaller
// tiles where 256 rows leave a last wave of tiles mostly empty; the A staging still copies 256 rows).
template <int EPI, bool CONV, int MI = 8>
struct GemmCta {
  static constexpr bool GATED_FF = EPI == EPI_SWIGLU_BF16 || EPI == EPI_GEGLU_BF16;  // W = gate | W2 = up, N = 2F
  static constexpr int WM = MI * 16;  // output rows per wave_m
  static constexpr int BMV = 2 * WM;  // output rows per tile
  const GemmParams& p;
  int tid, lane, wave, wave_m, wave_n, lr, lk;
  unsigned lds0;
  i32x4 a_rsrc, w_rsrc;
  unsigned ab[2], wb[2];  // per-lane LDS byte address of k-step s in buffer 0 (row base + swizzled chunk)
  // per output tile
  unsigned a_off[4], w_off[4];
  int cyx[4];  // CONV: output pixel (y << 16 | x) of the piece's row
  int ke;      // end of the k-tile range being staged
  int tm0;     // first output row of the tile

  __device__ __forceinline__ GemmCta(const GemmParams& p_, char* smem) : p(p_) {
    tid = threadIdx.x;
    lane = tid & 63;
    wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    wave_m = wave >> 2;  // 0..1
    wave_n = wave & 3;   // 0..3
    lr = lane & 15;
    lk = lane >> 4;
    lds0 = (unsigned)__builtin_amdgcn_readfirstlane((int)lds_addr_of(smem));
    a_rsrc = CONV ? make_rsrc(p.conv_in, (unsigned)p.conv_in_bytes) : make_rsrc(p.A, (unsigned)((long)p.M * p.lda * 2));
    // SwiGLU: W rows 8w + 64i lie in 16-row sub-tile (w>>1) + 4i, whose parity (gate / up) is (w>>1)&1
    const bf16_t* wsrc = (GATED_FF && ((wave >> 1) & 1)) ? p.W2 : p.W;
    const long w_rows = GATED_FF ? (long)(p.N >> 1) : (long)p.N;
    w_rsrc = make_rsrc(wsrc, (unsigned)(w_rows * p.ldw * 2));
    // Fragment reads (16x16x32 operand map): lane l holds row (l & 15), k = 8*(l>>4) + 0..7 of the 32-deep
    // k-step s -> 16-B chunk 4s + (l>>4) of a 128-B tile row. Rows: W tile wave_n*64 + ni*16 + (l&15),
    // A tile wave_m*128 + mi*16 + (l&15); the swizzle depends only on l&15 (row bases are multiples of 16).
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const unsigned coff = ((4 * s + lk) ^ swz(lr)) << 4;
      ab[s] = lds0 + (wave_m * WM + lr) * 128 + coff;
      wb[s] = lds0 + W_REGION + (wave_n * 64 + lr) * 128 + coff;
    }
  }

  // Per-lane staging offsets of output tile (m0, n0).
  // DMA piece q (0..31) covers tile rows 8q..8q+7; lane -> row 8q + lane/8, 16-B chunk (lane&7)^swz(row).
  // A: wave w copies pieces 4w..4w+3; W: pieces w, w+8, w+16, w+24 (rows 8w + 64i), so that under the SwiGLU
  // interleave (16-row sub-tiles alternate gate / up) all of a wave's W pieces come from one tensor.
  // Both operands are addressed as buffers: per-lane byte offset of (row, chunk) + uniform k offset in soffset.
  __device__ __forceinline__ void setup_tile(int m0, int n0) {
    tm0 = m0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      {
        const int row = (wave * 4 + i) * 8 + (lane >> 3);
        const int chunk = (lane & 7) ^ swz(row);
        const int am = min(m0 + row, p.M - 1);
        if constexpr (CONV) {
          const int hw = p.conv_oh * p.conv_ow;
          const int b = am / hw;
          const int r = am - b * hw;
          const int y = r / p.conv_ow;
          cyx[i] = (y << 16) | (r - y * p.conv_ow);
          a_off[i] = (unsigned)((long)b * p.conv_ih * p.conv_iw * p.conv_c + chunk * 8) * 2u;
        } else {
          a_off[i] = (unsigned)(((long)am * p.lda + chunk * 8) * 2);
          // 224-row tiles: wave 7's pieces are rows 224-255, which no MFMA reads. An out-of-range offset makes
          // the copy a zero fill that moves no bytes (1/8 of the A stream through L2 and into LDS; on the
          // power-limited part bytes cost clock, profiles/r03q). Same instruction count, same vmcnt accounting.
          if (MI == 7 && wave == 7 && (long)p.M * p.lda * 2 <= 0x7fffffffL) a_off[i] = 0x80000000u;
        }
      }
      {
        const int row = (wave + 8 * i) * 8 + (lane >> 3);
        const int chunk = (lane & 7) ^ swz(row);
        const int wn = min(n0 + row, p.N - 1);
        long wrow = wn;
        if constexpr (GATED_FF) {
          // virtual row wn: sub-tile wn>>4 is gate (even) / up (odd) of output columns (wn>>5)*16 + (wn&15)
          wrow = (long)(wn >> 5) * 16 + (wn & 15);
        } else if constexpr (EPI == EPI_QKV_NORM_BF16) {
          if (n0 < p.rope_cols) wrow = rope_perm(wn);  // rotation pairs side by side (qkv_norm_epilogue)
        }
        w_off[i] = (unsigned)((wrow * p.ldw + chunk * 8) * 2);
      }
    }
  }

  // DMA k-tile kt into LDS buffer buf (no-op when kt >= ke)
  __device__ __forceinline__ void stage(int kt, int buf) {
    const unsigned la = (unsigned)__builtin_amdgcn_readfirstlane((int)(lds0 + buf * TILE_BYTES + wave * 4096));
    const unsigned lw =
        (unsigned)__builtin_amdgcn_readfirstlane((int)(lds0 + W_REGION + buf * TILE_BYTES + wave * 1024));
    const unsigned kb = (unsigned)(kt * BK * 2);
    unsigned va[4];
    unsigned sa;
    if constexpr (CONV) {
      const int koff = kt * BK;
      const int tap = koff / p.conv_c;
      const int c0 = koff - tap * p.conv_c;
      const int ky = tap / 3 - 1, kx = tap % 3 - 1;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int iy = (cyx[i] >> 16) + ky, ix = (cyx[i] & 0xffff) + kx;
        const bool ok = iy >= 0 && iy < p.conv_oh && ix >= 0 && ix < p.conv_ow;
        const int sy = p.conv_up ? (iy >> 1) : iy;
        const int sx = p.conv_up ? (ix >> 1) : ix;
        va[i] = ok ? a_off[i] + (unsigned)((sy * p.conv_iw + sx) * p.conv_c + c0) * 2u : 0x80000000u;
      }
      sa = 0;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) va[i] = a_off[i];
      sa = kb;
    }
    stage_dma(a_rsrc, sa, va[0], va[1], va[2], va[3], w_rsrc, kb, w_off[0], w_off[1], w_off[2], w_off[3], la, lw,
              (unsigned)__builtin_amdgcn_readfirstlane(kt >= ke ? 1 : 0));
  }

  // Weight read-ahead for the GEMM after next (GemmParams::pf): this workgroup's 8 KiB pieces wg, wg + G, ... of
  // the range (at most 6), one 1 KiB LDS-DMA copy per wave each, into the PF_LDS area that nothing reads. Issued
  // after the mainloop, so their HBM latency overlaps the epilogue; the kernel waits for them at its end.
  __device__ __forceinline__ void read_ahead(int wg, int G) {
    const long pieces = (p.pf_bytes + 8191) >> 13;
    if (wg >= pieces) return;
    const i32x4 rs = make_rsrc(p.pf, (unsigned)p.pf_bytes);
    const unsigned lds = (unsigned)__builtin_amdgcn_readfirstlane((int)(lds0 + LDS_BYTES + wave * 1024));
    const unsigned voff = (unsigned)(wave * 1024 + lane * 16);
#pragma unroll 1
    for (int k = 0; k < 6; ++k) {
      const long i = wg + (long)k * G;
      if (i >= pieces) break;
      const unsigned soff = (unsigned)__builtin_amdgcn_readfirstlane((int)(i << 13));
      unsigned keep;
      asm volatile(
          "s_mov_b32 %[keep], m0\n\t"
          "s_mov_b32 m0, %[l]\n\t"
          "s_nop 0\n\t"
          "buffer_load_dwordx4 %[v], %[r], %[s] offen lds\n\t"
          "s_mov_b32 m0, %[keep]"
          : [keep] "=&s"(keep)
          : [l] "s"(lds), [r] "s"(rs), [s] "s"(soff), [v] "v"(voff)
          : "memory");
    }
  }

  // W fragment ni / A fragment mi of k-step s in buffer BUF
  template <int BUF>
  __device__ __forceinline__ bf16x8 rd_w(int s, int ni) const {
    return *(const LDS_AS bf16x8*)(wb[s] + BUF * TILE_BYTES + ni * 16 * 128);
  }
  template <int BUF>
  __device__ __forceinline__ bf16x8 rd_a(int s, int mi) const {
    return *(const LDS_AS bf16x8*)(ab[s] + BUF * TILE_BYTES + mi * 16 * 128);
  }
  // 16 MFMAs: A rows mi0..mi0+3 x all 4 W fragments (MV: the wave's 16-row blocks that hold output rows)
  template <int MV>
  __device__ __forceinline__ static void mfma_half(f32x4 (&acc)[8][4], const bf16x8 (&wf)[4],
                                                   const bf16x8 (&af)[4], int mi0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        if (mi0 + i < MV)
          acc[mi0 + i][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ni], af[i], acc[mi0 + i][ni], 0, 0, 0);
  }
  // spread NR ds_reads over a half-step's NM MFMAs
  template <int NR, int NM = 16>
  __device__ __forceinline__ static void interleave() {
    if constexpr (NM > 0) {
      constexpr int per = NM / NR;
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        __builtin_amdgcn_sched_group_barrier(SG_MFMA, per, 0);
        __builtin_amdgcn_sched_group_barrier(SG_DSR, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(SG_MFMA, NM - per * NR, 0);
    }
  }
  // MFMAs in the low (mi 0..3) and high (mi 4..7) half-steps of a wave with MV live row blocks
  static constexpr int lo_mfmas(int mv) { return (mv < 4 ? mv : 4) * 4; }
  static constexpr int hi_mfmas(int mv) { return (mv > 4 ? mv - 4 : 0) * 4; }

  // One 64-deep k-tile from LDS buffer BUF. Register sets: wx / wy = W fragments of alternating k-steps,
  // al / ah = A fragments mi 0..3 / 4..7.
  //   k0.lo: MFMA(wx, al) || read ah(k0), wy[0..1](k1)      k0.hi: MFMA(wx, ah) || read wy[2..3](k1), al(k1)
  //   k1.lo: MFMA(wy, al) || read ah(k1)
  //   wait for tile t+1 (own copies) + all reads of buffer t&1, barrier, DMA tile t+2 into buffer t&1
  //   k1.hi: MFMA(wy, ah) || read wx, al of k0 of tile t+1 (stale, unused data after the last tile)
  template <int BUF, int MV>
  __device__ __forceinline__ void ktile(f32x4 (&acc)[8][4], bf16x8 (&wx)[4], bf16x8 (&wy)[4], bf16x8 (&al)[4],
                                        bf16x8 (&ah)[4], int kt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) ah[i] = rd_a<BUF>(0, 4 + i);
    wy[0] = rd_w<BUF>(1, 0);
    wy[1] = rd_w<BUF>(1, 1);
    mfma_half<MV>(acc, wx, al, 0);
    interleave<6, lo_mfmas(MV)>();
    wy[2] = rd_w<BUF>(1, 2);
    wy[3] = rd_w<BUF>(1, 3);
#pragma unroll
    for (int i = 0; i < 4; ++i) al[i] = rd_a<BUF>(1, i);
    mfma_half<MV>(acc, wx, ah, 4);
    interleave<6, hi_mfmas(MV)>();
#pragma unroll
    for (int i = 0; i < 4; ++i) ah[i] = rd_a<BUF>(1, 4 + i);
    mfma_half<MV>(acc, wy, al, 0);
    interleave<4, lo_mfmas(MV)>();
    // Round-1 ablation builds priced this wait on MI355X: 3.5 % of the gate/up GEMM and 8-11 % of the K = 12288
    // projections (operands streamed from HBM), nothing at K = 3072, N <= 9216.
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // The two waves of a SIMD (w, w + 4) issue their copies of tile t+2 a half-step apart, so one of them
    // keeps the MFMA pipe fed while the other spends issue cycles on LDS-DMA. Not in CONV mode: there the
    // per-tap gather addressing makes the split schedule 1.9x slower (tools/kbench_conv.py).
    if constexpr (CONV)
      stage(kt + 2, BUF);
    else
      stage(wave_m == 0 ? kt + 2 : ke, BUF);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      wx[i] = rd_w<BUF ^ 1>(0, i);
      al[i] = rd_a<BUF ^ 1>(0, i);
    }
    mfma_half<MV>(acc, wy, ah, 4);
    interleave<8, hi_mfmas(MV)>();
    if constexpr (!CONV) stage(wave_m == 1 ? kt + 2 : ke, BUF);
  }

  // acc = A[m0.., kb*64 : kend*64] . W[n0.., same]^T  (setup_tile(m0, n0) first). Every k-tile runs the same
  // straight-line code; the loop is unrolled x2 so the LDS buffer index is static.
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
    if (kend - kb > 1)
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // this wave's 8 copies of the first tile
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // Ragged last tile: a wave whose 16-row blocks lie (partly) past row M skips their MFMAs. At M = 8224 with
    // 256-row tiles the last of 33 M-tiles holds 32 rows, so 2.7 % of the gate/up, qkv and down MFMA work was
    // spent on rows that are never stored (energy on a power-limited part, profiles/r03q). Staging, barriers and
    // fragment reads are those of the full loop, so every wave of the workgroup still meets every barrier.
    const int live = p.M - (tm0 + wave_m * WM);  // uniform per wave
    const int mv = live <= 0 ? 0 : min((live + 15) >> 4, MI);
    if (mv > 4)
      kloop<MI>(acc, kb, kend);
    else if (mv > 2)
      kloop<(MI < 4 ? MI : 4)>(acc, kb, kend);
    else if (mv > 0)
      kloop<2>(acc, kb, kend);
    else
      kloop<0>(acc, kb, kend);
  }
  template <int MV>
  __device__ __forceinline__ void kloop(f32x4 (&acc)[8][4], int kb, int kend) {
    bf16x8 wx[4], wy[4], al[4], ah[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      wx[i] = rd_w<0>(0, i);
      al[i] = rd_a<0>(0, i);
    }
    int kt = kb;
    for (; kt + 1 < kend; kt += 2) {
      ktile<0, MV>(acc, wx, wy, al, ah, kt);
      ktile<1, MV>(acc, wx, wy, al, ah, kt + 1);
    }
    if (kt < kend) ktile<0, MV>(acc, wx, wy, al, ah, kt);
  }

  // Gated residual x[m][n] += gate[seg(m)][n] * (acc + bias[n]) (model.py:289,297,301). A read-modify-write of
  // the fp32 residual: the loads of two accumulator rows (8 x + 8 gate, 16 B per lane) are issued together at
  // clamped, always-valid addresses and only the stores are masked, so the tile pays 4 memory round trips
  // instead of one per 16-B group (a bounds branch around each load makes hipcc wait vmcnt(0) per group).
  // X16 (EPI_RESID_BF16): the residual stream is bf16; the same fp32 expression, one rounding at the store.
  // WIDE (X16 with N % 8 == 0 and 16-B aligned rows): the x loads and stores move 16 B per lane in common.h's deal8
  // layout (8 consecutive columns of a 32-column pair of 16-column groups), one v_permlane16_swap per dword turning
  // them into the accumulator layout and back (the swap is its own inverse); without it 8 B per 4 columns.
  template <bool GATED, bool TWO_SEG, bool X16 = false, bool WIDE = false>
  __device__ __forceinline__ void resid_epilogue(const f32x4 (&acc)[8][4], int m_base, int n_base) {
    float bias[4][4];
    int nc[4];
    bool nok[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int n = n_base + ni * 16;
      nok[ni] = n < p.N;  // N % 4 == 0: a 4-column group is entirely in or out
      nc[ni] = nok[ni] ? n : 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) bias[ni][r] = (p.bias != nullptr && nok[ni]) ? bf2f(p.bias[nc[ni] + r]) : 0.f;
    }
    // The gate row depends only on the segment of the output row. When a segment is at least as tall as the
    // lane's row span, the lane's rows touch at most two segments: load those two gate rows once instead of one
    // per accumulator row (28 -> 8 loads per lane).
    f32x4 g2[2][4];
    int seg_lo = 0;
    if constexpr (TWO_SEG) {
      seg_lo = min(m_base, p.M - 1) / p.rows_per_seg;
      const int seg_hi = min(m_base + (MI - 1) * 16, p.M - 1) / p.rows_per_seg;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const float* grow = p.gate + (long)(s ? seg_hi : seg_lo) * p.gate_seg_stride;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) g2[s][ni] = *(const f32x4*)(grow + nc[ni]);
      }
    }
#pragma unroll
    for (int mb = 0; mb < 8; mb += 2) {
      f32x4 xv[2][4], gv[2][4];
      char* orow[2];
      bool mok[2];
      constexpr int XB = X16 ? 2 : 4;  // bytes per residual element
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int m = m_base + (mb + i) * 16;
        mok[i] = mb + i < MI && m < p.M;
        const int mc = mok[i] ? m : p.M - 1;
        orow[i] = (char*)p.out + (long)mc * p.ldo * XB;
        const int seg = GATED ? mc / p.rows_per_seg : 0;
        const float* grow = GATED ? p.gate + (long)seg * p.gate_seg_stride : nullptr;
        if constexpr (WIDE) {
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int pc = n_base - lk * 4 + 32 * q + deal8_col();  // this lane's 8-column piece of the pair
            const u32x4 w = *(const u32x4*)(orow[i] + (pc < p.N ? pc : 0) * XB);
            const auto t = __builtin_amdgcn_permlane16_swap(w.x, w.z, false, false);  // deal8's inverse
            const auto u = __builtin_amdgcn_permlane16_swap(w.y, w.w, false, false);
            const u32x2 a = {t[0], u[0]}, b = {t[1], u[1]};  // groups 2q and 2q + 1 in the accumulator layout
            xv[i][2 * q] = f32x4{__uint_as_float(a.x << 16), __uint_as_float(a.x & 0xffff0000u),
                                 __uint_as_float(a.y << 16), __uint_as_float(a.y & 0xffff0000u)};
            xv[i][2 * q + 1] = f32x4{__uint_as_float(b.x << 16), __uint_as_float(b.x & 0xffff0000u),
                                     __uint_as_float(b.y << 16), __uint_as_float(b.y & 0xffff0000u)};
          }
        }
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          if constexpr (WIDE) {
          } else if constexpr (X16) {
            const u32x2 w = *(const u32x2*)(orow[i] + nc[ni] * XB);
            xv[i][ni] = f32x4{__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                              __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u)};
          } else {
            xv[i][ni] = *(const f32x4*)(orow[i] + nc[ni] * XB);
          }
          if constexpr (TWO_SEG)
            gv[i][ni] = seg == seg_lo ? g2[0][ni] : g2[1][ni];
          else if constexpr (GATED)
            gv[i][ni] = *(const f32x4*)(grow + nc[ni]);
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        u32x2 pk[4];
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          f32x4 x = xv[i][ni];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = acc[mb + i][ni][r] + bias[ni][r];
            if constexpr (GATED)
              x[r] += v * gv[i][ni][r];
            else
              x[r] += v;
          }
          if constexpr (WIDE) {
            pk[ni] = u32x2{pack2bf(x[0], x[1]), pack2bf(x[2], x[3])};
          } else if constexpr (X16) {
            if (mok[i] && nok[ni]) *(u32x2*)(orow[i] + nc[ni] * XB) = u32x2{pack2bf(x[0], x[1]), pack2bf(x[2], x[3])};
          } else {
            if (mok[i] && nok[ni]) *(f32x4*)(orow[i] + nc[ni] * XB) = x;
          }
        }
        if constexpr (WIDE) {
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const u32x4 w = deal8(pk[2 * q], pk[2 * q + 1]);  // every lane takes part; only the store is masked
            const int pc = n_base - lk * 4 + 32 * q + deal8_col();
            if (mok[i] && pc < p.N) *(u32x4*)(orow[i] + pc * XB) = w;
          }
        }
      }
    }
  }

  // RoPE heads (q, k): the W rows (and bias) are read in rope_perm order (common.h), so every rotation pair of
  // apply_rotary_emb sits in two adjacent columns of one lane; v (no RoPE) keeps the original layout.

  // qkv / cross-q epilogue (EPI_QKV_NORM_BF16). A 256-column tile is exactly one head (n0 % 256 == 0). Columns
  // [0, norm_cols) get, in fp32 and with one bf16 rounding at the end: RoPE (apply_rotary_emb, model.py:403-414:
  // y1 = x1 c + x2 s, y2 = -x1 s + x2 c for the pairs (c, c + 128), tables of the bf16 model) on columns
  // [0, rope_cols), then QKNorm's RMSNorm over the head (model.py:115-126,180,197). On RoPE tiles the columns are
  // in rope_perm order, so each lane rotates its pairs in registers; the angles of those pairs belong to one axis
  // per wave (waves 0-1: y, 2-3: x) and come from the factorised table (RopeAxes) as one 16-B (cos, sin, cos, sin)
  // load per 4 columns, fetched one 16-row block ahead. The head's sum of squares is a 4-lane shuffle plus 4 wave
  // partials in LDS.
  __device__ __forceinline__ void qkv_norm_epilogue(f32x4 (&acc)[8][4], int m0, int n0, int m_base, int n_base) {
    const bool rope = n0 < p.rope_cols;  // tile-uniform
    float bias[4][4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n_base + ni * 16 + r;
        bias[ni][r] = (p.bias != nullptr && n < p.N) ? bf2f(p.bias[rope ? rope_perm(n) : n]) : 0.f;
      }
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[mi][ni][r] += bias[ni][r];
    const bool norm = n0 < p.norm_cols;  // tile-uniform
    if (norm) {
      if (rope) rope_rotate<MI>(acc, p.rope, m_base, p.M, wave_n, lk);
      __syncthreads();  // every wave is done with the k-tile buffers (the row partials below reuse LDS)
      // per-head RMSNorm: row sum of squares = 4 lanes (lk) x 4 waves (wave_n)
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
      if (wide) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const u32x4 w = deal8(pk[2 * q], pk[2 * q + 1]);
          if (m < p.M) *(u32x4*)(orow + n0 + wave_n * 64 + 32 * q + deal8_col()) = w;
        }
      } else if (m < p.M) {
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) *(u32x2*)(orow + n_base + ni * 16) = pk[ni];
      }
    }
  }

  // Wide bf16 stores (common.h deal8): 16-B pieces, 64 B per row and store instruction instead of 8-B pieces
  __device__ __forceinline__ int deal8_col() const { return ::flite::deal8_col(lk); }
  // 16-B stores are legal when every row start is 16-B aligned
  __device__ __forceinline__ bool wide_ok() const {
    return (p.ldo & 7) == 0 && ((uintptr_t)p.out & 15) == 0;
  }

  // ---- epilogue: lane holds C[m][n..n+3] for m = m_base + mi*16 + (lane&15), n = n_base + ni*16 + 4*(lane>>4)
  __device__ __forceinline__ void epilogue(f32x4 (&acc)[8][4], int m0, int n0) {
    const int m_base = m0 + wave_m * WM + lr;
    const int n_base = n0 + wave_n * 64 + lk * 4;

    if constexpr (EPI == EPI_QKV_NORM_BF16) {
      qkv_norm_epilogue(acc, m0, n0, m_base, n_base);
      return;
    } else if constexpr (GATED_FF) {
      // pairs (ni=0 gate, ni=1 up), (ni=2 gate, ni=3 up) -> output column (n0/2 + wave_n*32 + pair*16 + 4*(lane>>4))
      const int F = p.N >> 1;
      const bool wide = wide_ok();
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        const int m = m_base + mi * 16;
        u32x2 v[2];
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {
          const f32x4 g = acc[mi][2 * pr];
          const f32x4 u = acc[mi][2 * pr + 1];
          if constexpr (EPI == EPI_SWIGLU_BF16) {
            v[pr].x = pack2bf(silu_f(g[0]) * u[0], silu_f(g[1]) * u[1]);
            v[pr].y = pack2bf(silu_f(g[2]) * u[2], silu_f(g[3]) * u[3]);
          } else {
            v[pr].x = pack2bf(gelu_tanh_f(g[0]) * u[0], gelu_tanh_f(g[1]) * u[1]);
            v[pr].y = pack2bf(gelu_tanh_f(g[2]) * u[2], gelu_tanh_f(g[3]) * u[3]);
          }
        }
        bf16_t* orow = (bf16_t*)p.out + (long)m * p.ldo;
        if (wide) {  // F % 16 == 0: an 8-column group is entirely inside or outside [0, F)
          const u32x4 w = deal8(v[0], v[1]);
          const int oc = (n0 >> 1) + wave_n * 32 + deal8_col();
          if (m < p.M && oc < F) *(u32x4*)(orow + oc) = w;
        } else {
#pragma unroll
          for (int pr = 0; pr < 2; ++pr) {
            const int oc = (n0 >> 1) + wave_n * 32 + pr * 16 + lk * 4;
            if (m < p.M && oc < F) *(u32x2*)(orow + oc) = v[pr];
          }
        }
      }
      return;
    } else if constexpr (EPI == EPI_RESID_F32) {
      if (p.gate == nullptr)
        resid_epilogue<false, false>(acc, m_base, n_base);
      else if (p.rows_per_seg >= MI * 16)
        resid_epilogue<true, true>(acc, m_base, n_base);
      else
        resid_epilogue<true, false>(acc, m_base, n_base);
      return;
    } else if constexpr (EPI == EPI_RESID_BF16) {
      // 16-B lanes when every 8-column piece is inside or outside [0, N) and rows are 16-B aligned
      if ((p.N & 7) == 0 && wide_ok() && !p.resid_narrow) {
        if (p.gate == nullptr)
          resid_epilogue<false, false, true, true>(acc, m_base, n_base);
        else if (p.rows_per_seg >= MI * 16)
          resid_epilogue<true, true, true, true>(acc, m_base, n_base);
        else
          resid_epilogue<true, false, true, true>(acc, m_base, n_base);
      } else {
        if (p.gate == nullptr)
          resid_epilogue<false, false, true>(acc, m_base, n_base);
        else if (p.rows_per_seg >= MI * 16)
          resid_epilogue<true, true, true>(acc, m_base, n_base);
        else
          resid_epilogue<true, false, true>(acc, m_base, n_base);
      }
      return;
    } else {
      float bias[4][4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = n_base + ni * 16 + r;
          bias[ni][r] = (p.bias != nullptr && n < p.N) ? bf2f(p.bias[n]) : 0.f;
        }
      // N % 8 == 0: an 8-column group of deal8 is entirely inside or outside [0, N)
      const bool wide = EPI == EPI_STORE_BF16 && p.resid == nullptr && (p.N & 7) == 0 && wide_ok();
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        const int m = m_base + mi * 16;
        const long om = p.out_seg > 0 ? (m / p.out_seg) * p.out_seg_stride + p.out_seg_off + (m % p.out_seg) : m;
        if constexpr (EPI == EPI_STORE_BF16) {
          if (wide) {
            u32x2 pk[4];
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) {
              f32x4 v = acc[mi][ni];
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] += bias[ni][r];
              if (p.act == 1) {
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = silu_f(v[r]);
              }
              pk[ni].x = pack2bf(v[0], v[1]);
              pk[ni].y = pack2bf(v[2], v[3]);
            }
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              const u32x4 w = deal8(pk[2 * q], pk[2 * q + 1]);
              const int n = n0 + wave_n * 64 + 32 * q + deal8_col();
              if (m < p.M && n < p.N) *(u32x4*)((bf16_t*)p.out + om * p.ldo + n) = w;
            }
            continue;
          }
        }
        if (m >= p.M) continue;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const int n = n_base + ni * 16;
          if (n >= p.N) continue;
          f32x4 v = acc[mi][ni];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += bias[ni][r];
          if (p.act == 1) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = silu_f(v[r]);
          }
          if constexpr (EPI == EPI_STORE_BF16) {
            bf16_t* o = (bf16_t*)p.out + om * p.ldo + n;
            if (p.resid != nullptr) {  // ResnetBlock2D / attention residual (x + h), same layout as out
              const bf16_t* rr = p.resid + om * p.ldo + n;
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (n + r < p.N) v[r] += bf2f(rr[r]);
            }
            if (n + 3 < p.N) {
              u32x2 w;
              w.x = pack2bf(v[0], v[1]);
              w.y = pack2bf(v[2], v[3]);
              *(u32x2*)o = w;
            } else {
              for (int r = 0; r < 4 && n + r < p.N; ++r) o[r] = f2bf(v[r]);
            }
          } else if constexpr (EPI == EPI_STORE_F32) {
            float* o = (float*)p.out + om * p.ldo + n;
            if (n + 3 < p.N) {
              *(f32x4*)o = v;
            } else {
              for (int r = 0; r < 4 && n + r < p.N; ++r) o[r] = v[r];
            }
          }
        }
      }
    }
  }
};

// One launch: data-parallel (grid = tiles, one output tile per workgroup) or, when the launcher set
// p.sk_tiles, the persistent stream-K + data-parallel schedule above (grid = one workgroup per CU).
template <int EPI, bool CONV, int MI>
__global__ __launch_bounds__(NT, 2) void gemm_bf16_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using Cta = GemmCta<EPI, CONV, MI>;
  Cta c(p, smem);
  const int num_m = (p.M + Cta::BMV - 1) / Cta::BMV;
  const int num_n = (p.N + BN - 1) / BN;
  const int nk = p.K / BK;
  const int wg = sk::xcd_remap(blockIdx.x, gridDim.x);
  f32x4 acc[8][4];
  if constexpr (!CONV && MI == 8) {
    if (p.sk_tiles > 0) {
      sk::stream_k_body<NT>(c, acc, num_m, num_n, nk, wg);
      return;
    }
  }
  int m0, n0;
  sk::tile_origin(wg, num_m, num_n, m0, n0, Cta::BMV, BN);
  c.setup_tile(m0, n0);
  c.mainloop(acc, 0, nk);
  if constexpr (!CONV)
    if (p.pf != nullptr) c.read_ahead(wg, gridDim.x);
  c.epilogue(acc, m0, n0);
  if constexpr (!CONV)
    if (p.pf != nullptr) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the read-ahead has landed
}

int g_num_cu = 0;

// stream-K split (stream_k.h) when the caller passed a workspace
int choose_sk_tiles(const GemmParams& p, int T, int* gs) {
  *gs = 0;
  if (p.sk_ws == nullptr || p.sk_flags == nullptr) return 0;
  // Long launches with a short last round (>= 8 full rounds, leftover <= half a round: the SwiGLU gate/up at
  // 1024^2, 12 rounds + 96 tiles): the leftover tiles cut in two ranges each. The model below, fitted to 2-round
  // launches, prices this at +1 %; in the sampling loop it measured -0.7 % gate/up and +0.9 % image (3 of 3
  // same-lease rounds; cut in ~2.7 ranges: +0.5 %; profiles/r03t).
  const int G = g_num_cu, rem = G > 0 ? T % G : 0;
  if (G > 0 && T / G >= 8 && rem > 0 && 2 * rem <= G && p.K / BK >= 4) {
    *gs = 2 * rem;
    return rem;
  }
  static const bool no_sk = getenv("FLITE_GEMM_NO_SK") != nullptr;  // A/B switch for measurements
  if (no_sk) return 0;
  // A/B switch for measurements: every short launch with a partial last round cut in FLITE_GEMM_SK_FAN ranges per
  // leftover tile, whatever the model below predicts
  static const int fan = getenv("FLITE_GEMM_SK_FAN") ? atoi(getenv("FLITE_GEMM_SK_FAN")) : 0;
  if (fan >= 2 && G > 0 && rem > 0 && T / G < 8 && rem * (p.K / BK) >= 2 * std::min(G, fan * rem)) {
    *gs = std::min(G, fan * rem);
    return rem;
  }
  return sk::choose_sk_tiles(T, p.K / BK, G, gs);
}

// Tile height: 224-row tiles (MI = 7) where they take fewer rounds x tile size than 256-row tiles on the
// G CUs (e.g. M = 8224, N = 3072: 444 tiles = 2 rounds of 7/8-size tiles instead of 396 = 2 full rounds);
// stream-K (256-row tiles only) keeps priority where its model takes it.
bool use_bm224(const GemmParams& p) {
  static const bool off = getenv("FLITE_GEMM_NO_BM224") != nullptr;  // A/B switch for measurements
  if (off || p.conv_in != nullptr || g_num_cu <= 0) return false;
  const int G = g_num_cu;
  const int num_n = (p.N + BN - 1) / BN;
  const int t256 = (p.M + 255) / 256 * num_n, t224 = (p.M + 223) / 224 * num_n;
  const double r256 = (double)((t256 + G - 1) / G), r224 = (double)((t224 + G - 1) / G) * 0.875;
  // A 224-row tile issues 14 % more LDS-DMA pieces (it stages 256 A rows; since round 3 the unread ones move no
  // bytes) and reads 4.5 % more LDS bytes per FLOP than a 256-row one. On the power-limited part that costs clock:
  // inside the sampling loop the gate/up GEMM (predicted 12.25 vs 13 rounds) ran 2.8 % FASTER with 256-row tiles
  // (profiles/r03q; its L2-fabric bytes per launch did not change, 2.36 GB). So 224 rows only where they save a
  // large share of a round.
  return r224 < 0.93 * r256;
}

template <int EPI>
int launch(GemmParams p, hipStream_t s) {
  const int num_n = (p.N + BN - 1) / BN;
  const int T = (p.M + BM - 1) / BM * num_n;
  p.sk_tiles = choose_sk_tiles(p, T, &p.sk_wgs);
  if constexpr (EPI == EPI_RESID_BF16) {
    static const bool narrow = getenv("FLITE_GEMM_RESID_NARROW") != nullptr;  // A/B switch for measurements
    p.resid_narrow = narrow;
  }
  if (p.conv_in != nullptr) {
    if constexpr (EPI == EPI_STORE_BF16 || EPI == EPI_STORE_F32)  // gemm_bf16 admits only these with CONV
      hipLaunchKernelGGL((gemm_bf16_kernel<EPI, true, 8>), dim3(T), dim3(NT), LDS_ALLOC, s, p);
  } else if (p.sk_tiles) {
    hipLaunchKernelGGL((gemm_bf16_kernel<EPI, false, 8>), dim3(g_num_cu), dim3(NT), LDS_ALLOC, s, p);
  } else if (use_bm224(p)) {
    const int T224 = (p.M + 223) / 224 * num_n;
    hipLaunchKernelGGL((gemm_bf16_kernel<EPI, false, 7>), dim3(T224), dim3(NT), LDS_ALLOC, s, p);
  } else {
    hipLaunchKernelGGL((gemm_bf16_kernel<EPI, false, 8>), dim3(T), dim3(NT), LDS_ALLOC, s, p);
  }
  return 0;
}

bool attrs_done = false;

template <int EPI>
hipError_t set_attrs() {
  hipError_t e = hipFuncSetAttribute((const void*)gemm_bf16_kernel<EPI, false, 8>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, LDS_ALLOC);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute((const void*)gemm_bf16_kernel<EPI, false, 7>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          LDS_ALLOC);
  if (e != hipSuccess) return e;
  if constexpr (EPI == EPI_STORE_BF16 || EPI == EPI_STORE_F32)
    return hipFuncSetAttribute((const void*)gemm_bf16_kernel<EPI, true, 8>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, LDS_ALLOC);
  return hipSuccess;
}

}  // namespace

int gemm_init() {
  if (attrs_done) return 0;
  FLITE_HIP_CHECK(set_attrs<EPI_STORE_BF16>());
  FLITE_HIP_CHECK(set_attrs<EPI_STORE_F32>());
  FLITE_HIP_CHECK(set_attrs<EPI_RESID_F32>());
  FLITE_HIP_CHECK(set_attrs<EPI_RESID_BF16>());
  FLITE_HIP_CHECK(set_attrs<EPI_SWIGLU_BF16>());
  FLITE_HIP_CHECK(set_attrs<EPI_GEGLU_BF16>());
  FLITE_HIP_CHECK(set_attrs<EPI_QKV_NORM_BF16>());
  {
    int dev = 0;
    FLITE_HIP_CHECK(hipGetDevice(&dev));
    hipDeviceProp_t prop;
    FLITE_HIP_CHECK(hipGetDeviceProperties(&prop, dev));
    g_num_cu = prop.multiProcessorCount;
    int per_cu = 0;  // the stream-K grid needs every workgroup resident at once
    FLITE_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gemm_bf16_kernel<EPI_RESID_F32, false, 8>, NT,
                                                                LDS_ALLOC));
    if (per_cu < 1) g_num_cu = 0;
  }
  attrs_done = true;
  return 0;
}

int gemm_sk_workspace_cus() {
  if (gemm_init()) return 0;
  return g_num_cu;
}

size_t gemm_sk_workspace_bytes() {
  const int G = gemm_sk_workspace_cus();
  return (size_t)G * BM * BN * sizeof(float) + (size_t)G * sizeof(int);
}

int gemm_bf16(const GemmParams& p, int epi, hipStream_t stream) {
  FLITE_REQUIRE(p.M > 0 && p.N > 0 && p.K > 0, "gemm: empty problem");
  FLITE_REQUIRE(p.K % BK == 0, "gemm: K must be a multiple of 64");
  FLITE_REQUIRE(p.ldw % 8 == 0, "gemm: ldw must be a multiple of 8 elements");
  FLITE_REQUIRE(((uintptr_t)p.W & 15) == 0, "gemm: W must be 16-B aligned");
  FLITE_REQUIRE((long)p.N * p.ldw * 2 < (1L << 32), "gemm: W must be < 4 GiB (32-bit buffer offsets)");
  FLITE_REQUIRE(p.pf == nullptr || (p.pf_bytes > 0 && p.pf_bytes < (1L << 31)),
                "gemm: read-ahead range must be < 2 GiB");
  if (p.conv_in != nullptr) {
    FLITE_REQUIRE(p.conv_c % 64 == 0, "conv: input channels must be a multiple of 64");
    FLITE_REQUIRE(p.K == 9 * p.conv_c, "conv: K must be 9 * C_in");
    FLITE_REQUIRE(p.conv_oh == (p.conv_up ? 2 : 1) * p.conv_ih && p.conv_ow == (p.conv_up ? 2 : 1) * p.conv_iw,
                  "conv: output size must equal input size (x2 with upsample)");
    FLITE_REQUIRE(p.conv_in_bytes < (1L << 31), "conv: input must be < 2 GiB (32-bit buffer offsets)");
    FLITE_REQUIRE(epi == EPI_STORE_BF16 || epi == EPI_STORE_F32, "conv: store epilogues only");
  } else {
    FLITE_REQUIRE(p.lda % 8 == 0, "gemm: lda must be a multiple of 8 elements");
    FLITE_REQUIRE((long)p.M * p.lda * 2 < (1L << 32), "gemm: A must be < 4 GiB (32-bit buffer offsets)");
    FLITE_REQUIRE(((uintptr_t)p.A & 15) == 0, "gemm: A must be 16-B aligned");
  }
  if (gemm_init()) return 1;
  switch (epi) {
    case EPI_STORE_BF16:
      FLITE_REQUIRE(p.ldo % 4 == 0 || p.N < 4, "gemm: ldo must be a multiple of 4 (or N < 4)");
      launch<EPI_STORE_BF16>(p, stream);
      break;
    case EPI_STORE_F32:
      FLITE_REQUIRE(p.ldo % 4 == 0 || p.N < 4, "gemm: ldo must be a multiple of 4 (or N < 4)");
      launch<EPI_STORE_F32>(p, stream);
      break;
    case EPI_RESID_F32:
      FLITE_REQUIRE(p.N % 4 == 0 && p.ldo % 4 == 0, "gemm(resid): N, ldo must be multiples of 4");
      FLITE_REQUIRE(p.gate == nullptr || p.rows_per_seg > 0, "gemm(resid): rows_per_seg must be > 0");
      FLITE_REQUIRE(p.out_seg == 0 && p.act == 0, "gemm(resid): no row remap or activation");
      launch<EPI_RESID_F32>(p, stream);
      break;
    case EPI_RESID_BF16:
      FLITE_REQUIRE(p.N % 4 == 0 && p.ldo % 4 == 0 && ((uintptr_t)p.out & 7) == 0,
                    "gemm(resid bf16): N, ldo multiples of 4, 8-B aligned rows");
      FLITE_REQUIRE(p.gate == nullptr || p.rows_per_seg > 0, "gemm(resid): rows_per_seg must be > 0");
      FLITE_REQUIRE(p.out_seg == 0 && p.act == 0, "gemm(resid): no row remap or activation");
      launch<EPI_RESID_BF16>(p, stream);
      break;
    case EPI_QKV_NORM_BF16:
      FLITE_REQUIRE(p.N % 256 == 0 && p.ldo % 4 == 0 && p.norm_cols % 256 == 0 && p.rope_cols % 256 == 0 &&
                        p.rope_cols <= p.norm_cols && p.norm_cols <= p.N,
                    "gemm(qkv_norm): heads of 256 columns (N, norm_cols, rope_cols multiples of 256)");
      FLITE_REQUIRE(p.rope_cols == 0 || (p.rope.cs && p.rope.tokens > 0 && p.rope.h > 0 && p.rope.w > 0),
                    "gemm(qkv_norm): RoPE tables missing");
      FLITE_REQUIRE(p.out_seg == 0 && p.act == 0 && p.resid == nullptr, "gemm(qkv_norm): plain row layout only");
      launch<EPI_QKV_NORM_BF16>(p, stream);
      break;
    case EPI_SWIGLU_BF16:
      FLITE_REQUIRE(p.W2 != nullptr, "gemm(swiglu): up weight missing");
      FLITE_REQUIRE(p.N % 32 == 0, "gemm(swiglu): F must be a multiple of 16");
      FLITE_REQUIRE(p.bias == nullptr, "gemm(swiglu): bias not supported");
      launch<EPI_SWIGLU_BF16>(p, stream);
      break;
    case EPI_GEGLU_BF16:
      FLITE_REQUIRE(p.W2 != nullptr, "gemm(geglu): wi_1 weight missing");
      FLITE_REQUIRE(p.N % 32 == 0, "gemm(geglu): F must be a multiple of 16");
      FLITE_REQUIRE(p.bias == nullptr, "gemm(geglu): bias not supported");
      launch<EPI_GEGLU_BF16>(p, stream);
      break;
    default:
      FLITE_REQUIRE(false, "gemm: unknown epilogue");
  }
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace flite
