// Flash-attention forward for head_dim 256 with 256 query rows per workgroup (gfx950, bounded softmax): the DiT's
// self-attention (reference f_lite/model.py:203-210, flash_attn_varlen_func over the CFG-batched image tokens).
//
// Why a second kernel. attention.hip runs 128 query rows per workgroup (4 waves x 32) over 64-key tiles. Per tile
// and CU it moves 64 KiB of K/V by LDS-DMA (64 one-KiB pieces: 1024 cycles of the texture path at 64 B/clk, the
// whole of its S-phase MFMA time) and every wave reads the whole K and V tile from LDS for its 32 rows
// (256 KiB of LDS reads per 2048 MFMA cycles). Here each wave owns 64 query rows (two 32-row blocks qb 0/1) over
// 32-key tiles: every K fragment and every V^T fragment read from LDS feeds two MFMAs (one per block), so per
// MFMA the staged bytes, the LDS-DMA pieces and the LDS reads all halve. The price is registers: O for 64 rows x
// 256 columns is 256 fp32 per lane (all 256 AGPRs) and Q^T for 64 rows is 128 VGPRs; S (2 x 32 keys) and the P
// operands fit beside them because the key tile is 32 wide.
//
// Per 32-key tile and wave (the pipelined key loop of attention.hip, same phases, same bit-exact sum orders):
//   phase A: S_{j+1}[qb] = K_{j+1} . Q^T[qb]   16 K-fragment reads, 32 MFMAs, 8 LDS-DMA pieces (K_{j+2}, V_{j+1})
//   phase B: O^T[qb] += V_j^T . P_j^T[qb]      16 V^T fragments (32 transposed reads), 32 MFMAs, the softmax of
//                                              S_{j+1} (32 exp2 + row sums + bf16 packs), one per MFMA
//
// Schedule. At T = 4112 a sequence has 16 full 256-row q-tiles and a 16-row tail; B = 2, H = 12 give 384 full
// tiles, 1.5 rounds of 256 CUs. So the launcher splits: the first n_whole full tiles run over all keys, the other
// n_half run as two key halves (each a workgroup), and each pair's tail rows run as n_tail key chunks. Split pieces
// write unnormalised (O, l) slabs (write-through) and bump a counter; the last arriver adds the slabs in a fixed
// order (deterministic) and normalises. The bounded softmax has no running max, so partial sums add without any
// rescale. The split counts come from a list-scheduling simulation of the hardware dispatcher (q256_plan).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <map>
#include <mutex>
#include <queue>
#include <vector>

#include "attn_common.h"
#include "common.h"
#include "fp8.h"
#include "kernels.h"

namespace flite {

namespace {

constexpr int QW = 64;             // query rows per wave
constexpr int QT = 4 * QW;         // query rows per workgroup
constexpr int KT = 32;             // keys per tile
constexpr int HD = 256;            // head dim
constexpr int NT = 256;            // threads
constexpr int TILE = KT * HD * 2;  // 16 KiB: one K or V tile
// LDS: [K buf0 | K buf1 | V buf0 | V buf1]
constexpr int K_OFF = 0;
constexpr int V_OFF = 2 * TILE;
constexpr int LDS_BYTES = 4 * TILE;  // 64 KiB
// slab: O^T accumulators lane-linear [wave 4][qb 2][dt 8][r4 4][lane 64] f32x4, then l [wave 4][qb 2][lane 64]
constexpr int SLAB_O_F4 = 4 * 2 * 8 * 4 * 64;
constexpr int SLAB_FLOATS = SLAB_O_F4 * 4 + 4 * 2 * 64;
constexpr long SLAB_BYTES = (long)SLAB_FLOATS * 4;
// counters at the workspace start: one per split tile, one per tail pair. The same 4 KiB block as the 128-row
// kernel's (attention.hip CNT_BYTES): a caller's workspace serves both kernels (the engine's attn_ws_), whose slabs
// overwrite everything past it, and each launch leaves its counters zeroed, so only this block must stay zero.
constexpr long CNT_BYTES = 4096;
constexpr int MAX_TAIL = 16;       // key chunks per tail
constexpr int MIN_KEYS = 1024;     // shorter key ranges keep the 128-row kernel (a tile's prologue dominates)

struct Q256Params {
  AttnParams a;
  int n_main;       // full 256-row q-tiles per (sequence, head)
  int n_whole;      // full tiles [0, n_whole) (pair-major) over all keys
  int n_half;       // full tiles [n_whole, n_whole + n_half) as two key halves
  int n_tail;       // key chunks of each pair's tail rows (0: none)
};

template <int N>
__device__ __forceinline__ void o_fence16(f32x16 (&o)[16]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3"
               : "+a"(o[8 * N + 0]), "+a"(o[8 * N + 1]), "+a"(o[8 * N + 2]), "+a"(o[8 * N + 3]), "+a"(o[8 * N + 4]),
                 "+a"(o[8 * N + 5]), "+a"(o[8 * N + 6]), "+a"(o[8 * N + 7]));
}

__global__ __launch_bounds__(NT, 1) void attn_q256_kernel(Q256Params P) {
  const AttnParams& p = P.a;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // ---- work decode: [whole tiles][key halves of the split tiles][tail chunks], each segment XCD-remapped ----
  const int pairs = p.B * p.H;
  const int nW = P.n_whole, nS = P.n_half, nTl = P.n_tail > 0 ? pairs * P.n_tail : 0;
  int pair, q0, chunk = 0, nchunk = 1, cnt_i = 0;
  long slab_i = 0;
  {
    const int bid = blockIdx.x;
    if (bid < nW) {
      const int f = xcd_remap(bid, nW);
      pair = f / P.n_main;
      q0 = (f % P.n_main) * QT;
    } else if (bid < nW + 2 * nS) {
      const int v = xcd_remap(bid - nW, 2 * nS);  // the two halves of a tile are neighbours on one XCD
      const int f = nW + (v >> 1);
      pair = f / P.n_main;
      q0 = (f % P.n_main) * QT;
      chunk = v & 1;
      nchunk = 2;
      cnt_i = v >> 1;
      slab_i = (long)(v >> 1) * 2;
    } else {
      const int v = xcd_remap(bid - nW - 2 * nS, nTl);
      pair = v / P.n_tail;
      chunk = v % P.n_tail;
      nchunk = P.n_tail;
      q0 = P.n_main * QT;
      cnt_i = nS + pair;
      slab_i = (long)nS * 2 + (long)pair * P.n_tail;
    }
  }
  const int h = pair % p.H;
  const int b = pair / p.H;
  const int q_start = p.cu_q[b];
  const int q_len = p.cu_q[b + 1] - q_start;
  const int rows = min(QT, q_len - q0);
  if (rows <= 0) return;  // uniform over the workgroup (and over every chunk of a tile)
  const int k_start = p.cu_k[b];
  const int k_len = p.cu_k[b + 1] - k_start;
  const bool live = wave * QW < rows;  // wave-uniform: this wave has query rows

  const int lq = lane & 31;
  const int hh = lane >> 5;

  const int nk = k_len > 0 ? (k_len + KT - 1) / KT : 0;
  int t_begin = 0, t_end = nk;
  if (nchunk > 1) {
    const int per = (nk + nchunk - 1) / nchunk;
    t_begin = min(chunk * per, nk);
    t_end = min(t_begin + per, nk);
  }
  const int nt = t_end - t_begin;

  // ---- Q^T fragments of both 32-row blocks in VGPRs (128), pre-scaled to log2 units (attention.hip: one bf16
  // rounding of q). Measured alternative: block 1 kept in LDS and read beside each K fragment frees 64 VGPRs but
  // made phase A LDS-read-bound (2 x 4096 x 4096, H 8: 236.5 vs 222.1 us) ----
  bf16x8 qf[32];
  {
    const float qs = p.scale * 1.4426950408889634f;
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      const int qc = min(q0 + wave * QW + qb * 32 + lq, q_len - 1);
      const bf16_t* qp = p.q + (long)(q_start + qc) * p.q_row_stride + (long)h * p.q_head_stride + 8 * hh;
#pragma unroll
      for (int s = 0; s < 16; ++s) qf[qb * 16 + s] = *(const bf16x8*)(qp + 16 * s);
#pragma unroll
      for (int s = 0; s < 16; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[qb * 16 + s][j] = (__bf16)((float)qf[qb * 16 + s][j] * qs);
    }
  }

  // ---- staging: 4 K + 4 V LDS-DMA pieces per wave per tile; piece i of wave w covers tile rows 2(4w+i), +1 ----
  const long k_base = (long)k_start * p.k_row_stride + (long)h * p.k_head_stride;
  const long v_base = (long)k_start * p.v_row_stride + (long)h * p.v_head_stride;
  const unsigned lds0 = (unsigned)__builtin_amdgcn_readfirstlane((int)lds_addr_of(smem));
  // Per-lane source byte offsets of piece i, and (below) the K fragment read offsets, are derived inside each phase A
  // from an opaque copy of the lane index (`lane_a`): hipcc would otherwise hoist the 8 + 8 loop-invariant values
  // into registers that stay allocated through phase B, where the register file is full (Q^T 128, S 32, P 32).
  const unsigned krow_b = (unsigned)(p.k_row_stride * 2), vrow_b = (unsigned)(p.v_row_stride * 2);
  auto k_src = [&](int i, int ln) __attribute__((always_inline)) {
    const int row = 2 * (wave * 4 + i) + (ln >> 5), pos = ln & 31;
    return (unsigned)row * krow_b + (unsigned)((pos ^ (row & 15)) * 16);  // K: 16-B chunk XOR (row & 15)
  };
  auto v_src = [&](int i, int ln) __attribute__((always_inline)) {
    const int row = 2 * (wave * 4 + i) + (ln >> 5), pos = ln & 31;
    return (unsigned)row * vrow_b + (unsigned)(((((pos >> 2) ^ (row & 3)) << 2) | (pos & 3)) * 16);  // V: 64-B XOR
  };
  const unsigned k_tile_b = (unsigned)(KT * p.k_row_stride * 2), v_tile_b = (unsigned)(KT * p.v_row_stride * 2);
  const long k_total_b = (long)k_len * p.k_row_stride * 2, v_total_b = (long)k_len * p.v_row_stride * 2;
  const char* k_ptr0 = (const char*)(p.k + k_base);
  const char* v_ptr0 = (const char*)(p.v + v_base);
  auto rsrc_tile = [&](const char* base, unsigned tile_b, long total_b, int t, bool on) __attribute__((always_inline)) {
    const unsigned long off = (unsigned long)(unsigned)t * tile_b;
    const long left = total_b - (long)off;
    const int hi = (int)(left >> 32);
    const unsigned lo = (unsigned)left;
    const unsigned range = (!on || hi < 0) ? 0u : (hi > 0 || lo > 0x7fffffffu) ? 0x7fffffffu : lo;
    return make_rsrc(base + off, range);
  };

  f32x16 o_acc[16];  // [qb * 8 + d-tile]
#pragma unroll
  for (int qb = 0; qb < 2; ++qb)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) o_acc[qb * 8 + i][r] = 0.f;
  float l_run[2] = {0.f, 0.f};

  // per-lane LDS read bases. K (A operand of S^T): row lq, k-step s reads chunk (2s + hh) ^ (lq & 15), i.e.
  // (s >> 3) * 256 B + ((2 (s & 7) + hh) ^ (lq & 15)) * 16 (the XOR leaves chunk bit 4 alone)
  const char* kbase = smem + K_OFF + lq * 512;
  // V (tr-read): group G = lane >> 4, li = lane & 15 -> row vq = li >> 2, 4-column piece vp = li & 3; d-tile dt at
  // (dt >> 2) * 256 B + voff[dt & 3]
  const int G = lane >> 4;
  const int vq = (lane & 15) >> 2;
  const int vp = lane & 3;
  const char* vbase = smem + V_OFF + (4 * (G >> 1) + vq) * 512 + (16 * (G & 1) + 4 * vp) * 2;
  int voff[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) voff[d] = (d ^ vq) * 64;

  typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using BT = std::integral_constant<bool, true>;
  using BF = std::integral_constant<bool, false>;
  constexpr int KAHEAD = 2;  // K (+ block-1 Q) fragments read this many k-steps ahead
  constexpr int VAHEAD = 2;  // V^T fragments read this many fragments (= 4 MFMAs) ahead
  static_assert(VAHEAD >= 1, "attn_common.h mfma_o: the read-ahead block separates the softmax from the PV MFMAs");
  f32x16 s0, s1;             // S^T of the pending tile: query block 0 / 1
  u32x4 pa[4], pb[4];        // P^T operands [qb * 2 + 16-key step] of two consecutive tiles, bf16 pairs

  // phase A. KB: K buffer read; DKB / DVB: buffers the K / V copies land in; DMA: copies issued; LIVE: MFMAs run
  auto phase_a = [&](auto kb_, auto dkb_, auto dvb_, auto dma_, auto live_, int tk, bool k_on, int tv, bool v_on) __attribute__((always_inline)) {
    constexpr int KB = decltype(kb_)::value, DKB = decltype(dkb_)::value, DVB = decltype(dvb_)::value;
    constexpr bool DMA = decltype(dma_)::value, LIVE = decltype(live_)::value;
    const char* Kb = kbase + KB * TILE;
    i32x4 krs = {0, 0, 0, 0}, vrs = {0, 0, 0, 0};
    if constexpr (DMA) {
      krs = rsrc_tile(k_ptr0, k_tile_b, k_total_b, tk, k_on);
      vrs = rsrc_tile(v_ptr0, v_tile_b, v_total_b, tv, v_on);
    }
    int lane_a = lane;
    asm volatile("" : "+v"(lane_a));  // opaque per phase: the offsets below are not hoisted out of the key loop
    const int kx = lane_a & 15, kh = lane_a >> 5;
    bf16x8 kf[16];
    auto rdk = [&](int s) __attribute__((always_inline)) {
      const int off = (s >> 3) * 256 + (((2 * (s & 7) + kh) ^ kx) << 4);
      kf[s] = *(const bf16x8*)(Kb + off);
    };
    if constexpr (LIVE) {
#pragma unroll
      for (int s = 0; s < KAHEAD; ++s) rdk(s);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if constexpr (LIVE) {
        if (s + KAHEAD < 16) rdk(s + KAHEAD);
        __builtin_amdgcn_sched_barrier(0);
        if (s == 0) {
          mfma_sv_first(s0, kf[0], qf[0]);
          mfma_sv_first(s1, kf[0], qf[16]);
        } else {
          mfma_sv(s0, kf[s], qf[s]);
          mfma_sv(s1, kf[s], qf[16 + s]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (DMA) {  // K pieces first (needed first), then V: one per two k-steps
        if ((s & 1) == 0) {
          const int i = s >> 1;
          if (i < 4)
            blds16(krs, k_src(i, lane_a), lds0 + DKB * TILE + (wave * 4 + i) * 1024 + K_OFF);
          else
            blds16(vrs, v_src(i - 4, lane_a), lds0 + DVB * TILE + (wave * 4 + i - 4) * 1024 + V_OFF);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (LIVE) {
      mfma_read_fence(s0, s1);  // MFMA write of S -> VALU read (softmax in the next phase B)
    }
  };
  // softmax of score e (0..31: block e >> 4, register r = e & 15) of the pending S into the P^T operand pn; the row
  // sum adds the PREVIOUS score's p (same adds, same order; no v_add waiting on the v_exp just issued)
  auto softmax_elem = [&](u32x4 (&pn)[4], int e, float& e_prev) __attribute__((always_inline)) {
    const int qb = e >> 4, r = e & 15;
    const float v = __builtin_amdgcn_exp2f(qb ? s1[r] : s0[r]);
    if (e > 0) l_run[(e - 1) >> 4] += e_prev;
    if (e & 1) {
      const bf16x2 pr = {(__bf16)e_prev, (__bf16)v};
      pn[qb * 2 + (r >> 3)][(r & 7) >> 1] = __builtin_bit_cast(unsigned, pr);
    }
    e_prev = v;
  };
  // phase B: O^T += V^T . P^T (operands pc) from Vbuf[VB]; EX: the softmax of the pending S into pn
  auto phase_b = [&](auto vb_, auto ex_, u32x4 (&pc)[4], u32x4 (&pn)[4]) __attribute__((always_inline)) {
    constexpr int VB = decltype(vb_)::value;
    constexpr bool EX = decltype(ex_)::value;
    const char* Vb = vbase + VB * TILE;
    float e_prev = 0.f;
    // fragment f = 8 s + dt (16-key step s, d-tile dt) feeds MFMAs 2f (block 0) and 2f + 1 (block 1)
    s16x4 lo[16], hi[16];
    auto rd = [&](int f) __attribute__((always_inline)) {
      const int s = f >> 3, dt = f & 7;
      lo[f] = ds_tr16(Vb + (16 * s) * 512 + (dt >> 2) * 256 + voff[dt & 3]);
      hi[f] = ds_tr16(Vb + (16 * s + 8) * 512 + (dt >> 2) * 256 + voff[dt & 3]);
    };
#pragma unroll
    for (int f = 0; f < VAHEAD; ++f) rd(f);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int m = 0; m < 32; ++m) {
      const int f = m >> 1, qb = m & 1, s = f >> 3, dt = f & 7;
      if (qb == 0 && f + VAHEAD < 16) rd(f + VAHEAD);
      __builtin_amdgcn_sched_barrier(0);
      const s16x8 c = __builtin_shufflevector(lo[f], hi[f], 0, 1, 2, 3, 4, 5, 6, 7);
      const bf16x8 vf = __builtin_bit_cast(bf16x8, c);
      // P was packed a whole phase A earlier (no VALU -> MFMA hazard left to clear), so it is read in place: the NOP
      // form's "+v" operand would make hipcc copy each block's P into a scratch register set before every group
      bf16x8 pk = __builtin_bit_cast(bf16x8, pc[qb * 2 + s]);
      mfma_o<false>(o_acc[qb * 8 + dt], vf, pk);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (EX) softmax_elem(pn, m, e_prev);
      __builtin_amdgcn_sched_barrier(0);
    }  // the P operands of the last two MFMAs
    if constexpr (EX) l_run[1] += e_prev;
  };
  // iteration j (parity PAR): phase A for S_{j+1} (HS) and phase B for PV_j with the softmax of S_{j+1}
  // Every iteration runs both phases, also past the last tile (phase A then computes the S of a tile past the range
  // from zero-filled copies, and its softmax is kept out of the row sums): one code path for every tile. A remainder
  // iteration outside the loop had its own register assignment, and there hipcc moved O accumulators through AGPR
  // copies (v_accvgpr_write / mov) right before the asm MFMAs reading them, a VALU -> MFMA hazard it cannot see
  // through the asm (measured: wrong d-tiles of block 1 in the last tile); a mid-loop exit spilled O to scratch.
  auto iter = [&](auto par_, auto live_, int j) __attribute__((always_inline)) {
    constexpr int PAR = decltype(par_)::value;
    constexpr bool LIVE = decltype(live_)::value;
    const bool next = j + 1 < nt;  // the tile whose S phase A computes exists
    if constexpr (PAR == 0)
      phase_a(I1{}, I0{}, I1{}, BT{}, live_, t_begin + j + 2, j + 2 < nt, t_begin + j + 1, next);
    else
      phase_a(I0{}, I1{}, I0{}, BT{}, live_, t_begin + j + 2, j + 2 < nt, t_begin + j + 1, next);
    if constexpr (LIVE) {
      const float l0 = l_run[0], l1 = l_run[1];
      if constexpr (PAR == 0)
        phase_b(I0{}, BT{}, pa, pb);
      else
        phase_b(I1{}, BT{}, pb, pa);
      l_run[0] = next ? l_run[0] : l0;
      l_run[1] = next ? l_run[1] : l1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  auto key_loop = [&](auto live_) __attribute__((always_inline)) {
    constexpr bool LIVE = decltype(live_)::value;
    // prologue: K_0, V_0 into buffer 0 and K_1 into Kbuf 1; S_0 and its softmax into pa
    {
      const i32x4 krs = rsrc_tile(k_ptr0, k_tile_b, k_total_b, t_begin, true);
      const i32x4 vrs = rsrc_tile(v_ptr0, v_tile_b, v_total_b, t_begin, true);
      const i32x4 krs1 = rsrc_tile(k_ptr0, k_tile_b, k_total_b, t_begin + 1, nt > 1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        blds16(krs, k_src(i, lane), lds0 + (wave * 4 + i) * 1024 + K_OFF);
        blds16(vrs, v_src(i, lane), lds0 + (wave * 4 + i) * 1024 + V_OFF);
        blds16(krs1, k_src(i, lane), lds0 + TILE + (wave * 4 + i) * 1024 + K_OFF);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if constexpr (LIVE) {
      phase_a(I0{}, I0{}, I0{}, BF{}, live_, 0, false, 0, false);
      float e_prev = 0.f;
#pragma unroll
      for (int e = 0; e < 32; ++e) softmax_elem(pa, e, e_prev);
      l_run[1] += e_prev;
    }
    __syncthreads();  // every wave's K_0 reads are done before iteration 0 refills Kbuf 0
    int j = 0;
    // tiles in pairs, one exit: with nt odd the last pair's second tile is a ghost whose V copy was staged as zeros
    // (v_on false), so its PV adds exact zeros to O, and whose softmax was kept out of the row sums
    for (; j < nt; j += 2) {
      iter(I0{}, live_, j);
      iter(I1{}, live_, j + 1);
    }
  };
  if (nt > 0) {
    if (live)
      key_loop(BT{});
    else
      key_loop(BF{});  // no query rows: stage this wave's share of every tile and keep the barriers
  }
  o_fence16<0>(o_acc);
  o_fence16<1>(o_acc);

  // keys past the end were staged as zero rows: each contributed exp2(0) = 1 to l and 0 to O
  const int n_pad = (nt > 0 && t_end == nk) ? nk * KT - k_len : 0;
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    l_run[qb] += __shfl_xor(l_run[qb], 32, 64);  // the two lane halves hold the sums of complementary keys
    l_run[qb] -= (float)n_pad;
  }

  if (nchunk > 1) {
    // ---- split hand-off (MI355X guide §6 G16: write-through payload, vmcnt drain, relaxed counter) ----
    char* slab0 = (char*)p.split_ws + CNT_BYTES + (size_t)slab_i * SLAB_BYTES;
    if (live) {
      const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(slab0 + (size_t)chunk * SLAB_BYTES), (short)0, (int)SLAB_BYTES, 0x00020000);
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int r4 = 0; r4 < 4; ++r4) {
            const f32x4 v = {o_acc[qb * 8 + i][4 * r4], o_acc[qb * 8 + i][4 * r4 + 1], o_acc[qb * 8 + i][4 * r4 + 2],
                             o_acc[qb * 8 + i][4 * r4 + 3]};
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), srs,
                                                   ((((wave * 2 + qb) * 8 + i) * 4 + r4) * 64 + lane) * 16, 0,
                                                   16 /* sc1 */);
          }
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(l_run[qb]), srs,
                                              SLAB_O_F4 * 16 + ((wave * 2 + qb) * 64 + lane) * 4, 0, 16 /* sc1 */);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* cnt = (int*)p.split_ws + cnt_i;
    volatile LDS_AS int* flag = (volatile LDS_AS int*)lds0;  // K/V buffers are idle now
    if (tid == 0) *flag = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (*flag != nchunk - 1) return;  // not the last arriver (uniform)
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (tid == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (nchunk == 2) {
      // two key halves: the last arriver adds the other half's slab to its own registers (a + b == b + a, so the
      // sum is the same whichever half came last); batches of 16 loads bound the registers in flight
      if (!live) return;
      const float* sl = (const float*)(slab0 + (size_t)(chunk ^ 1) * SLAB_BYTES);
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        l_run[qb] += sl[SLAB_O_F4 * 4 + (wave * 2 + qb) * 64 + lane];
#pragma unroll
        for (int ib = 0; ib < 8; ib += 4) {
          f32x4 v[4][4];
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4)
              v[i][r4] = *(const f32x4*)(sl + ((((wave * 2 + qb) * 8 + ib + i) * 4 + r4) * 64 + lane) * 4);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4)
#pragma unroll
              for (int e = 0; e < 4; ++e) o_acc[qb * 8 + ib + i][4 * r4 + e] += v[i][r4][e];
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    } else {
      // tail chunks: the whole workgroup sums every chunk's slab in chunk order (deterministic), normalises and
      // stores the live rows; the row sums first, into LDS after the flag word
      const int n_live_w = (rows + QW - 1) / QW;
      volatile LDS_AS float* lsum = (volatile LDS_AS float*)(lds0 + 16);
      const int ns = nchunk;
      if (tid < n_live_w * 128) {
        float lv[MAX_TAIL];
#pragma unroll
        for (int c = 0; c < MAX_TAIL; ++c)
          lv[c] = ((const float*)(slab0 + (size_t)min(c, ns - 1) * SLAB_BYTES))[SLAB_O_F4 * 4 + tid];
        float l = 0.f;
#pragma unroll
        for (int c = 0; c < MAX_TAIL; ++c) l += c < ns ? lv[c] : 0.f;
        lsum[tid] = l;
      }
      __syncthreads();
      for (int e = tid; e < n_live_w * 4096; e += NT) {
        const int w = e >> 12, qb = (e >> 11) & 1, i = (e >> 8) & 7, r4 = (e >> 6) & 3, ln = e & 63;
        const int row = q0 + w * QW + qb * 32 + (ln & 31);
        if (row >= q_len) continue;
        f32x4 v[MAX_TAIL];
#pragma unroll
        for (int c = 0; c < MAX_TAIL; ++c)
          v[c] = *(const f32x4*)((const float*)(slab0 + (size_t)min(c, ns - 1) * SLAB_BYTES) + e * 4);
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < MAX_TAIL; ++c)
          if (c < ns) acc += v[c];
        const float l = lsum[(w * 2 + qb) * 64 + ln];
        const float inv = l > 0.f ? 1.f / l : 0.f;
        const int d = i * 32 + 8 * r4 + 4 * (ln >> 5);
        u32x2 st;
        st.x = pack2bf(acc[0] * inv, acc[1] * inv);
        st.y = pack2bf(acc[2] * inv, acc[3] * inv);
        *(u32x2*)(p.o + (long)(q_start + row) * p.o_row_stride + (long)h * p.o_head_stride + d) = st;
      }
      if (p.o8) {  // the tail rows' MXFP8 copy, from the bf16 rows this workgroup just stored (as attention.hip)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        for (int t = tid; t < rows * 8; t += NT) {
          const int row = q0 + (t >> 3), i = t & 7;
          const long grow = q_start + row;
          const u32x4* src = (const u32x4*)(p.o + grow * p.o_row_stride + (long)h * p.o_head_stride + i * 32);
          float x[32];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const u32x4 w = src[q];
            const unsigned ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              x[8 * q + 2 * j] = __uint_as_float(ws[j] << 16);
              x[8 * q + 2 * j + 1] = __uint_as_float(ws[j] & 0xffff0000u);
            }
          }
          float amax = 0.f;
#pragma unroll
          for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(x[j]));
          const int e = mx_exp(amax);
          const float is = mx_inv(e);
          u32x4 o[2];
#pragma unroll
          for (int hf = 0; hf < 2; ++hf)
            o[hf] = u32x4{pack4_fp8(x + 16 * hf, is), pack4_fp8(x + 16 * hf + 4, is), pack4_fp8(x + 16 * hf + 8, is),
                          pack4_fp8(x + 16 * hf + 12, is)};
          u32x4* dst = (u32x4*)(p.o8 + grow * p.o_row_stride + (long)h * p.o_head_stride + i * 32);
          dst[0] = o[0];
          dst[1] = o[1];
          const long kb = (long)h * (HD / 32) + i;
          p.o8_scale[((kb >> 2) * p.o8_rows_pad + grow) * 4 + (kb & 3)] = (uint8_t)(e + 127);
        }
      }
      return;
    }
  }

  // ---- store: lane (row, hh) holds columns i*32 + 8*r4 + 4*hh + 0..3 of its row (attention.hip's epilogue) ----
  if (!live) return;
  if (p.o8) {  // MXFP8 straight from the accumulators (the fp8 DiT's proj operand; attention.hip's o8 epilogue)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      const int q_row = q0 + wave * QW + qb * 32 + lq;
      const bool ok = q_row < q_len;
      const float inv = l_run[qb] > 0.f ? 1.f / l_run[qb] : 0.f;
      const long grow = q_start + min(q_row, q_len - 1);
      uint8_t* o8row = p.o8 + grow * p.o_row_stride + (long)h * p.o_head_stride;
      unsigned sc_lo = 0, sc_hi = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float x[16];
        float amax = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          x[r] = bf2f(f2bf(o_acc[qb * 8 + i][r] * inv));  // the bf16 value quant_rows_fp8 would have read
          amax = fmaxf(amax, fabsf(x[r]));
        }
        amax = fmaxf(amax, __shfl_xor(amax, 32, 64));
        const int e = mx_exp(amax);
        const float is = mx_inv(e);
        unsigned d[4];
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) d[r4] = pack4_fp8(x + 4 * r4, is);  // columns 8 r4 + 4 hh + 0..3
#pragma unroll
        for (int rp = 0; rp < 2; ++rp) {
          const auto w = __builtin_amdgcn_permlane32_swap(d[2 * rp], d[2 * rp + 1], false, false);
          if (ok) *(u32x2*)(o8row + i * 32 + 16 * rp + 8 * hh) = u32x2{w[0], w[1]};
        }
        const unsigned byte = (unsigned)(e + 127) << (8 * (i & 3));
        if (i < 4) sc_lo |= byte; else sc_hi |= byte;
      }
      const long kt = (long)h * (HD / 128) + hh;  // the row's 8 block scales of this head: two 128-deep k-tiles
      if (ok) *(unsigned*)(p.o8_scale + (kt * p.o8_rows_pad + grow) * 4) = hh ? sc_hi : sc_lo;
    }
    return;
  }
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int q_row = q0 + wave * QW + qb * 32 + lq;
    const bool ok = q_row < q_len;  // lanes l and l + 32 hold the same row: the swap pairs stay whole
    const float inv = l_run[qb] > 0.f ? 1.f / l_run[qb] : 0.f;
    bf16_t* orow = p.o + (long)(q_start + min(q_row, q_len - 1)) * p.o_row_stride + (long)h * p.o_head_stride;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int rp = 0; rp < 2; ++rp) {
        const int ra = 8 * rp, rb = 8 * rp + 4;
        unsigned a0 = pack2bf(o_acc[qb * 8 + i][ra + 0] * inv, o_acc[qb * 8 + i][ra + 1] * inv);
        unsigned a1 = pack2bf(o_acc[qb * 8 + i][ra + 2] * inv, o_acc[qb * 8 + i][ra + 3] * inv);
        unsigned b0 = pack2bf(o_acc[qb * 8 + i][rb + 0] * inv, o_acc[qb * 8 + i][rb + 1] * inv);
        unsigned b1 = pack2bf(o_acc[qb * 8 + i][rb + 2] * inv, o_acc[qb * 8 + i][rb + 3] * inv);
        const auto x0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
        const auto x1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
        const u32x4 w = {x0[0], x1[0], x0[1], x1[1]};
        if (ok) *(u32x4*)(orow + i * 32 + 16 * rp + 8 * hh) = w;
      }
    }
  }
}

// ---- host: the split plan ----
struct Plan {
  int n_whole = 0, n_half = 0, n_tail = 0;
  long ws_bytes = 0;
  bool wins = false;  // predicted faster than the 128-row kernel's schedule (route policy)
  double t256 = 0, t128 = 0;
};

// Makespan of the item list on `cus` CUs when each CU takes the next item as it frees (the dispatcher, to first
// order). Costs in key tiles: a workgroup's prologue (Q + first K/V) ~ 4 tiles, a two-way hand-off ~ 2.
double simulate(int cus, int n_whole, int n_half, int pairs, int n_tail, int nk, int tail_rows) {
  std::priority_queue<double, std::vector<double>, std::greater<double>> q;
  for (int i = 0; i < cus; ++i) q.push(0.0);
  double end = 0.0;
  auto run = [&](double c) {
    const double t = q.top() + c;
    q.pop();
    q.push(t);
    end = std::max(end, t);
  };
  // a 32-key iteration of this kernel costs 0.96 of a 64-key iteration of the 128-row kernel (the same MFMA work;
  // measured 222.1 vs 231.8 us on 2 x 4096 x 4096, H 8, one round of each); the prologue (the Q burst) ~6
  const double it = 0.96, pro = 6.0;
  for (int i = 0; i < n_whole; ++i) run(it * (nk + (nk & 1)) + pro);  // an odd count runs one ghost iteration
  const int half = (nk + 1) / 2;
  for (int i = 0; i < 2 * n_half; ++i) run(it * (half + (half & 1)) + pro + 2.0);  // + the slab hand-off
  if (n_tail > 0) {
    const int per = (nk + n_tail - 1) / n_tail;
    const double live = (tail_rows + QW - 1) / QW;  // live waves: MFMA work of the chunk relative to a full tile
    for (int i = 0; i < pairs * n_tail; ++i)
      run(it * (per + (per & 1)) * std::max(0.35, live / 4.0) + pro * 0.5 + 0.5 * n_tail / 4.0);
  }
  return end;
}

// The 128-row kernel's schedule (attention.hip attn_fwd) in the same units: full 128-row q-tiles over every 64-key
// tile, then the tail chunks (min(CUs / pairs, 16) key ranges per pair)
double simulate128(int cus, int pairs, int max_q, int max_k) {
  std::priority_queue<double, std::vector<double>, std::greater<double>> q;
  for (int i = 0; i < cus; ++i) q.push(0.0);
  double end = 0.0;
  auto run = [&](double c) {
    const double t = q.top() + c;
    q.pop();
    q.push(t);
    end = std::max(end, t);
  };
  const int nk = (max_k + 63) / 64, n_main = max_q / 128, tail = max_q - 128 * n_main;
  const double pro = 4.0;
  for (int i = 0; i < pairs * n_main; ++i) run(nk + pro);
  if (tail > 0) {
    const int S = std::max(1, std::min(cus / pairs, 16));
    const int per = (nk + S - 1) / S;
    for (int i = 0; i < pairs * S; ++i) run(per + pro * 0.5 + 0.5 * S / 4.0);
  }
  return end;
}

Plan make_plan(int cus, int pairs, int max_q, int max_k) {
  Plan pl;
  const int n_main = max_q / QT;
  const int tail_rows = max_q - n_main * QT;
  const int F = pairs * n_main;
  const int nk = (max_k + KT - 1) / KT;
  double best = 1e30;
  static const int kTails[] = {1, 2, 3, 4, 6, 8, 10, 12, 16};
  for (int ti = 0; ti < (tail_rows > 0 ? 9 : 1); ++ti) {
    const int nt = tail_rows > 0 ? kTails[ti] : 0;
    // halving more than two rounds' worth of tiles only lengthens the list (a half costs 0.6 of a whole tile), so
    // the search stops there: O(CUs * F) simulations instead of O(F^2) for large batches
    for (int s = 0; s <= std::min(F, 2 * cus); ++s) {
      const double m = simulate(cus, F - s, s, pairs, nt, nk, tail_rows);
      if (m < best - 1e-9) {
        best = m;
        pl.n_whole = F - s;
        pl.n_half = s;
        pl.n_tail = nt;
      }
    }
  }
  // diagnostic A/B switch: FLITE_Q256_PLAN="<split tiles>,<tail chunks>" (clamped to the launch's tiles)
  if (const char* f = getenv("FLITE_Q256_PLAN")) {
    int hs = 0, ts = 1;
    if (sscanf(f, "%d,%d", &hs, &ts) == 2) {
      pl.n_half = std::max(0, std::min(hs, F));
      pl.n_whole = F - pl.n_half;
      pl.n_tail = tail_rows > 0 ? std::max(1, std::min(ts, MAX_TAIL)) : 0;
    }
  }
  pl.ws_bytes = CNT_BYTES + ((long)pl.n_half * 2 + (long)pairs * pl.n_tail) * SLAB_BYTES;
  pl.t256 = simulate(cus, pl.n_whole, pl.n_half, pairs, pl.n_tail, nk, tail_rows);
  pl.t128 = simulate128(cus, pairs, max_q, max_k);
  // margin 4.5 %: measured against the prediction (2 x T self-attention, 12 heads): T = 4720 predicted 0.949, measured
  // 473 vs 505 us (taken); T = 4112 predicted 0.972, 405 vs 384 us; T = 9232 predicted 0.960, 1856 vs 1783 us
  pl.wins = pl.t256 < 0.955 * pl.t128;
  if (getenv("FLITE_Q256_VERBOSE"))
    fprintf(stderr, "[q256] pairs %d max_q %d max_k %d: %d whole + %d split tiles, %d tail chunks; predicted %.1f vs "
            "%.1f (128-row kernel): %s\n", pairs, max_q, max_k, pl.n_whole, pl.n_half, pl.n_tail, pl.t256, pl.t128,
            pl.wins ? "256-row" : "128-row");
  return pl;
}

// Route state: the mode and key floor are atomics set once from the environment (std::call_once) and by
// flite_attn_set_q256; the kernel attribute and the CU count are per device; plans are cached per (CUs, pairs,
// max_q, max_k) under g_plan_mu, and the cache is cleared past kMaxPlans entries (a varlen caller whose lengths
// change every batch would otherwise grow it without bound; a plan is rebuilt in well under a millisecond).
std::mutex g_plan_mu;
std::map<std::tuple<int, int, int, int>, Plan> g_plans;
constexpr size_t kMaxPlans = 256;
std::map<int, int> g_dev_cus;  // device -> CU count, present once the attribute is set on that device
std::once_flag g_env_once;
std::atomic<int> g_q256_mode{2};  // 0 never, 1 always, 2 by the plan's prediction
std::atomic<int> g_min_keys{MIN_KEYS};

// the CU count of the current device (0 on failure), setting the kernel attribute there on first use
int q256_init() {
  std::call_once(g_env_once, [] {
    // route policy: by default a launch takes the 256-row kernel where its split plan is predicted
    // >= 4.5 % faster than the 128-row kernel's schedule (the 1344x896 self-attention, T = 4720: 465 vs 495 us
    // measured; not at 1024^2, T = 4112, whose 768 128-row q-tiles are exactly 3 rounds of 256 CUs: 401 vs 375 us).
    // FLITE_ATTN_Q256=1 / 0 or flite_attn_set_q256(1 / 0): always / never (the tests and A/B tools)
    const char* on = getenv("FLITE_ATTN_Q256");
    g_q256_mode = !on ? 2 : on[0] == '1' ? 1 : 0;
    if (const char* mk = getenv("FLITE_Q256_MIN_KEYS")) g_min_keys = std::max(KT, atoi(mk));  // A/B: key-range floor
  });
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> g(g_plan_mu);
  auto it = g_dev_cus.find(dev);
  if (it != g_dev_cus.end()) return it->second;
  int cus = 0;
  if (hipFuncSetAttribute((const void*)attn_q256_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) !=
          hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  g_dev_cus[dev] = cus;
  return cus;
}

// the plan for this launch shape on the current device (copied out: the cache may be cleared by another thread)
bool plan_for(int pairs, int max_q, int max_k, Plan* out) {
  const int cus = q256_init();
  if (cus <= 0) return false;
  std::lock_guard<std::mutex> g(g_plan_mu);
  const auto key = std::make_tuple(cus, pairs, max_q, max_k);
  auto it = g_plans.find(key);
  if (it == g_plans.end()) {
    if (g_plans.size() >= kMaxPlans) g_plans.clear();
    it = g_plans.emplace(key, make_plan(cus, pairs, max_q, max_k)).first;
  }
  *out = it->second;
  return true;
}

}  // namespace

int attn_q256_set(int mode) {
  q256_init();  // the environment's choice is read first, so this call wins over it
  g_q256_mode = mode < 0 ? 0 : mode > 2 ? 2 : mode;
  return 0;
}

bool attn_q256_eligible(const AttnParams& p) {
  if (q256_init() <= 0 || g_q256_mode == 0) return false;
  return p.head_dim == HD && p.max_score > 0.f && p.part_mode == 0 && !p.k_end && p.split_ws &&
         p.max_q >= QT && p.max_k >= g_min_keys && p.B * p.H * (p.max_q / QT) <= (int)(CNT_BYTES / 4) - p.B * p.H;
}

long attn_q256_workspace_bytes(int B, int H, int max_q, int max_k) {
  if (q256_init() <= 0 || max_q < QT || max_k < g_min_keys) return 0;
  // launches past the counter block never take this route (attn_q256_eligible): no plan, no slabs
  if ((long)B * H * (max_q / QT) > (long)(CNT_BYTES / 4) - (long)B * H) return 0;
  Plan pl;
  return plan_for(B * H, max_q, max_k, &pl) ? pl.ws_bytes : 0;
}

// attn_fwd's route for eligible launches whose workspace holds the plan's slabs; returns -1 when it does not apply
int attn_q256_fwd(const AttnParams& p, hipStream_t stream) {
  if (!attn_q256_eligible(p)) return -1;
  Plan pl;
  if (!plan_for(p.B * p.H, p.max_q, p.max_k, &pl) || pl.ws_bytes > p.split_ws_bytes || (g_q256_mode == 2 && !pl.wins))
    return -1;
  Q256Params q;
  q.a = p;
  q.n_main = p.max_q / QT;
  q.n_whole = pl.n_whole;
  q.n_half = pl.n_half;
  q.n_tail = pl.n_tail;
  const int pairs = p.B * p.H;
  dim3 grid(q.n_whole + 2 * q.n_half + pairs * q.n_tail);
  hipLaunchKernelGGL(attn_q256_kernel, grid, dim3(NT), LDS_BYTES, stream, q);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace flite
