// Prototype (tools only): the hd-256 flash attention with TWO waves per SIMD. A workgroup of 8 waves takes 128
// query rows; the waves w and w ^ 4 share 32 query rows (pair w & 3) and split each 64-key tile: wave half
// h = w >> 2 computes S for keys [32h, 32h + 32) over the full head (Q^T in 64 AGPRs), its softmax and P, and
// O for the head-dim half [128h, 128h + 128) (64 AGPRs) over ALL 64 keys -- the other 32 keys' P comes from the
// partner wave through LDS (2 KiB per wave, lane-linear: both waves hold P in the same register layout). Per
// wave and tile: 16 S + 16 O MFMAs, 8 LDS-DMA pieces, 16 softmax elements -- half of attention.hip's, with a
// second wave on the SIMD to fill the MFMA pipe while one issues DMA / softmax / waits.
// Bounded softmax only (fixed shift), full 128-row q-tiles only (no tail split). Question it answers: does the
// second wave per SIMD beat attention.hip's one-wave kernel (MFMA busy 0.51)? Driver: tools/attn_pair_bench.py.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "common.h"

using namespace flite;

namespace {

constexpr int QT = 128, KT = 64, HD = 256, NT = 512;
constexpr int TILE = KT * HD * 2;  // 32 KiB
constexpr int K_OFF = 0, V_OFF = 2 * TILE, P_OFF = 4 * TILE;
constexpr int P_SLOT = 2048;                      // one wave's P: 64 lanes x 32 B
constexpr int LDS_BYTES = 4 * TILE + 2 * 8 * P_SLOT;  // 160 KiB

typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;

__device__ __forceinline__ s16x4 ds_tr16(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(p));
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
__device__ __forceinline__ void blds16(const i32x4& rsrc, unsigned voff, unsigned lds_addr) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rsrc), "s"(lds_addr)
      : "memory");
}
template <bool NOP>
__device__ __forceinline__ void mfma_o(f32x16& acc, const bf16x8& v, bf16x8& pk) {
  if constexpr (NOP)
    asm("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %2, %1, %0" : "+a"(acc), "+v"(pk) : "v"(v));
  else
    asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(v), "v"(pk));
}
__device__ __forceinline__ void mfma_s_first(f32x16& acc, const bf16x8& k, const bf16x8& q) {
  asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(k), "a"(q));
}
__device__ __forceinline__ void mfma_s(f32x16& acc, const bf16x8& k, const bf16x8& q) {
  asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(k), "a"(q));
}
__device__ __forceinline__ void mfma_read_fence(f32x16& a) { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+v"(a)); }
__device__ __forceinline__ void o_acc_fence(f32x16 (&o)[4]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+a"(o[0]), "+a"(o[1]), "+a"(o[2]), "+a"(o[3]));
}
__device__ __forceinline__ unsigned lds_addr_of(const void* p) {
  return (unsigned)(unsigned long long)(const LDS_AS char*)p;
}
__device__ __forceinline__ int xcd_remap(int bid, int n) {
  const int xcd = bid & 7, q8 = n >> 3, r8 = n & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
}

struct P {
  const bf16_t *q, *k, *v;
  bf16_t* o;
  long q_row_stride, k_row_stride, v_row_stride, o_row_stride;
  long q_head_stride, k_head_stride, v_head_stride, o_head_stride;
  const int *cu_q, *cu_k;
  int B, H, n_main;
  float scale, max_score;
};

__global__ __launch_bounds__(NT, 1) void attn_pair_kernel(P p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pq = wave & 3;   // query block of 32 rows
  const int hf = wave >> 2;  // key half of S / head-dim half of O
  int b, h, q0;
  {
    const int v = xcd_remap(blockIdx.x, gridDim.x);
    q0 = (v % p.n_main) * QT;
    const int pair = v / p.n_main;
    h = pair % p.H;
    b = pair / p.H;
  }
  const int q_start = p.cu_q[b];
  const int q_len = p.cu_q[b + 1] - q_start;
  if (q0 >= q_len) return;
  const int k_start = p.cu_k[b];
  const int k_len = p.cu_k[b + 1] - k_start;
  const int lq = lane & 31;
  const int hh = lane >> 5;
  const int q_row = q0 + pq * 32 + lq;
  const int nt = (k_len + KT - 1) / KT;

  bf16x8 qf[16];
  {
    const int qc = min(q_row, q_len - 1);
    const bf16_t* qp = p.q + (long)(q_start + qc) * p.q_row_stride + (long)h * p.q_head_stride + 8 * hh;
#pragma unroll
    for (int s = 0; s < 16; ++s) qf[s] = *(const bf16x8*)(qp + 16 * s);
#pragma unroll
    for (int s = 0; s < 16; ++s) asm volatile("" : "+a"(qf[s]));
    asm volatile("s_nop 4" ::: "memory");
  }

  // staging: 4 K + 4 V pieces per wave per tile; piece i covers tile rows 2 (4 wave + i) + {0, 1}
  const long k_base = (long)k_start * p.k_row_stride + (long)h * p.k_head_stride;
  const long v_base = (long)k_start * p.v_row_stride + (long)h * p.v_head_stride;
  const unsigned lds0 = (unsigned)__builtin_amdgcn_readfirstlane((int)lds_addr_of(smem));
  unsigned k_src[4], v_src[4];  // (dead in the ping-pong build: only the one-phase loop's copies use them)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 2 * (wave * 4 + i) + hh;
    const int pos = lane & 31;
    const int kc = pos ^ (row & 15);
    const int vc = (((pos >> 2) ^ (row & 3)) << 2) | (pos & 3);
    k_src[i] = (unsigned)(row * p.k_row_stride * 2 + kc * 16);
    v_src[i] = (unsigned)(row * p.v_row_stride * 2 + vc * 16);
  }
  auto rsrc_tile = [&](const bf16_t* base, long off, long stride, int t, bool live) {
    const long rows_left = live ? k_len - (long)t * KT : 0;
    return make_rsrc(base + off + (long)t * KT * stride, (unsigned)max(0L, min(rows_left * stride * 2, 0x7fffffffL)));
  };

  f32x16 o_acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o_acc[i][r] = 0.f;
  const float sl2 = p.scale * 1.4426950408889634f;
  const float m_run = p.max_score * 1.4426950408889634f;
  float l_run = 0.f;

  const char* kbase = smem + K_OFF + (32 * hf + lq) * 512;  // key row 32 hf + lq of the tile
  // chunk (2s + hh) ^ (lq & 15) of the key row: s >= 8 is s - 8's chunk + 16 (256 B), an immediate
  int k_off[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) k_off[s] = ((2 * s + hh) ^ (lq & 15)) << 4;
  auto koff = [&](int s) { return k_off[s & 7] + (s >> 3) * 256; };
  const int G = lane >> 4;
  const int vq = (lane & 15) >> 2;
  const int vp = lane & 3;
  const char* vbase = smem + V_OFF + (4 * (G >> 1) + vq) * 512 + (16 * (G & 1) + 4 * vp) * 2;
  int v_off[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) v_off[dt] = ((4 * hf + dt) ^ vq) * 64;
  // P exchange slots: [parity][wave] x 2 KiB as [2 steps][64 lanes] x 16 B (conflict-free b128 accesses)
  const unsigned pslot_own = lds0 + P_OFF + wave * P_SLOT + lane * 16;
  const unsigned pslot_par = lds0 + P_OFF + (wave ^ 4) * P_SLOT + lane * 16;

#ifndef PAIR_KAHEAD
#define PAIR_KAHEAD 3
#endif
#ifndef PAIR_VAHEAD
#define PAIR_VAHEAD 4
#endif
#ifndef PAIR_DMA
#define PAIR_DMA 0  // 0: one piece per even k-step; 1: all 8 after the first k-step; 2: one per k-step from s = 8
#endif
  constexpr int KAHEAD = PAIR_KAHEAD, VAHEAD = PAIR_VAHEAD;
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using BT = std::integral_constant<bool, true>;
  using BF = std::integral_constant<bool, false>;
  f32x16 sh;          // S of this wave's key half, tile whose softmax is pending
  u32x4 pa[2], pb[2];  // own P^T operands (16-key steps s = 0, 1 of the own half) of two consecutive tiles

  auto phase_a = [&](auto kb_, auto dkb_, auto dvb_, auto dma_, int tk, bool k_live, int tv, bool v_live) {
    constexpr int KB = decltype(kb_)::value, DKB = decltype(dkb_)::value, DVB = decltype(dvb_)::value;
    constexpr bool DMA = decltype(dma_)::value;
    const char* Kb = kbase + KB * TILE;
    i32x4 krs = {0, 0, 0, 0}, vrs = {0, 0, 0, 0};
    if constexpr (DMA) {
      krs = rsrc_tile(p.k, k_base, p.k_row_stride, tk, k_live);
      vrs = rsrc_tile(p.v, v_base, p.v_row_stride, tv, v_live);
    }
    bf16x8 kf[16];
#pragma unroll
    for (int s = 0; s < KAHEAD; ++s) kf[s] = *(const bf16x8*)(Kb + koff(s));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s + KAHEAD < 16) kf[s + KAHEAD] = *(const bf16x8*)(Kb + koff(s + KAHEAD));
      __builtin_amdgcn_sched_barrier(0);
      if (s == 0)
        mfma_s_first(sh, kf[0], qf[0]);
      else
        mfma_s(sh, kf[s], qf[s]);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (DMA) {
        auto piece = [&](int i) {  // 0..7: K pieces 0..3, then V pieces 0..3
          if (i < 4)
            blds16(krs, k_src[i], lds0 + DKB * TILE + (wave * 4 + i) * 1024 + K_OFF);
          else
            blds16(vrs, v_src[i - 4], lds0 + DVB * TILE + (wave * 4 + i - 4) * 1024 + V_OFF);
        };
        if (PAIR_DMA == 0 && (s & 1) == 0) piece(s >> 1);
        if (PAIR_DMA == 1 && s == 0)
          for (int i = 0; i < 8; ++i) piece(i);
        if (PAIR_DMA == 2 && s >= 8) piece(s - 8);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    mfma_read_fence(sh);
  };
  // softmax of element e (0..15) of sh into the own P operand pn[e >> 3]
  auto softmax_elem = [&](u32x4 (&pn)[2], int e, float& e_prev) {
    const float v = __builtin_amdgcn_exp2f(sh[e] * sl2 - m_run);
    l_run += v;
    if (e & 1) {
      const bf16x2 pr = {(__bf16)e_prev, (__bf16)v};
      pn[e >> 3][(e & 7) >> 1] = __builtin_bit_cast(unsigned, pr);
    }
    e_prev = v;
  };
  // phase B: O^T(head-dim half) += V^T . P^T over all 64 keys of Vbuf[VB]; own P pc (keys of half hf), the
  // partner's (other half) from its LDS slot of parity PP; EX: the softmax of the pending S into pn
  auto phase_b = [&](auto vb_, auto pp_, auto ex_, u32x4 (&pc)[2], u32x4 (&pn)[2]) {
    constexpr int VB = decltype(vb_)::value, PP = decltype(pp_)::value;
    constexpr bool EX = decltype(ex_)::value;
    const char* Vb = vbase + VB * TILE;
    u32x4 px[2];
    px[0] = *(const LDS_AS u32x4*)(pslot_par + PP * 8 * P_SLOT);
    px[1] = *(const LDS_AS u32x4*)(pslot_par + PP * 8 * P_SLOT + 1024);
    float e_prev = 0.f;
    // MFMA m = 4 g + dt: g = (half, s) with the own key half first (its P in registers) and the partner's second;
    // V^T from key rows 32 kh + 16 s (+8) of the tile, head-dim tile 4 hf + dt
    const char* vb_h[2] = {Vb + hf * 32 * 512, Vb + (hf ^ 1) * 32 * 512};
    s16x4 lo[16], hi[16];
    auto rd = [&](int m) {
      const int g = m >> 2, dt = m & 3, o = g >> 1, s = g & 1;
      lo[m] = ds_tr16(vb_h[o] + (16 * s) * 512 + v_off[dt]);
      hi[m] = ds_tr16(vb_h[o] + (16 * s + 8) * 512 + v_off[dt]);
    };
#pragma unroll
    for (int m = 0; m < VAHEAD; ++m) rd(m);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      if (m + VAHEAD < 16) rd(m + VAHEAD);
      __builtin_amdgcn_sched_barrier(0);
      const int g = m >> 2, dt = m & 3, o = g >> 1, s = g & 1;
      const s16x8 c = __builtin_shufflevector(lo[m], hi[m], 0, 1, 2, 3, 4, 5, 6, 7);
      const bf16x8 vf = __builtin_bit_cast(bf16x8, c);
      bf16x8 pk = __builtin_bit_cast(bf16x8, o == 0 ? pc[s] : px[s]);
      if (dt == 0)
        mfma_o<true>(o_acc[dt], vf, pk);
      else
        mfma_o<false>(o_acc[dt], vf, pk);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (EX) softmax_elem(pn, m, e_prev);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto publish = [&](const u32x4 (&pn)[2], int par) {
    *(LDS_AS u32x4*)(pslot_own + par * 8 * P_SLOT) = pn[0];
    *(LDS_AS u32x4*)(pslot_own + par * 8 * P_SLOT + 1024) = pn[1];
  };
#define ATTN_TILE_SYNC()                             \
  do {                                               \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); \
    __syncthreads();                                 \
  } while (0)
  // iteration j (parity PJ = j & 1): phase A for S_{j+1} (HS), phase B for PV_j (P_j own + partner's of slot
  // parity PJ) with the softmax of S_{j+1}; P_{j+1} own published to slot parity PJ ^ 1
  auto iter = [&](auto par_, auto hs_, int j) {
    constexpr int PJ = decltype(par_)::value;
    constexpr bool HS = decltype(hs_)::value;
    if constexpr (HS) {
      if constexpr (PJ == 0)
        phase_a(I1{}, I0{}, I1{}, BT{}, j + 2, j + 2 < nt, j + 1, true);
      else
        phase_a(I0{}, I1{}, I0{}, BT{}, j + 2, j + 2 < nt, j + 1, true);
    }
    if constexpr (PJ == 0) {
      phase_b(I0{}, I0{}, hs_, pa, pb);
      if constexpr (HS) publish(pb, 1);
    } else {
      phase_b(I1{}, I1{}, hs_, pb, pa);
      if constexpr (HS) publish(pa, 0);
    }
    ATTN_TILE_SYNC();
  };
#ifndef PAIR_PINGPONG
#define PAIR_PINGPONG 0
#endif
#if PAIR_PINGPONG
  // Ping-pong with ONE instruction stream: every wave runs  [A_j; barrier; B_j; wait own copies; barrier]  for
  // j = 0.., but the key-half-1 waves (Y) pass one extra barrier first and the half-0 waves (X) one at the end,
  // so between any two barriers X runs B_j while Y runs A_j, or X A_{j+1} while Y B_j: a SIMD's two waves are
  // always in opposite phases (one reading K, doing S MFMAs and LDS-DMA; the other reading V, doing O MFMAs and
  // the softmax). X stages the K tiles (K_{j+2} in A_j), Y the V tiles (V_{j+1} in A_j); each role waits for its
  // own copies after its B phase, one phase before their first reader. The role is data only (source, stride,
  // LDS region, tile offset): both roles share the code, so nothing is duplicated and nothing spills.
  const bool X = hf == 0;
  unsigned src8[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = 2 * ((wave & 3) * 8 + i) + hh;
    const int pos = lane & 31;
    src8[i] = X ? (unsigned)(row * p.k_row_stride * 2 + ((pos ^ (row & 15)) * 16))
                : (unsigned)(row * p.v_row_stride * 2 + (((((pos >> 2) ^ (row & 3)) << 2) | (pos & 3)) * 16));
  }
  const bf16_t* dsrc = X ? p.k + k_base : p.v + v_base;
  const long dstride = X ? p.k_row_stride : p.v_row_stride;
  const int dshift = X ? 2 : 1;
  const unsigned dreg = lds0 + (X ? K_OFF : V_OFF) + (wave & 3) * 8 * 1024;
  // A_j: S_{j+1} from Kbuf[KB]; this role's tile j + dshift into its buffer (tile & 1)
  auto phase_a_pp = [&](auto kb_, int j) {
    constexpr int KB = decltype(kb_)::value;
    const char* Kb = kbase + KB * TILE;
    const int td = j + dshift;
    const long rows_left = td < nt ? k_len - (long)td * KT : 0;
    const i32x4 rs = make_rsrc(dsrc + (long)td * KT * dstride, (unsigned)max(0L, min(rows_left * dstride * 2, 0x7fffffffL)));
    const unsigned dst = (unsigned)__builtin_amdgcn_readfirstlane((int)(dreg + (td & 1) * TILE));
    bf16x8 kf[16];
#pragma unroll
    for (int s = 0; s < KAHEAD; ++s) kf[s] = *(const bf16x8*)(Kb + koff(s));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s + KAHEAD < 16) kf[s + KAHEAD] = *(const bf16x8*)(Kb + koff(s + KAHEAD));
      __builtin_amdgcn_sched_barrier(0);
      if (s == 0)
        mfma_s_first(sh, kf[0], qf[0]);
      else
        mfma_s(sh, kf[s], qf[s]);
      __builtin_amdgcn_sched_barrier(0);
      if ((s & 1) == 0) blds16(rs, src8[s >> 1], dst + (s >> 1) * 1024);
      __builtin_amdgcn_sched_barrier(0);
    }
    mfma_read_fence(sh);
  };
  // B_j: O += V_j P_j (own in pc, partner's from parity j & 1), softmax of S_{j+1} (EX) into pn -> parity (j+1) & 1
  auto B = [&](auto pj_, auto ex_, u32x4 (&pc)[2], u32x4 (&pn)[2]) {
    constexpr int PJ = decltype(pj_)::value;
    constexpr bool EX = decltype(ex_)::value;
    phase_b(std::integral_constant<int, PJ>{}, std::integral_constant<int, PJ>{}, ex_, pc, pn);
    if constexpr (EX) publish(pn, PJ ^ 1);
  };
  auto end_b = [&]() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  if (nt > 0) {
    {  // X: K_0 into Kbuf 0 and K_1 into Kbuf 1; Y: V_0 into Vbuf 0
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (!X && t == 1) break;
        const long rows_left = t < nt ? k_len - (long)t * KT : 0;
        const i32x4 rs = make_rsrc(dsrc + (long)t * KT * dstride, (unsigned)max(0L, min(rows_left * dstride * 2, 0x7fffffffL)));
#pragma unroll
        for (int i = 0; i < 8; ++i) blds16(rs, src8[i], dreg + t * TILE + i * 1024);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    phase_a(I0{}, I0{}, I0{}, BF{}, 0, false, 0, false);  // S_0
    {
      float e_prev = 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) softmax_elem(pa, e, e_prev);
    }
    publish(pa, 0);
    __syncthreads();
    if (!X) __syncthreads();  // Y runs one phase behind X
    // pa holds P_j for even j, pb for odd j
    int j = 0;
    for (; j + 2 < nt; j += 2) {
      phase_a_pp(I1{}, j);
      __syncthreads();
      B(I0{}, BT{}, pa, pb);
      end_b();
      phase_a_pp(I0{}, j + 1);
      __syncthreads();
      B(I1{}, BT{}, pb, pa);
      end_b();
    }
    if (nt - j == 2) {
      phase_a_pp(I1{}, j);
      __syncthreads();
      B(I0{}, BT{}, pa, pb);
      end_b();
      __syncthreads();  // (no A_{nt-1})
      B(I1{}, BF{}, pb, pa);
      end_b();
    } else {
      __syncthreads();  // (no A_{nt-1})
      B(I0{}, BF{}, pa, pb);
      end_b();
    }
    if (X) __syncthreads();
  }
#else
  if (nt > 0) {
    {  // K_0, V_0 into buffer 0, K_1 into Kbuf 1
      const i32x4 k0 = rsrc_tile(p.k, k_base, p.k_row_stride, 0, true);
      const i32x4 v0 = rsrc_tile(p.v, v_base, p.v_row_stride, 0, true);
      const i32x4 k1 = rsrc_tile(p.k, k_base, p.k_row_stride, 1, nt > 1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        blds16(k0, k_src[i], lds0 + (wave * 4 + i) * 1024 + K_OFF);
        blds16(v0, v_src[i], lds0 + (wave * 4 + i) * 1024 + V_OFF);
        blds16(k1, k_src[i], lds0 + TILE + (wave * 4 + i) * 1024 + K_OFF);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    phase_a(I0{}, I0{}, I0{}, BF{}, 0, false, 0, false);
    {
      float e_prev = 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) softmax_elem(pa, e, e_prev);
    }
    publish(pa, 0);
    __syncthreads();  // K_0 reads done before iteration 0 refills Kbuf 0; P_0 published
    int j = 0;
    for (; j + 2 < nt; j += 2) {
      iter(I0{}, BT{}, j);
      iter(I1{}, BT{}, j + 1);
    }
    if (nt - j == 2) {
      iter(I0{}, BT{}, j);
      iter(I1{}, BF{}, j + 1);
    } else {
      iter(I0{}, BF{}, j);
    }
  }
#endif
  o_acc_fence(o_acc);
  // row sums: lanes l, l + 32 hold complementary keys of the half; padded keys (zero rows of the last tile)
  // each added exp2(-m); then the partner's half through LDS
  l_run += __shfl_xor(l_run, 32, 64);
  {
    const int valid_last = k_len - (nt - 1) * KT;  // 1..64 keys of the last tile
    const int pad_h = 32 - min(max(valid_last - 32 * hf, 0), 32);
    l_run -= (float)pad_h * __builtin_amdgcn_exp2f(-m_run);
  }
  *(LDS_AS float*)(lds0 + P_OFF + wave * 256 + lq * 4) = l_run;  // P slots are idle after the last sync
  __syncthreads();
  l_run += *(const LDS_AS float*)(lds0 + P_OFF + (wave ^ 4) * 256 + lq * 4);

  if (q_row >= q_len) return;
  const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
  bf16_t* orow = p.o + (long)(q_start + q_row) * p.o_row_stride + (long)h * p.o_head_stride + 128 * hf;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int rp = 0; rp < 2; ++rp) {
      const int ra = 8 * rp, rb = 8 * rp + 4;
      unsigned a0 = pack2bf(o_acc[i][ra + 0] * inv, o_acc[i][ra + 1] * inv);
      unsigned a1 = pack2bf(o_acc[i][ra + 2] * inv, o_acc[i][ra + 3] * inv);
      unsigned b0 = pack2bf(o_acc[i][rb + 0] * inv, o_acc[i][rb + 1] * inv);
      unsigned b1 = pack2bf(o_acc[i][rb + 2] * inv, o_acc[i][rb + 3] * inv);
      const auto x0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
      const auto x1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
      const u32x4 w = {x0[0], x1[0], x0[1], x1[1]};
      *(u32x4*)(orow + i * 32 + 16 * rp + 8 * hh) = w;
    }
  }
}

}  // namespace

// q/k/v/o [B*T, H, 256] bf16 (row stride H*256), cu_q = cu_k = [0, T, 2T, ...] on the device; T % 128 == 0
extern "C" int attn_pair_proto(const void* q, const void* k, const void* v, void* o, const int* cu_q,
                               const int* cu_k, int B, int H, int T, float scale, float max_score, void* stream) {
  if (T % QT) return 2;
  static bool init = false;
  if (!init) {
    if (hipFuncSetAttribute((const void*)attn_pair_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES))
      return 1;
    init = true;
  }
  P p;
  p.q = (const bf16_t*)q;
  p.k = (const bf16_t*)k;
  p.v = (const bf16_t*)v;
  p.o = (bf16_t*)o;
  p.q_row_stride = p.k_row_stride = p.v_row_stride = p.o_row_stride = (long)H * HD;
  p.q_head_stride = p.k_head_stride = p.v_head_stride = p.o_head_stride = HD;
  p.cu_q = cu_q;
  p.cu_k = cu_k;
  p.B = B;
  p.H = H;
  p.n_main = T / QT;
  p.scale = scale;
  p.max_score = max_score;
  hipLaunchKernelGGL(attn_pair_kernel, dim3(B * H * p.n_main), dim3(NT), LDS_BYTES, (hipStream_t)stream, p);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
