// Flash-attention forward for head_dim 256 on gfx950 (non-causal, varlen via cu_seqlens).
//
// Replaces flash_attn_interface.flash_attn_varlen_func (reference f_lite/model.py:203-210), used for the
// self-attention over the CFG-batched image tokens (cu_seqlens = [0, T, 2T, ...]) and the cross-attention
// onto the text context (cu_seqlens_k from the context mask, model.py:530).
//
// Workgroup = 4 waves (one per SIMD, up to 512 registers each) = 128 query rows of one (sequence, head);
// wave w owns 32 query rows and sweeps every 64-key tile (two 32-key S^T tiles).
// Per tile and wave:  S^T = K . Q^T  (v_mfma_f32_32x32x16_bf16, K fragments from LDS, Q^T in registers)
//   -> query index on the lane, keys in registers: softmax sums are lane-local (+1 swap at the end);
//   O^T += V^T . P^T  with P^T taken straight from the S^T accumulator registers (no LDS round trip) and
//   V^T fragments read with ds_read_b64_tr_b16 (hardware transpose) from a row-major, XOR-swizzled V tile.
// K/V tiles stream HBM->LDS with buffer_load ... lds (swizzle on the source address; keys past the sequence
// end read as zeros through the buffer range check), double-buffered; the loop is unrolled over the two
// buffers so every LDS address is a per-lane base + an immediate offset.
#include "common.h"
#include "kernels.h"

namespace flite {

namespace {

constexpr int QT = 128;     // query rows per workgroup
constexpr int KT = 64;      // keys per tile
constexpr int HD = 256;     // head dim
constexpr int NT = 256;
constexpr int TILE = KT * HD * 2;  // 32 KiB: one K or V tile
// LDS: [K buf0 | K buf1 | V buf0 | V buf1]
constexpr int K_OFF = 0;
constexpr int V_OFF = 2 * TILE;
constexpr int LDS_BYTES = 4 * TILE;  // 128 KiB

__device__ __forceinline__ s16x4 ds_tr16(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(p));
}

typedef __attribute__((ext_vector_type(4))) int i32x4;

// Buffer descriptor (raw, stride 0) from wave-uniform values (readfirstlane makes uniformity provable).
__device__ __forceinline__ i32x4 make_rsrc(const void* base, unsigned bytes) {
  const unsigned long long a = (unsigned long long)base;
  i32x4 r;
  r.x = __builtin_amdgcn_readfirstlane((int)(a & 0xffffffffu));
  r.y = __builtin_amdgcn_readfirstlane((int)(a >> 32));
  r.z = __builtin_amdgcn_readfirstlane((int)bytes);
  r.w = 0x00020000;
  return r;
}

// 16-B-per-lane LDS-DMA: LDS[m0 + lane*16] = buffer[voff] (0 when voff is out of range). Inline asm on
// purpose: hipcc counts a builtin LDS-DMA in vmcnt and then waits for it (vmcnt(0)) before every later
// ds_read, serialising the next tile's prefetch with this tile's compute; the waits are placed by hand
// (vmcnt(0) + barrier at the end of each tile).
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

__device__ __forceinline__ unsigned lds_addr_of(const void* p) {
  return (unsigned)(unsigned long long)(const LDS_AS char*)p;
}

// BOUNDED: every score s*scale is known to lie in [-max_score, max_score] (QK-normed q and k: |q|,|k| <= 16
// for head_dim 256, so |q.k|/16 <= 16 -- model.py:180,197 precede every attention call of the DiT). Softmax is
// shift-invariant, so the running max is replaced by the fixed bound: no row max, no O/l rescale, p <= 1.
template <bool BOUNDED>
__global__ __launch_bounds__(NT, 1) void attn_fwd_hd256_kernel(AttnParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  // XCD-aware mapping of the 1-D grid: workgroups are dealt round-robin over the 8 XCDs (bid % 8), so the
  // bijective remap gives each XCD a contiguous range of (sequence, head, q-tile) work in which consecutive
  // workgroups share one (sequence, head) and its K/V stream.
  int b, h, qt;
  {
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    qt = v % p.n_qtiles;
    const int pair = v / p.n_qtiles;
    h = pair % p.H;
    b = pair / p.H;
  }

  const int q_start = p.cu_q[b];
  const int q_len = p.cu_q[b + 1] - q_start;
  if (qt * QT >= q_len) return;  // uniform over the workgroup
  const int k_start = p.cu_k[b];
  const int k_len = p.cu_k[b + 1] - k_start;

  const int lq = lane & 31;
  const int hh = lane >> 5;
  const int q_row = qt * QT + wave * 32 + lq;  // this lane's query (within the sequence)

  if (k_len <= 0) {  // no keys: output zeros
    if (q_row < q_len) {
      bf16_t* o = p.o + (long)(q_start + q_row) * p.o_row_stride + (long)h * p.o_head_stride;
      for (int d = hh * 128; d < hh * 128 + 128; d += 4) *(u32x2*)(o + d) = u32x2{0u, 0u};
    }
    return;
  }

  // ---- Q^T fragments (B operand): lane holds Q[q][16s + 8*hh + j], s = 0..15 ----
  bf16x8 qf[16];
  {
    const int qc = min(q_row, q_len - 1);
    const bf16_t* qp = p.q + (long)(q_start + qc) * p.q_row_stride + (long)h * p.q_head_stride + 8 * hh;
#pragma unroll
    for (int s = 0; s < 16; ++s) qf[s] = *(const bf16x8*)(qp + 16 * s);
  }

  // ---- staging: 8 K + 8 V LDS-DMA pieces per wave per tile; piece qi covers tile rows 2qi, 2qi+1.
  // Keys >= k_len get an out-of-range offset -> the buffer range check returns zeros.
  const i32x4 krs = make_rsrc(p.k + (long)k_start * p.k_row_stride + (long)h * p.k_head_stride, 0x7fffffffu);
  const i32x4 vrs = make_rsrc(p.v + (long)k_start * p.v_row_stride + (long)h * p.v_head_stride, 0x7fffffffu);
  const unsigned lds0 = (unsigned)__builtin_amdgcn_readfirstlane((int)lds_addr_of(smem));
  unsigned k_src[8], v_src[8];  // byte offsets of this lane's piece elements for key row `row` (tile 0)
  int st_row[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = 2 * (wave * 8 + i) + hh;
    const int pos = lane & 31;
    const int kc = pos ^ (row & 15);                              // K: 16-B chunk XOR (row & 15)
    const int vc = (((pos >> 2) ^ (row & 3)) << 2) | (pos & 3);   // V: 64-B block XOR (row & 3)
    st_row[i] = row;
    k_src[i] = (unsigned)(kc * 16);
    v_src[i] = (unsigned)(vc * 16);
  }
  auto stage = [&](int t, int buf) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int qi = wave * 8 + i;
      const int key = t * KT + st_row[i];
      const bool ok = key < k_len;
      const unsigned ko = ok ? (unsigned)(key * p.k_row_stride * 2) + k_src[i] : 0x80000000u;
      const unsigned vo = ok ? (unsigned)(key * p.v_row_stride * 2) + v_src[i] : 0x80000000u;
      const unsigned dst = (unsigned)__builtin_amdgcn_readfirstlane((int)(lds0 + buf * TILE + qi * 1024));
      blds16(krs, ko, dst + K_OFF);
      blds16(vrs, vo, dst + V_OFF);
    }
  };

  f32x16 o_acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o_acc[i][r] = 0.f;
  const float sl2 = p.scale * 1.4426950408889634f;
  float m_run = BOUNDED ? p.max_score * 1.4426950408889634f : -1e30f;
  float l_run = 0.f;

  // per-lane LDS read bases (everything else is an immediate offset)
  // K (A operand of S^T): row lq of the 32-key half, chunk (2s + hh) ^ (lq & 15)
  const char* kbase = smem + K_OFF + lq * 512;
  int k_off[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) k_off[s] = ((2 * s + hh) ^ (lq & 15)) << 4;
  // V (tr-read): group G = lane>>4, li = lane&15 -> row vq = li>>2, 4-column piece vp = li&3
  const int G = lane >> 4;
  const int vq = (lane & 15) >> 2;
  const int vp = lane & 3;
  const char* vbase = smem + V_OFF + (4 * (G >> 1) + vq) * 512 + (16 * (G & 1) + 4 * vp) * 2;
  int v_off[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) v_off[dt] = (dt ^ vq) * 64;

  auto compute = [&](const int buf) {
    const char* Kb = kbase + buf * TILE;
    const char* Vb = vbase + buf * TILE;
    // S^T for both 32-key halves: all 32 K fragments first, two independent accumulation chains
    f32x16 s0, s1;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s0[r] = 0.f;
      s1[r] = 0.f;
    }
    bf16x8 k0[16], k1[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      k0[s] = *(const bf16x8*)(Kb + k_off[s]);
      k1[s] = *(const bf16x8*)(Kb + 32 * 512 + k_off[s]);
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k0[s], qf[s], s0, 0, 0, 0);
      s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k1[s], qf[s], s1, 0, 0, 0);
    }
    // schedule: 8 fragment reads ahead, then MFMA pairs each followed by the next two reads
    __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    if constexpr (!BOUNDED) {
      float tmax = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, fmaxf(s0[r], s1[r]));
      tmax = fmaxf(tmax * sl2, __shfl_xor(tmax * sl2, 32, 64));
      const float m_new = fmaxf(m_run, tmax);
      const float alpha = exp2f(m_run - m_new);
      l_run *= alpha;
      m_run = m_new;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) o_acc[i][r] *= alpha;
    }
    // P^T = exp2(S*scale*log2e - m) -> bf16 B operands; O^T += V^T P^T
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      f32x16& sacc = kh ? s1 : s0;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = __builtin_amdgcn_exp2f(sacc[r] * sl2 - m_run);
        sacc[r] = e;
        l_run += e;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 pk;
#pragma unroll
        for (int j = 0; j < 8; ++j) pk[j] = (__bf16)sacc[8 * s + j];
        // k-step (kh, s): keys kh*32 + 16s + {8(j>>2) + 4hh + (j&3)}; V rows = that key set
        s16x4 lo[8], hi[8];
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
          lo[dt] = ds_tr16(Vb + (kh * 32 + 16 * s) * 512 + v_off[dt]);
          hi[dt] = ds_tr16(Vb + (kh * 32 + 16 * s + 8) * 512 + v_off[dt]);
        }
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
          const s16x8 c = __builtin_shufflevector(lo[dt], hi[dt], 0, 1, 2, 3, 4, 5, 6, 7);
          const bf16x8 vf = __builtin_bit_cast(bf16x8, c);
          o_acc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pk, o_acc[dt], 0, 0, 0);
        }
        // 16 transposed reads: 4 ahead, then one MFMA per two reads
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      }
    }
  };

  const int ntiles = (k_len + KT - 1) / KT;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < ntiles; t += 2) {
    if (t + 1 < ntiles) stage(t + 1, 1);
    compute(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + 1 >= ntiles) break;
    if (t + 2 < ntiles) stage(t + 2, 0);
    compute(1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // keys past the end were staged as zero rows: each contributed exp2(0*sl2 - m) to l and 0 to O
  l_run += __shfl_xor(l_run, 32, 64);  // the two lane halves hold the sums of complementary keys
  const int n_pad = ntiles * KT - k_len;
  l_run -= (float)n_pad * __builtin_amdgcn_exp2f(-m_run);
  if (q_row >= q_len) return;
  const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
  bf16_t* orow = p.o + (long)(q_start + q_row) * p.o_row_stride + (long)h * p.o_head_stride;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int r4 = 0; r4 < 4; ++r4) {
      const int d = i * 32 + 8 * r4 + 4 * hh;
      u32x2 w;
      w.x = pack2bf(o_acc[i][4 * r4 + 0] * inv, o_acc[i][4 * r4 + 1] * inv);
      w.y = pack2bf(o_acc[i][4 * r4 + 2] * inv, o_acc[i][4 * r4 + 3] * inv);
      *(u32x2*)(orow + d) = w;
    }
  }
}

bool attr_done = false;

}  // namespace

int attn_init() {
  if (attr_done) return 0;
  FLITE_HIP_CHECK(hipFuncSetAttribute((const void*)attn_fwd_hd256_kernel<true>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
  FLITE_HIP_CHECK(hipFuncSetAttribute((const void*)attn_fwd_hd256_kernel<false>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
  attr_done = true;
  return 0;
}

int attn_fwd(const AttnParams& p, hipStream_t stream) {
  FLITE_REQUIRE(p.head_dim == HD, "attention: only head_dim 256 is supported");
  FLITE_REQUIRE(p.B > 0 && p.H > 0 && p.max_q > 0, "attention: empty problem");
  FLITE_REQUIRE(p.q_row_stride % 8 == 0 && p.k_row_stride % 8 == 0 && p.v_row_stride % 8 == 0 &&
                    p.o_row_stride % 4 == 0,
                "attention: row strides must be multiples of 8 elements");
  FLITE_REQUIRE(p.q_head_stride % 8 == 0 && p.k_head_stride % 8 == 0 && p.v_head_stride % 8 == 0,
                "attention: head strides must be multiples of 8 elements");
  if (attn_init()) return 1;
  AttnParams q = p;
  q.n_qtiles = (p.max_q + QT - 1) / QT;
  dim3 grid(q.n_qtiles * p.H * p.B);
  if (p.max_score > 0.f)
    hipLaunchKernelGGL(attn_fwd_hd256_kernel<true>, grid, dim3(NT), LDS_BYTES, stream, q);
  else
    hipLaunchKernelGGL(attn_fwd_hd256_kernel<false>, grid, dim3(NT), LDS_BYTES, stream, q);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace flite
