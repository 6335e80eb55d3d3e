// Flash-attention forward for head_dim 256 on gfx950 (non-causal, varlen via cu_seqlens).
//
// Replaces flash_attn_interface.flash_attn_varlen_func (reference f_lite/model.py:203-210), used for the
// self-attention over the CFG-batched image tokens (cu_seqlens = [0, T, 2T, ...]) and the cross-attention
// onto the text context (cu_seqlens_k from the context mask, model.py:530).
//
// Workgroup = 4 waves (one per SIMD, up to 512 registers each) = 128 query rows of one (sequence, head);
// wave w owns 32 query rows and sweeps every 64-key tile (two 32-key S^T tiles).
// Per tile and wave:  S^T = K . Q^T  (v_mfma_f32_32x32x16_bf16, K fragments from LDS, Q^T in registers)
//   -> query index on the lane, keys in registers: the online-softmax max/sum are lane-local + 1 swap;
//   O^T += V^T . P^T  with P^T taken straight from the S^T accumulator registers (no LDS round trip) and
//   V^T fragments read with ds_read_b64_tr_b16 (hardware transpose) from a row-major, XOR-swizzled V tile.
// K/V tiles stream HBM->LDS with global_load_lds (swizzle on the source address), double-buffered.
#include "common.h"
#include "kernels.h"

namespace flite {

namespace {

constexpr int QT = 128;     // query rows per workgroup
constexpr int KT = 64;      // keys per tile
constexpr int HD = 256;     // head dim
constexpr int NT = 256;
constexpr int KV_TILE_BYTES = KT * HD * 2;          // 32 KiB
constexpr int STAGE_BYTES = 2 * KV_TILE_BYTES;      // K + V
constexpr int LDS_BYTES = 2 * STAGE_BYTES;          // double buffer

__device__ __forceinline__ void glds16(const void* gsrc, void* ldst) {
  __builtin_amdgcn_global_load_lds((const GLB_AS void*)gsrc, (LDS_AS void*)ldst, 16, 0, 0);
}

__device__ __forceinline__ s16x4 ds_tr16(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(p));
}

__global__ __launch_bounds__(NT, 1) void attn_fwd_hd256_kernel(AttnParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int g = wave;
  const int b = blockIdx.z;
  const int h = blockIdx.y;
  const int qt = blockIdx.x;

  const int q_start = p.cu_q[b];
  const int q_len = p.cu_q[b + 1] - q_start;
  if (qt * QT >= q_len) return;  // uniform over the workgroup
  const int k_start = p.cu_k[b];
  const int k_len = p.cu_k[b + 1] - k_start;

  const int lq = lane & 31;
  const int hh = lane >> 5;
  const int q_row = qt * QT + g * 32 + lq;  // this lane's query (within the sequence)

  if (k_len <= 0) {  // no keys: output zeros (rows owned by lanes of key-half 0)
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

  // ---- staging sources: 4 K + 4 V glds per wave per tile; instruction qi covers tile rows 2qi, 2qi+1 ----
  const bf16_t* kbase = p.k + (long)k_start * p.k_row_stride + (long)h * p.k_head_stride;
  const bf16_t* vbase = p.v + (long)k_start * p.v_row_stride + (long)h * p.v_head_stride;
  auto stage = [&](int t, int buf) {
    char* kb = smem + buf * STAGE_BYTES;
    char* vb = kb + KV_TILE_BYTES;
    const int pos = lane & 31;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int qi = wave * 8 + i;
      const int row = 2 * qi + hh;
      const int kc = pos ^ (row & 15);
      const int vc = (((pos >> 2) ^ (row & 3)) << 2) | (pos & 3);
      const long key = min(t * KT + row, k_len - 1);
      glds16(kbase + key * p.k_row_stride + kc * 8, kb + qi * 1024);
      glds16(vbase + key * p.v_row_stride + vc * 8, vb + qi * 1024);
    }
  };

  f32x16 o_acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o_acc[i][r] = 0.f;
  float m_run = -1e30f;
  float l_run = 0.f;
  const float sl2 = p.scale * 1.4426950408889634f;

  const int ntiles = (k_len + KT - 1) / KT;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // per-lane constant LDS offsets
  const int k_rd = lq * 512;                      // key row (within a 32-key half) for the A operand of S^T
  const int k_sw = lq & 15;                       // XOR swizzle of that row
  // V tr-read: group G = lane>>4, lane-in-group li = lane&15 -> q = li>>2 (row), pq = li&3 (4-col piece)
  const int G = lane >> 4;
  const int li = lane & 15;
  const int vq = li >> 2;
  const int vp = li & 3;

  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntiles) stage(t + 1, cur ^ 1);
    const char* Kb = smem + cur * STAGE_BYTES;
    const char* Vb = Kb + KV_TILE_BYTES;

    // S^T[key][q] for the two 32-key halves of the tile
    f32x16 s_acc[2];
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s_acc[kh][r] = 0.f;
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int chunk = 2 * s + hh;
        const bf16x8 kf = *(const bf16x8*)(Kb + kh * 32 * 512 + k_rd + ((chunk ^ k_sw) << 4));
        s_acc[kh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], s_acc[kh], 0, 0, 0);
      }
    }

    // online softmax (log2 domain); key of register r of half kh: kh*32 + (r&3) + 8*(r>>2) + 4*hh
    float tmax = -INFINITY;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = t * KT + kh * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        float v = s_acc[kh][r] * sl2;
        v = (key < k_len) ? v : -INFINITY;
        s_acc[kh][r] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float m_new = fmaxf(m_run, tmax);
    const float alpha = exp2f(m_run - m_new);
    float rsum = 0.f;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s_acc[kh][r] = exp2f(s_acc[kh][r] - m_new);
        rsum += s_acc[kh][r];
      }
    rsum += __shfl_xor(rsum, 32, 64);
    l_run = l_run * alpha + rsum;
    m_run = m_new;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) o_acc[i][r] *= alpha;

    // O^T[d][q] += V^T[d][key] . P^T[key][q]; k-step (kh, s) covers keys kh*32 + 16s + {8(j>>2) + 4hh + (j&3)}
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 pk;
#pragma unroll
        for (int j = 0; j < 8; ++j) pk[j] = (__bf16)s_acc[kh][8 * s + j];
        const int row1 = kh * 32 + 16 * s + 4 * (G >> 1) + vq;  // (row1 & 3) == vq
        const int row2 = row1 + 8;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
          const int col_blk = (dt ^ vq);                       // swizzled 32-col block
          const int cin = 16 * (G & 1) + 4 * vp;               // col within block
          const s16x4 lo = ds_tr16(Vb + row1 * 512 + (col_blk * 32 + cin) * 2);
          const s16x4 hi = ds_tr16(Vb + row2 * 512 + (col_blk * 32 + cin) * 2);
          bf16x8 vf;
          const __bf16* lp = (const __bf16*)&lo;
          const __bf16* hp = (const __bf16*)&hi;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            vf[j] = lp[j];
            vf[4 + j] = hp[j];
          }
          o_acc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pk, o_acc[dt], 0, 0, 0);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- normalise and store: lane holds O^T[d = i*32 + (r&3) + 8(r>>2) + 4hh][q] ----
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
  FLITE_HIP_CHECK(hipFuncSetAttribute((const void*)attn_fwd_hd256_kernel,
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
  dim3 grid((p.max_q + QT - 1) / QT, p.H, p.B);
  hipLaunchKernelGGL(attn_fwd_hd256_kernel, grid, dim3(NT), LDS_BYTES, stream, p);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace flite
