// T5 v1.1 encoder kernels for gfx950: the text-encoder step of the F-Lite pipeline.
//
// The reference encodes each prompt once (f_lite/pipeline.py:126-175: hidden_states[-8] of the text encoder;
// the 7B / 10B DiTs take cross_attn_input_size = 4096 = T5-XXL's d_model, train.py:685-698, pt.py:150-155).
// The T5 encoder layer (transformers T5EncoderModel, the reference's dependency) is RMSNorm -> self-attention
// with a bucketed relative-position bias and no 1/sqrt(d) scaling -> residual, RMSNorm -> gated-GELU FF ->
// residual. Its GEMMs run on the DiT GEMM (gemm.hip; the GEGLU epilogue there), its norms on rmsnorm_mod; this
// file holds what is T5-specific:
//   * t5_attention: softmax(q k^T + bias[h][j - i] + mask[b][j]) v for head_dim 64 and L <= 512 keys. One
//     workgroup = (sequence, head, 64 queries), 4 waves x 16 queries. The head's K ([L][64], row-major) and V^T
//     ([64][L]) are staged whole in LDS (<= 138 KiB), so the softmax is exact (full score rows in registers:
//     128 per lane at L = 512) rather than online. S^T = K Q^T and O^T = V^T P^T on v_mfma_f32_16x16x32_bf16;
//     P^T comes straight from the S^T accumulators (the key order inside a 32-key step is permuted the same
//     way on the V^T side).
//   * embed_rows_f32: token-embedding gather into the fp32 residual stream.
#include <algorithm>

#include "common.h"
#include "t5.h"

namespace flite {

namespace {

constexpr int T5_HD = 64;
constexpr int T5_MAXL = 512;
constexpr int T5_NT = 256;
constexpr int K_STRIDE = T5_HD + 8;  // bf16 elements per K row in LDS (144 B: rows spread over the banks)

__global__ __launch_bounds__(T5_NT, 1) void t5_attention_kernel(T5AttnParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Lp = (p.L + 31) & ~31;      // keys padded to the 32-key PV step
  const int vt_stride = Lp + 8;         // bf16 elements per V^T row
  bf16_t* k_lds = (bf16_t*)smem;                                    // [Lp][K_STRIDE]
  bf16_t* vt_lds = k_lds + (size_t)Lp * K_STRIDE;                   // [64][vt_stride]
  float* tab = (float*)(vt_lds + (size_t)T5_HD * vt_stride);        // [2L - 1] bias by (key - query + L - 1)
  float* msk = tab + 2 * T5_MAXL;                                   // [Lp] additive key mask

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int qblocks = (p.L + 63) / 64;
  const int qb = blockIdx.x % qblocks;
  const int h = (blockIdx.x / qblocks) % p.H;
  const int b = blockIdx.x / (qblocks * p.H);
  const long row0 = (long)b * p.L;

  // ---- stage K rows, V^T, the bias row of head h and the key mask
  for (int e = tid; e < Lp * 8; e += T5_NT) {  // 8 chunks of 8 bf16 per key
    const int key = e >> 3, c = e & 7;
    u32x4 kv = {0u, 0u, 0u, 0u}, vv = {0u, 0u, 0u, 0u};
    if (key < p.L) {
      kv = *(const u32x4*)(p.k + (row0 + key) * p.ldk + (long)h * T5_HD + c * 8);
      vv = *(const u32x4*)(p.v + (row0 + key) * p.ldv + (long)h * T5_HD + c * 8);
    }
    *(u32x4*)(k_lds + key * K_STRIDE + c * 8) = kv;
    const bf16_t* vs = (const bf16_t*)&vv;
#pragma unroll
    for (int j = 0; j < 8; ++j) vt_lds[(c * 8 + j) * vt_stride + key] = vs[j];
  }
  for (int r = tid; r < 2 * p.L - 1; r += T5_NT) tab[r] = bf2f(p.rel_weight[(long)p.bucket[r] * p.H + h]);
  for (int j = tid; j < Lp; j += T5_NT)
    msk[j] = j >= p.L ? -INFINITY : (p.mask != nullptr ? p.mask[row0 + j] : 0.f);
  __syncthreads();

  // ---- S^T = K Q^T: lane holds keys 16 blk + 4 (lane >> 4) + r of query q0 + (lane & 15)
  const int lr = lane & 15, lg = lane >> 4;
  const int q = qb * 64 + wave * 16 + lr;
  const int qc = std::min(q, p.L - 1);
  bf16x8 qf[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
    qf[ks] = *(const bf16x8*)(p.q + (row0 + qc) * p.ldq + (long)h * T5_HD + ks * 32 + lg * 8);
  const int nblk = Lp / 16;
  f32x4 s[T5_MAXL / 16];
#pragma unroll
  for (int blk = 0; blk < T5_MAXL / 16; ++blk) {
    if (blk < nblk) {
      s[blk] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 kf = *(const bf16x8*)(k_lds + (blk * 16 + lr) * K_STRIDE + ks * 32 + lg * 8);
        s[blk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[ks], s[blk], 0, 0, 0);
      }
    }
  }
  // ---- + bias + mask, exact softmax over the full row
  float mx = -INFINITY;
#pragma unroll
  for (int blk = 0; blk < T5_MAXL / 16; ++blk) {
    if (blk < nblk) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = blk * 16 + lg * 4 + r;
        const float v = s[blk][r] + tab[std::min(key, p.L - 1) - qc + p.L - 1] + msk[key];
        s[blk][r] = v;
        mx = fmaxf(mx, v);
      }
    }
  }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  const float msub = mx == -INFINITY ? 0.f : mx;  // a fully masked row gives p = 0 and a zero output
  float sum = 0.f;
#pragma unroll
  for (int blk = 0; blk < T5_MAXL / 16; ++blk) {
    if (blk < nblk) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = __expf(s[blk][r] - msub);
        s[blk][r] = e;
        sum += e;
      }
    }
  }
  sum += __shfl_xor(sum, 16, 64);
  sum += __shfl_xor(sum, 32, 64);

  // ---- O^T = V^T P^T. k-index 8 g + j of 32-key step ks <-> key 32 ks + (j < 4 ? 4 g + j : 16 + 4 g + j - 4)
  f32x4 o[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < T5_MAXL / 32; ++ks) {
    if (ks < Lp / 32) {
      bf16x8 pk;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pk[r] = (__bf16)s[2 * ks][r];
        pk[4 + r] = (__bf16)s[2 * ks + 1][r];
      }
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const bf16_t* vrow = vt_lds + (d * 16 + lr) * vt_stride + ks * 32 + lg * 4;
        const u32x2 lo = *(const u32x2*)vrow;
        const u32x2 hi = *(const u32x2*)(vrow + 16);
        const u32x4 vv = {lo.x, lo.y, hi.x, hi.y};
        o[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, vv), pk, o[d], 0, 0, 0);
      }
    }
  }
  if (q >= p.L) return;
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
  bf16_t* orow = p.o + (row0 + q) * p.ldo + (long)h * T5_HD;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    u32x2 w;
    w.x = pack2bf(o[d][0] * inv, o[d][1] * inv);
    w.y = pack2bf(o[d][2] * inv, o[d][3] * inv);
    *(u32x2*)(orow + d * 16 + lg * 4) = w;
  }
}

__global__ void embed_rows_f32_kernel(const bf16_t* table, const int* ids, float* out, long n, int cols, long vocab) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;  // one thread per 4 columns
  const int per_row = cols / 4;
  if (i >= n * per_row) return;
  const long r = i / per_row;
  const int c = (int)(i - r * per_row) * 4;
  const long id = std::min(std::max((long)ids[r], 0L), vocab - 1);
  const u32x2 v = *(const u32x2*)(table + id * cols + c);
  f32x4 f = {__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u), __uint_as_float(v.y << 16),
             __uint_as_float(v.y & 0xffff0000u)};
  *(f32x4*)(out + r * cols + c) = f;
}

bool t5_attr_done = false;

size_t t5_lds_bytes(int L) {
  const int Lp = (L + 31) & ~31;
  return (size_t)Lp * K_STRIDE * 2 + (size_t)T5_HD * (Lp + 8) * 2 + (2 * T5_MAXL + Lp) * 4;
}

}  // namespace

int t5_attention(const T5AttnParams& p, hipStream_t s) {
  FLITE_REQUIRE(p.B > 0 && p.H > 0 && p.L > 0, "t5_attention: empty problem");
  FLITE_REQUIRE(p.L <= T5_MAXL, "t5_attention: at most 512 tokens (max_sequence_length)");
  FLITE_REQUIRE(p.ldq % 8 == 0 && p.ldk % 8 == 0 && p.ldv % 8 == 0 && p.ldo % 4 == 0,
                "t5_attention: row strides must be multiples of 8 elements");
  FLITE_REQUIRE(p.q && p.k && p.v && p.o && p.bucket && p.rel_weight, "t5_attention: null operand");
  if (!t5_attr_done) {
    FLITE_HIP_CHECK(hipFuncSetAttribute((const void*)t5_attention_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)t5_lds_bytes(T5_MAXL)));
    t5_attr_done = true;
  }
  const int qblocks = (p.L + 63) / 64;
  hipLaunchKernelGGL(t5_attention_kernel, dim3(p.B * p.H * qblocks), dim3(T5_NT), t5_lds_bytes(p.L), s, p);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int embed_rows_f32(const bf16_t* table, const int* ids, float* out, long n, int cols, long vocab, hipStream_t s) {
  FLITE_REQUIRE(cols % 4 == 0 && n >= 0 && vocab > 0, "embed_rows_f32: cols must be a multiple of 4");
  if (n == 0) return 0;
  const long threads = n * (cols / 4);
  hipLaunchKernelGGL(embed_rows_f32_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, table, ids, out,
                     n, cols, vocab);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace flite
