// Shared device/host helpers for the F-Lite MI355X (gfx950) kernels.
// All device code here is written for CDNA4 only: 64-lane waves, MFMA, LDS.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

namespace flite {

typedef uint16_t bf16_t;  // storage type for bf16 tensors (bit pattern)

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

#define LDS_AS __attribute__((address_space(3)))
#define GLB_AS __attribute__((address_space(1)))

__device__ __forceinline__ float bf2f(bf16_t h) {
  return __uint_as_float(((unsigned)h) << 16);
}
// round-to-nearest-even (matches torch's float->bfloat16 cast for finite values)
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 h = (__bf16)f;
  return *reinterpret_cast<bf16_t*>(&h);
}
__device__ __forceinline__ unsigned pack2bf(float lo, float hi) {
  return (unsigned)f2bf(lo) | ((unsigned)f2bf(hi) << 16);
}
// Wide epilogue stores of the GEMMs (gemm.hip, gemm_fp8.hip). For one output row, a 16-column group of a wave is
// held as 4 columns by each of the lanes lr + 16 lk (lk = 0..3), so one store instruction would write 16 rows of
// 4-column pieces; every tile of a round stores at the same time, with the MFMA pipes idle. Two such groups a
// (columns [c, c+16)) and b ([c+16, c+32)), one dword per 2 (bf16) or 4 (e4m3) columns, are re-dealt by one
// v_permlane16_swap per dword (odd 16-lane rows of `a` <-> even rows of `b`) so that lane lk holds the 8
// consecutive columns c + deal8_col(lk) + 0..7: half the store instructions, each twice as wide. Every lane must
// be active (the partner lanes lr + 16 lk share the row, so callers mask only the store).
__device__ __forceinline__ u32x4 deal8(const u32x2& a, const u32x2& b) {
  const auto x = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
  const auto y = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
  return u32x4{x[0], y[0], x[1], y[1]};
}
__device__ __forceinline__ u32x2 deal8(unsigned a, unsigned b) {
  const auto x = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  return u32x2{x[0], x[1]};
}
__device__ __forceinline__ int deal8_col(int lk) { return 8 * (lk >> 1) + 16 * (lk & 1); }

// x * sigmoid(x) with v_exp_f32 and v_rcp_f32 (1 ulp) instead of an IEEE division (~10 VALU per element in
// the SwiGLU GEMM epilogue). Limits: x -> -inf gives -0, x -> +inf gives x.
__device__ __forceinline__ float silu_f(float x) {
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}

// GELU, tanh approximation (transformers' "gelu_new", the T5 v1.1 gated FF): 0.5 x (1 + tanh(u)),
// u = sqrt(2/pi) (x + 0.044715 x^3), with tanh(u) = 1 - 2 / (1 + e^{2u}).
__device__ __forceinline__ float gelu_tanh_f(float x) {
  const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
  const float t = 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(2.8853900817779268f * u));
  return 0.5f * x * (1.0f + t);
}

// Column order of the RoPE heads (q, k) written by the fused qkv GEMM epilogues: output position j of a 256-wide
// head holds original column j/2 (j even) or 128 + j/2 (j odd), so each rotation pair (c, c + 128) of
// apply_rotary_emb lands in two adjacent columns of one lane. q and k share it, so q.k is unchanged.
__host__ __device__ __forceinline__ int rope_perm(int n) {
  const int j = n & 255;
  return (n & ~255) | (j >> 1) | ((j & 1) << 7);
}

// Factorised 2-D RoPE table read by the fused qkv GEMM epilogues (rope_axes_table, elementwise.hip). TwoDimRotary
// (model.py:334-386) gives token t = reg + y*w + x the angles cat(y * inv_freq, x * inv_freq) (64 each) and the
// registers angle 0, so the [T][128] cos / sin tables of rope_table hold only 1 + h + w distinct 64-angle rows:
// row 0 = registers (cos 1, sin 0), row 1 + y = the y axis, row 1 + h + x = the x axis, each [64][2] fp32 with cos
// and sin interleaved. Same values in (1 + h + w) rows instead of T: 72 KB at 1344x896, L2-resident.
struct RopeAxes {
  const float* cs = nullptr;  // [1 + h + w][64][2]
  int tokens = 0;             // rows per sequence in the launch: row m is local token m % tokens
  int tok0 = 0;               // global token of local token 0 (sequence parallelism: rank * tokens)
  int reg = 0, h = 0, w = 0;
  float inv_w = 0.f;          // 1 / w

  // table row of global token g for angles [0, 64) (axis_mask 0) or [64, 128) (axis_mask -1); tokens past the sequence
  // (padding rows of the last sequence-parallel rank) clamp to its last row
  // (branch-free: a select here had become per-block control flow that kept every block's loads in flight)
  __device__ __forceinline__ int row(int g, int axis_mask) const {
    const int q = max(g - reg, 0);
    int y = (int)((float)q * inv_w);
    int x = q - y * w;
    const int lo = x >> 31;  // x < 0: one row too far
    y += lo;
    x += lo & w;
    const int hi = (w - 1 - x) >> 31;  // x >= w: one row short
    y -= hi;
    x -= hi & w;
    y = min(y, h - 1);
    const int r = 1 + ((y & ~axis_mask) | ((h + x) & axis_mask));
    return r & ((reg - 1 - g) >> 31);  // registers (g < reg): row 0
  }
};

// RoPE (apply_rotary_emb, model.py:403-414: y1 = x1 c + x2 s, y2 = -x1 s + x2 c) of one wave's GEMM accumulators
// in the gemm.hip / gemm_fp8.hip layout: the lane holds C[m][n .. n+3], m = m_base + mi*16, n = n0 + wave_n*64 +
// lk*4 + ni*16, columns in rope_perm order, so (r 0, 1) and (r 2, 3) are rotation pairs with angles i0 and i0 + 1,
// i0 = wave_n*32 + lk*2 + ni*8: waves 0-1 take the y axis, 2-3 the x axis. The table is small enough to stay
// L2-resident. Rows >= M rotate garbage and are never stored.
template <int MI>
__device__ __forceinline__ void rope_rotate(f32x4 (&acc)[8][4], const RopeAxes& ra, int m_base, int M, int wave_n,
                                            int lk) {
  const int axis_mask = wave_n >= 2 ? -1 : 0;
  const float* base = ra.cs + ((wave_n & 1) * 32 + lk * 2) * 2;
  const int T = ra.tokens;
  const int step = 16 % T;  // next block's token (sequences may be shorter than 16 rows)
  int tok = min(m_base, M - 1) % T;
  auto fetch = [&](int t, f32x4(&d)[4]) {
    const float* b = base + (long)ra.row(ra.tok0 + t, axis_mask) * 128;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) d[ni] = *(const f32x4*)(b + ni * 16);
  };
  f32x4 cur[4], nxt[4];
  fetch(tok, cur);
#pragma unroll
  for (int mi = 0; mi < MI; ++mi) {
    if (mi + 1 < MI) {
      tok += step;
      if (tok >= T) tok -= T;
      fetch(tok, nxt);
    }
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const float c = cur[ni][2 * pr], sn = cur[ni][2 * pr + 1];
        const float x1 = acc[mi][ni][2 * pr], x2 = acc[mi][ni][2 * pr + 1];
        acc[mi][ni][2 * pr] = x1 * c + x2 * sn;
        acc[mi][ni][2 * pr + 1] = -x1 * sn + x2 * c;
      }
    __builtin_amdgcn_sched_barrier(0);  // at most two 16-row blocks' table loads in flight (registers)
    if (mi + 1 < MI) {
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) cur[ni] = nxt[ni];
    }
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Host-side error plumbing (thread-local last error, never throws across the C ABI)
void set_last_error(const std::string& msg);
const char* get_last_error();

}  // namespace flite

#define FLITE_HIP_CHECK(expr)                                                         \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess) {                                                           \
      ::flite::set_last_error(std::string(#expr) + ": " + hipGetErrorString(_e));     \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

#define FLITE_REQUIRE(cond, msg)                                                      \
  do {                                                                                \
    if (!(cond)) {                                                                    \
      ::flite::set_last_error(std::string("flite: ") + (msg));                        \
      return 2;                                                                       \
    }                                                                                 \
  } while (0)

// roctx ranges (rocprofv3 --marker-trace): host-side markers per denoise step / DiT block / VAE decode, so kernel
// traces split by phase. Near-free without a tool attached; inside a hipGraph capture they mark the capture.
#include <rocprofiler-sdk-roctx/roctx.h>
namespace flite {
struct RoctxRange {
  explicit RoctxRange(const char* name) { roctxRangePushA(name); }
  ~RoctxRange() { roctxRangePop(); }
  RoctxRange(const RoctxRange&) = delete;
  RoctxRange& operator=(const RoctxRange&) = delete;
};
}  // namespace flite
