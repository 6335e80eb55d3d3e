// MXFP8 helpers and the fp8 GEMM interface (gfx950). See fp8.hip for the format and the scale layout.
#pragma once
#include "common.h"

namespace flite {

// E8M0 exponent of a block with absolute maximum `amax`: ceil(log2(amax / 448)) in [-127, 126]
// (amax * (1/448) is one fp32 multiply, RNE; the oracle does the same multiply).
__device__ __forceinline__ int mx_exp(float amax) {
  const unsigned b = __float_as_uint(amax * (1.0f / 448.0f));
  const int e = (int)((b >> 23) & 0xff) - 127 + ((b & 0x7fffffu) ? 1 : 0);
  return e < -127 ? -127 : (e > 126 ? 126 : e);
}
// 2^-e (exact; e in [-127, 126])
__device__ __forceinline__ float mx_inv(int e) { return __uint_as_float((unsigned)(127 - e) << 23); }

// 4 floats * inv -> 4 OCP e4m3fn bytes (RNE), saturated to +-448 first
__device__ __forceinline__ unsigned pack4_fp8(const float* x, float inv) {
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = fminf(fmaxf(x[j] * inv, -448.f), 448.f);
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], w, true);
  return (unsigned)w;
}

// fp8 GEMM: C[M,N] = dequant(A8)[M,K] . dequant(W8)[N,K]^T with MX block scales; fp32 accumulate.
//   A8 / W8: e4m3 bytes, row stride lda / ldw bytes; As / Ws: scales [K/128][a_rows_pad / w_rows_pad][4].
enum GemmFp8Epilogue {
  EPI8_STORE_BF16 = 0,  // out_bf16[m][n] = acc + bias[n]
  EPI8_RESID_F32 = 2,   // out_f32[m][n] += gate[seg(m)][n] * (acc + bias[n])
  EPI8_RESID_BF16 = 7,  // the same on a bf16 residual stream: fp32 math, one rounding (gemm.hip EPI_RESID_BF16)
  EPI8_SWIGLU_FP8 = 4,  // W8 = gate|up interleaved in 16-row sub-tiles (N = 2F): out8[m][f] = MX(silu(g) * u),
                        // scales to out_sc [F/128][out_rows_pad][4]
  EPI8_QKV_NORM_BF16 = 5,  // engine-internal: bf16 store with RoPE + QK-norm of columns [0, norm_cols) (gemm.hip)
  EPI8_SWIGLU_BF16 = 6,    // as EPI8_SWIGLU_FP8, out_bf16[m][f] = silu(g) * u (an fp8 gate/up feeding a bf16 down)
};

struct GemmFp8Params {
  const uint8_t* A = nullptr;
  long lda = 0;
  const uint8_t* As = nullptr;
  long a_rows_pad = 0;
  const uint8_t* W = nullptr;
  long ldw = 0;
  const uint8_t* Ws = nullptr;
  long w_rows_pad = 0;
  const bf16_t* bias = nullptr;
  void* out = nullptr;  // bf16 / fp32 / fp8 bytes (row stride ldo elements; bytes for fp8)
  long ldo = 0;
  uint8_t* out_sc = nullptr;
  long out_rows_pad = 0;
  const float* gate = nullptr;
  long gate_seg_stride = 0;
  int rows_per_seg = 1;
  int M = 0, N = 0, K = 0;
  // EPI8_QKV_NORM_BF16 (as gemm.hip's EPI_QKV_NORM_BF16): factorised RoPE table (common.h RopeAxes); columns
  // [0, rope_cols) are q/k heads whose W rows were quantised in rope_perm order (quant_rows_fp8_perm)
  RopeAxes rope;
  int rope_cols = 0, norm_cols = 0;
  float norm_eps = 1e-6f;
  // stream-K workspace (optional, gemm.hip layout: fp32 partial tiles [CUs][256*256] + int flags [CUs], zeroed):
  // the launcher may cut a partial last wave of 256x256 tiles into equal k-ranges (stream_k.h)
  float* sk_ws = nullptr;
  int* sk_flags = nullptr;
  int sk_tiles = 0;  // set by the launcher
  int sk_wgs = 0;    // set by the launcher
  int resid_narrow = 0;  // set by the launcher: EPI8_RESID_BF16 with 8-B lanes (FLITE_GEMM_RESID_NARROW, A/B switch)
};

int gemm_fp8(const GemmFp8Params& p, int epi, hipStream_t s);
int quant_rows_fp8(const bf16_t* src, long ld_src, long rows, int K, uint8_t* dst, long ld_dst, uint8_t* scales,
                   long rows_pad, hipStream_t s);
// quant_rows_fp8 with destination row v < perm_rows taken from source row rope_perm(v) (the fused fp8 qkv epilogue)
int quant_rows_fp8_perm(const bf16_t* src, long ld_src, long rows, int K, uint8_t* dst, long ld_dst, uint8_t* scales,
                        long rows_pad, long perm_rows, hipStream_t s);
int quant_gateup_fp8(const bf16_t* gate, const bf16_t* up, long ld_src, int F, int K, uint8_t* dst, uint8_t* scales,
                     hipStream_t s);

// rows rounded up for the scale arrays (the GEMM stages scales for 256-row tiles)
inline long mx_rows_pad(long rows) { return (rows + 255) / 256 * 256; }

}  // namespace flite
