// MXFP8 quantisation for the fp8 DiT path (BASELINE.json configs[4]: fp8 weights + activations on the
// gfx950 block-scaled MFMA, v_mfma_scale_f32_16x16x128_f8f6f4).
//
// Format (OCP MX): elements OCP e4m3fn (gfx950 is OCP, not the MI300 fnuz variant), one E8M0 scale per 32
// consecutive elements along K. Scale exponent e = ceil(log2(amax / 448)) so the largest element of a block
// maps into (224, 448]; element = RNE(clamp(x * 2^-e, +-448)). The oracle restates the same arithmetic
// (oracle/flite_ref.py: mx_quant) bit for bit.
//
// Scale layout, shared by weights and activations ("k-tile major"): S[K/128][rows_pad][4] bytes, i.e. one 32-bit
// word per (128-deep k-tile, row) holding the row's 4 block scales of that k-tile, so the GEMM stages a k-tile's
// scales for 256 rows with ONE 1-KiB LDS-DMA piece.
#include "common.h"
#include "fp8.h"

namespace flite {

namespace {

// 32 consecutive elements of one row per thread: 4 x 16-B loads, 2 x 16-B stores, one scale byte.
// INTERLEAVE (SwiGLU gate/up weights): destination row v is row (v >> 5) * 16 + (v & 15) of src (16-row sub-tile
// v >> 4 even) or src2 (odd) -- the gate|up sub-tile order the GEMM's SwiGLU epilogue pairs up.
// PERM (fused qkv epilogue): destination row v < perm_rows is source row rope_perm(v).
template <bool INTERLEAVE, bool PERM = false>
__global__ __launch_bounds__(256) void quant_rows_kernel(const bf16_t* src, const bf16_t* src2, long lds, long rows,
                                                         int K, uint8_t* dst, long ldd, uint8_t* sc, long rows_pad,
                                                         long perm_rows = 0) {
  const long nblk = (long)K / 32;
  const long total = rows * nblk;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long v = i / nblk;
    const int b = (int)(i - v * nblk);
    const bf16_t* s = src;
    long r = v;
    if constexpr (INTERLEAVE) {
      s = ((v >> 4) & 1) ? src2 : src;
      r = (v >> 5) * 16 + (v & 15);
    }
    if constexpr (PERM) {
      if (v < perm_rows) r = rope_perm((int)v);
    }
    const u32x4* p = (const u32x4*)(s + r * lds + b * 32);
    float x[32];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const u32x4 w = p[q];
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
    const float inv = mx_inv(e);
    u32x4 o[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      unsigned ow[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) ow[j] = pack4_fp8(x + 16 * h + 4 * j, inv);
      o[h] = u32x4{ow[0], ow[1], ow[2], ow[3]};
    }
    u32x4* d = (u32x4*)(dst + v * ldd + b * 32);
    d[0] = o[0];
    d[1] = o[1];
    sc[((long)(b >> 2) * rows_pad + v) * 4 + (b & 3)] = (uint8_t)(e + 127);
  }
}

int grid_for(long total) {
  long g = (total + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}

}  // namespace

int quant_rows_fp8(const bf16_t* src, long ld_src, long rows, int K, uint8_t* dst, long ld_dst, uint8_t* scales,
                   long rows_pad, hipStream_t s) {
  FLITE_REQUIRE(K % 128 == 0, "quant_fp8: K must be a multiple of 128");
  FLITE_REQUIRE(ld_src % 8 == 0 && ld_dst % 16 == 0, "quant_fp8: row strides must keep 16-B alignment");
  FLITE_REQUIRE(rows_pad >= rows, "quant_fp8: rows_pad < rows");
  hipLaunchKernelGGL(quant_rows_kernel<false>, dim3(grid_for(rows * (K / 32))), dim3(256), 0, s, src, src, ld_src,
                     rows, K, dst, ld_dst, scales, rows_pad);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int quant_rows_fp8_perm(const bf16_t* src, long ld_src, long rows, int K, uint8_t* dst, long ld_dst, uint8_t* scales,
                        long rows_pad, long perm_rows, hipStream_t s) {
  FLITE_REQUIRE(K % 128 == 0, "quant_fp8: K must be a multiple of 128");
  FLITE_REQUIRE(ld_src % 8 == 0 && ld_dst % 16 == 0, "quant_fp8: row strides must keep 16-B alignment");
  FLITE_REQUIRE(rows_pad >= rows && perm_rows % 256 == 0 && perm_rows <= rows, "quant_fp8_perm: bad row counts");
  hipLaunchKernelGGL((quant_rows_kernel<false, true>), dim3(grid_for(rows * (K / 32))), dim3(256), 0, s, src, src,
                     ld_src, rows, K, dst, ld_dst, scales, rows_pad, perm_rows);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int quant_gateup_fp8(const bf16_t* gate, const bf16_t* up, long ld_src, int F, int K, uint8_t* dst, uint8_t* scales,
                     hipStream_t s) {
  FLITE_REQUIRE(K % 128 == 0 && F % 16 == 0, "quant_gateup_fp8: K % 128, F % 16");
  const long rows = 2L * F;
  hipLaunchKernelGGL(quant_rows_kernel<true>, dim3(grid_for(rows * (K / 32))), dim3(256), 0, s, gate, up, ld_src,
                     rows, K, dst, (long)K, scales, rows);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace flite
