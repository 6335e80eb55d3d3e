// Bandwidth-bound kernels of the Flux VAE decoder (diffusers AutoencoderKL.decode, called at
// reference pipeline.py:307). Activations are NHWC bf16 (one image); the 3x3 convolutions and the
// mid-block attention matmuls run on the MFMA GEMM (gemm.hip, implicit-GEMM conv mode).
#include <math.h>

#include <algorithm>

#include "common.h"
#include "fp8.h"
#include "kernels.h"

namespace flite {

namespace {

// GroupNorm statistics, pass 1: per-workgroup sum / sum of squares per group into partial[block][G][2], NHWC
// rows of C channels. Each thread reads 8 channels (16 B); groups hold C/G channels (4, 8 or 16). Every sum
// runs in a fixed order (no atomics), so the decode is bit-reproducible.
__global__ __launch_bounds__(256) void gn_stats_kernel(const bf16_t* x, long rows, int C, int G, float* partial) {
  __shared__ float ps[256][4];
  const int cg = C / G;  // channels per group
  const int vec_per_row = C / 8;
  const long total = rows * vec_per_row;
  float ls[2] = {0.f, 0.f}, lq[2] = {0.f, 0.f};
  int g0 = -1;
  // a thread's vector index v keeps the same channel offset when the stride is a multiple of vec_per_row
  const long stride = (long)gridDim.x * blockDim.x;
  const long v0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int c0 = (int)(v0 % vec_per_row) * 8;
  g0 = c0 / cg;
  for (long v = v0; v < total; v += stride) {
    const u32x4 w = *(const u32x4*)(x + v * 8);
    float f[8];
    f[0] = __uint_as_float(w.x << 16);
    f[1] = __uint_as_float(w.x & 0xffff0000u);
    f[2] = __uint_as_float(w.y << 16);
    f[3] = __uint_as_float(w.y & 0xffff0000u);
    f[4] = __uint_as_float(w.z << 16);
    f[5] = __uint_as_float(w.z & 0xffff0000u);
    f[6] = __uint_as_float(w.w << 16);
    f[7] = __uint_as_float(w.w & 0xffff0000u);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int gi = (cg >= 8) ? 0 : (j / cg);  // cg == 4 -> two groups per vector
      ls[gi] += f[j];
      lq[gi] += f[j] * f[j];
    }
  }
  (void)g0;
  ps[threadIdx.x][0] = ls[0];
  ps[threadIdx.x][1] = lq[0];
  ps[threadIdx.x][2] = ls[1];
  ps[threadIdx.x][3] = lq[1];
  __syncthreads();
  // thread u's vectors sit at channel (u % vec_per_row) * 8 (the grid stride is a multiple of vec_per_row)
  if ((int)threadIdx.x < G) {
    const int g = threadIdx.x;
    float s = 0.f, q = 0.f;
    for (int u = 0; u < 256; ++u) {
      const int gu = (u % vec_per_row) * 8 / cg;
      if (gu == g) {
        s += ps[u][0];
        q += ps[u][1];
      } else if (cg < 8 && gu + 1 == g) {
        s += ps[u][2];
        q += ps[u][3];
      }
    }
    partial[((long)blockIdx.x * G + g) * 2] = s;
    partial[((long)blockIdx.x * G + g) * 2 + 1] = q;
  }
}

// GroupNorm statistics, pass 2: stats[g] = (sum, sum of squares) over the workgroups' partials. 16 lanes per
// group (threads g*16 .. g*16+15, inside one wave) each sum the blocks b = lane (mod 16) in block order, then a
// fixed xor-shuffle tree adds the 16 lane sums: the order is fixed, so the result is bit-reproducible. (One
// thread per group walking all 1024 partials serially was latency-bound at ~250 us per launch.)
constexpr int GN_FIN_LANES = 16;
// It then turns the sums into the group's mean and rstd (stats[2g], stats[2g+1]), once per group instead of once
// per element in the apply pass; the expressions are unchanged, so the normalised output is too.
__global__ __launch_bounds__(1024) void gn_finalize_kernel(const float* partial, int nblocks, int G, double n,
                                                           float eps, double* stats) {
  const int g = threadIdx.x / GN_FIN_LANES;
  const int lane = threadIdx.x % GN_FIN_LANES;
  double s = 0.0, q = 0.0;
  if (g < G) {
#pragma unroll 4
    for (int b = lane; b < nblocks; b += GN_FIN_LANES) {
      const float2 p = *(const float2*)(partial + ((long)b * G + g) * 2);
      s += (double)p.x;
      q += (double)p.y;
    }
  }
#pragma unroll
  for (int off = GN_FIN_LANES / 2; off > 0; off >>= 1) {
    s += __shfl_xor(s, off, GN_FIN_LANES);
    q += __shfl_xor(q, off, GN_FIN_LANES);
  }
  if (g < G && lane == 0) {
    const double mean = s / n;
    const double var = fmax(q / n - mean * mean, 0.0);
    stats[2 * g] = mean;
    stats[2 * g + 1] = (double)(float)(1.0 / sqrt(var + (double)eps));
  }
}

template <bool SILU>
__global__ __launch_bounds__(256) void gn_apply_kernel(const bf16_t* x, bf16_t* y, long rows, int C, int G,
                                                       const double* stats, const bf16_t* gamma,
                                                       const bf16_t* beta) {
  const int cg = C / G;
  const int vec_per_row = C / 8;
  const long total = rows * vec_per_row;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long v = (long)blockIdx.x * blockDim.x + threadIdx.x; v < total; v += stride) {
    const int c0 = (int)(v % vec_per_row) * 8;
    const u32x4 w = *(const u32x4*)(x + v * 8);
    const u32x4 gw = *(const u32x4*)(gamma + c0);
    const u32x4 bw = *(const u32x4*)(beta + c0);
    const unsigned xs[4] = {w.x, w.y, w.z, w.w}, gs[4] = {gw.x, gw.y, gw.z, gw.w}, bs[4] = {bw.x, bw.y, bw.z, bw.w};
    unsigned outw[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float o[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = c0 + 2 * q + h;
        const int g = c / cg;
        const double mean = stats[2 * g];
        const float rstd = (float)stats[2 * g + 1];
        const float xv = __uint_as_float(h ? (xs[q] & 0xffff0000u) : (xs[q] << 16));
        const float gv = __uint_as_float(h ? (gs[q] & 0xffff0000u) : (gs[q] << 16));
        const float bv = __uint_as_float(h ? (bs[q] & 0xffff0000u) : (bs[q] << 16));
        float t = (xv - (float)mean) * rstd * gv + bv;
        if (SILU) t = silu_f(t);
        o[h] = t;
      }
      outw[q] = pack2bf(o[0], o[1]);
    }
    *(u32x4*)(y + v * 8) = u32x4{outw[0], outw[1], outw[2], outw[3]};
  }
}

// row softmax: P[r][:L] = softmax(scale * S[r][:L]) (fp32 in, bf16 out), P[r][L:ld] = 0 (the zero padding of
// the P.V GEMM's k dimension); rows of ld (a multiple of 4) elements, one workgroup per row
__global__ __launch_bounds__(256) void softmax_rows_kernel(const float* S, bf16_t* P, int L, int ld, float scale) {
  __shared__ float red[8];
  const float* s = S + (long)blockIdx.x * ld;
  bf16_t* pr = P + (long)blockIdx.x * ld;
  float m = -INFINITY;
  for (int i = threadIdx.x * 4; i < ld; i += 1024) {
    const f32x4 v = *(const f32x4*)(s + i);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (i + j < L) m = fmaxf(m, v[j]);
  }
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])) * scale;
  __syncthreads();
  float sum = 0.f;
  for (int i = threadIdx.x * 4; i < ld; i += 1024) {
    const f32x4 v = *(const f32x4*)(s + i);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (i + j < L) sum += __expf(v[j] * scale - m);
  }
  sum = wave_sum(sum);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sum;
  __syncthreads();
  const float inv = 1.f / (red[0] + red[1] + red[2] + red[3]);
  for (int i = threadIdx.x * 4; i < ld; i += 1024) {
    const f32x4 v = *(const f32x4*)(s + i);
    float e[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) e[j] = i + j < L ? __expf(v[j] * scale - m) * inv : 0.f;
    u32x2 w;
    w.x = pack2bf(e[0], e[1]);
    w.y = pack2bf(e[2], e[3]);
    *(u32x2*)(pr + i) = w;
  }
}

// bf16 transpose [R, C] -> [C, ldy] (columns R..ldy-1 untouched) through a 64x64 LDS tile
__global__ __launch_bounds__(256) void transpose_kernel(const bf16_t* x, bf16_t* y, int R, int C, int ldy) {
  __shared__ bf16_t t[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int r = i / 64, c = i % 64;
    if (r0 + r < R && c0 + c < C) t[r][c] = x[(long)(r0 + r) * C + c0 + c];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int c = i / 64, r = i % 64;
    if (r0 + r < R && c0 + c < C) y[(long)(c0 + c) * ldy + r0 + r] = t[r][c];
  }
}

// latents (fp32, channel planes of `plane` elements, rows of `ldz`) -> NHWC bf16 [th*tw, Cpad] of the th x tw
// window at z: z / scaling + shift (pipeline.py:304). The whole image is the window with ldz = tw.
__global__ __launch_bounds__(256) void latent_to_nhwc_kernel(const float* z, long plane, int ldz, int tw, long hw,
                                                             bf16_t* x, int C, int Cpad, float inv_scale,
                                                             float shift) {
  const long total = hw * Cpad;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cpad);
    const long p = i / Cpad;
    const long y = p / tw, xx = p - y * tw;
    x[i] = c < C ? f2bf(z[(long)c * plane + y * ldz + xx] * inv_scale + shift) : (bf16_t)0;
  }
}

// Tiled decode (diffusers AutoencoderKL.tiled_decode, enabled by the reference at generate.py:77-78): blend the
// first e rows (vertical) or columns of decoded tile b with the last e of its upper / left neighbour a, in place:
// b = a * (1 - t/e) + b * (t/e) (AutoencoderKL.blend_v / blend_h). Tiles are fp32 [h][w][4].
__global__ __launch_bounds__(256) void tile_blend_kernel(const float* a, int a_h, int a_w, float* b, int b_w, int rows,
                                                         int cols, int e, int vertical) {
  const long total = (long)rows * cols * 4;
  const float inv_e = 1.0f / (float)e;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i & 3);
    const long q = i >> 2;
    const int y = (int)(q / cols), x = (int)(q - (long)y * cols);
    const float t = (float)(vertical ? y : x) * inv_e;
    const long ai = vertical ? ((long)(a_h - e + y) * a_w + x) : ((long)y * a_w + (a_w - e + x));
    float& bv = b[((long)y * b_w + x) * 4 + c];
    bv = a[ai * 4 + c] * (1.f - t) + bv * t;
  }
}

// the uint8 post-processing (pipeline.py:324-326) of the rows x cols top-left crop of a decoded tile
// (fp32 [.][tw][4]) into the image (uint8 [.][img_w][3]) at (y0, x0)
__global__ __launch_bounds__(256) void tile_to_uint8_kernel(const float* t, int tw, unsigned char* img, int img_w,
                                                            int y0, int x0, int rows, int cols) {
  const long total = (long)rows * cols * 3;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i / 3;
    const int c = (int)(i - p * 3);
    const int y = (int)(p / cols), x = (int)(p - (long)y * cols);
    float v = t[((long)y * tw + x) * 4 + c] * 0.5f + 0.5f;
    v = fminf(fmaxf(v, 0.f), 1.f) * 255.f;
    v = rintf(v);
    img[((long)(y0 + y) * img_w + x0 + x) * 3 + c] = (unsigned char)fminf(fmaxf(v, 0.f), 255.f);
  }
}

// conv_out result (fp32 [H*W, ld]) -> uint8 HWC image: ((x/2 + 0.5).clamp(0,1) * 255).round() (pipeline.py:324-326)
__global__ __launch_bounds__(256) void to_uint8_kernel(const float* o, int ld, unsigned char* img, long hw) {
  const long total = hw * 3;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i / 3;
    const int c = (int)(i % 3);
    float v = o[p * ld + c] * 0.5f + 0.5f;
    v = fminf(fmaxf(v, 0.f), 1.f) * 255.f;
    v = rintf(v);
    img[i] = (unsigned char)fminf(fmaxf(v, 0.f), 255.f);
  }
}

// conv weight [Cout][Cin][3][3] -> [Cout][3][3][Cin_pad] (tap-major, zero channel padding)
__global__ __launch_bounds__(256) void pack_conv_kernel(const bf16_t* w, bf16_t* o, int Cout, int Cin, int Cpad) {
  const long total = (long)Cout * 9 * Cpad;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cpad);
    const int tap = (int)((i / Cpad) % 9);
    const long oc = i / (9L * Cpad);
    o[i] = c < Cin ? w[(oc * Cin + c) * 9 + tap] : (bf16_t)0;
  }
}

int grid_of(long total) {
  long g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  return (int)(g < 1 ? 1 : g);
}

}  // namespace

int group_norm(const bf16_t* x, bf16_t* y, long rows, int C, int G, const bf16_t* gamma, const bf16_t* beta,
               float eps, bool silu, double* stats, hipStream_t s) {
  // gn_stats_kernel reduces 8-channel vectors: a vector must lie inside one group (C/G a multiple of 8) or
  // hold exactly two whole groups (C/G == 4); C/G = 12, 20, ... would straddle groups
  FLITE_REQUIRE(C % G == 0 && C % 8 == 0 && (C / G == 4 || (C / G) % 8 == 0), "group_norm: unsupported channels");
  FLITE_REQUIRE(G <= 64, "group_norm: at most 64 groups");
  const long vecs = rows * (C / 8);
  // the grid stride (blocks * 256) must be a multiple of C/8 so that each thread stays on one channel vector
  FLITE_REQUIRE(256 % (C / 8) == 0, "group_norm: C/8 must divide 256");
  const int blocks = std::min(1024, grid_of(vecs));
  // workspace: stats double[2 * 64], then the per-workgroup partials float[1024][64][2]
  float* partial = (float*)(stats + 2 * 64);
  hipLaunchKernelGGL(gn_stats_kernel, dim3(blocks), dim3(256), 0, s, x, rows, C, G, partial);
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(1), dim3(64 * GN_FIN_LANES), 0, s, partial, blocks, G,
                     (double)rows * (C / G), eps, stats);
  if (silu)
    hipLaunchKernelGGL(gn_apply_kernel<true>, dim3(grid_of(vecs)), dim3(256), 0, s, x, y, rows, C, G, stats, gamma,
                       beta);
  else
    hipLaunchKernelGGL(gn_apply_kernel<false>, dim3(grid_of(vecs)), dim3(256), 0, s, x, y, rows, C, G, stats, gamma,
                       beta);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int softmax_rows(const float* S, bf16_t* P, int R, int L, int ld, float scale, hipStream_t s) {
  FLITE_REQUIRE(ld % 4 == 0 && ld >= L, "softmax_rows: ld must be a multiple of 4 and >= L");
  hipLaunchKernelGGL(softmax_rows_kernel, dim3(R), dim3(256), 0, s, S, P, L, ld, scale);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int transpose_bf16(const bf16_t* x, bf16_t* y, int R, int C, int ldy, hipStream_t s) {
  FLITE_REQUIRE(ldy >= R, "transpose_bf16: ldy must be >= R");
  hipLaunchKernelGGL(transpose_kernel, dim3((C + 63) / 64, (R + 63) / 64), dim3(256), 0, s, x, y, R, C, ldy);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int latent_to_nhwc(const float* z, long plane, int ldz, int th, int tw, bf16_t* x, int C, int Cpad, float scaling,
                   float shift, hipStream_t s) {
  const long hw = (long)th * tw;
  hipLaunchKernelGGL(latent_to_nhwc_kernel, dim3(grid_of(hw * Cpad)), dim3(256), 0, s, z, plane, ldz, tw, hw, x, C,
                     Cpad, 1.0f / scaling, shift);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int tile_blend(const float* a, int a_h, int a_w, float* b, int b_h, int b_w, int e, bool vertical, hipStream_t s) {
  FLITE_REQUIRE(e > 0 && e <= (vertical ? std::min(a_h, b_h) : std::min(a_w, b_w)), "tile_blend: bad extent");
  FLITE_REQUIRE(vertical ? a_w == b_w : a_h == b_h, "tile_blend: neighbours must share the blended edge");
  const int rows = vertical ? e : b_h, cols = vertical ? b_w : e;
  hipLaunchKernelGGL(tile_blend_kernel, dim3(grid_of((long)rows * cols * 4)), dim3(256), 0, s, a, a_h, a_w, b, b_w,
                     rows, cols, e, vertical ? 1 : 0);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int tile_to_uint8(const float* t, int tw, unsigned char* img, int img_w, int y0, int x0, int rows, int cols,
                  hipStream_t s) {
  hipLaunchKernelGGL(tile_to_uint8_kernel, dim3(grid_of((long)rows * cols * 3)), dim3(256), 0, s, t, tw, img, img_w,
                     y0, x0, rows, cols);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int to_uint8(const float* o, int ld, unsigned char* img, long hw, hipStream_t s) {
  hipLaunchKernelGGL(to_uint8_kernel, dim3(grid_of(hw * 3)), dim3(256), 0, s, o, ld, img, hw);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

// fp8 weight storage (VaeEngine::enable_fp8_weights, the analogue of diffusers' layerwise casting with an fp8
// storage dtype): a packed conv weight [Cout][K] -> OCP e4m3 bytes + one E8M0 scale per 32 consecutive K
// (MXFP8, fp8.h rounding: bit-exact to oracle/flite_ref.py mx_quant), row-major scales [Cout][K/32]; and back
// to bf16 right before the conv (exact: an e4m3 value times 2^e has at most 4 significant bits).
__global__ __launch_bounds__(256) void mx_quant_rm_kernel(const bf16_t* x, long nblk, uint8_t* q, uint8_t* sc) {
  const long b = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblk) return;
  float v[32];
  const u32x4* src = (const u32x4*)(x + b * 32);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const u32x4 w = src[c];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[8 * c + 2 * k] = __uint_as_float(w[k] << 16);
      v[8 * c + 2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
    }
  }
  float amax = 0.f;
#pragma unroll
  for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(v[j]));
  const int e = mx_exp(amax);
  const float inv = mx_inv(e);
  u32x4 o[2];
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j >> 2][j & 3] = pack4_fp8(v + 4 * j, inv);
  ((u32x4*)(q + b * 32))[0] = o[0];
  ((u32x4*)(q + b * 32))[1] = o[1];
  sc[b] = (uint8_t)(e + 127);
}

__global__ __launch_bounds__(256) void mx_dequant_rm_kernel(const uint8_t* q, const uint8_t* sc, long nblk,
                                                            bf16_t* x) {
  const long b = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblk) return;
  const float scale = __uint_as_float((unsigned)sc[b] << 23);  // 2^(byte - 127); byte >= 0: e >= -127
  const u32x4* src = (const u32x4*)(q + b * 32);
  u32x4* dst = (u32x4*)(x + b * 32);
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const u32x4 w = src[c];
    u32x4 lo, hi;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const f32x2 a = __builtin_amdgcn_cvt_pk_f32_fp8((int)w[k], false);
      const f32x2 d = __builtin_amdgcn_cvt_pk_f32_fp8((int)w[k], true);
      const unsigned p0 = pack2bf(a[0] * scale, a[1] * scale), p1 = pack2bf(d[0] * scale, d[1] * scale);
      if (k < 2) {
        lo[2 * k] = p0;
        lo[2 * k + 1] = p1;
      } else {
        hi[2 * (k - 2)] = p0;
        hi[2 * (k - 2) + 1] = p1;
      }
    }
    dst[2 * c] = lo;
    dst[2 * c + 1] = hi;
  }
}

int mx_quant_rows_rm(const bf16_t* x, long rows, int K, uint8_t* q, uint8_t* sc, hipStream_t s) {
  FLITE_REQUIRE(K % 32 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)q & 15) == 0, "mx_quant_rows: K % 32, 16-B");
  const long nblk = rows * (K / 32);
  hipLaunchKernelGGL(mx_quant_rm_kernel, dim3((unsigned)((nblk + 255) / 256)), dim3(256), 0, s, x, nblk, q, sc);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int mx_dequant_rows_rm(const uint8_t* q, const uint8_t* sc, long rows, int K, bf16_t* x, hipStream_t s) {
  FLITE_REQUIRE(K % 32 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)q & 15) == 0, "mx_dequant_rows: K % 32");
  const long nblk = rows * (K / 32);
  hipLaunchKernelGGL(mx_dequant_rm_kernel, dim3((unsigned)((nblk + 255) / 256)), dim3(256), 0, s, q, sc, nblk, x);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int pack_conv_weight(const bf16_t* w, bf16_t* o, int Cout, int Cin, int Cpad, hipStream_t s) {
  hipLaunchKernelGGL(pack_conv_kernel, dim3(grid_of((long)Cout * 9 * Cpad)), dim3(256), 0, s, w, o, Cout, Cin, Cpad);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace flite
