// Bandwidth-bound kernels of the Flux VAE decoder (diffusers AutoencoderKL.decode, called at
// reference pipeline.py:307). Activations are NHWC bf16 (one image); the 3x3 convolutions and the
// mid-block attention matmuls run on the MFMA GEMM (gemm.hip, implicit-GEMM conv mode).
#include <math.h>

#include "common.h"
#include "kernels.h"

namespace flite {

namespace {

// GroupNorm statistics: sum / sum of squares per group (double accumulation), NHWC rows of C channels.
// Each thread reads 8 channels (16 B); groups hold C/32 channels (4, 8 or 16).
__global__ __launch_bounds__(256) void gn_stats_kernel(const bf16_t* x, long rows, int C, int G, double* stats) {
  __shared__ float s_sum[64], s_sq[64];
  if (threadIdx.x < 64) {
    s_sum[threadIdx.x] = 0.f;
    s_sq[threadIdx.x] = 0.f;
  }
  __syncthreads();
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
  atomicAdd(&s_sum[g0], ls[0]);
  atomicAdd(&s_sq[g0], lq[0]);
  if (cg < 8) {
    atomicAdd(&s_sum[g0 + 1], ls[1]);
    atomicAdd(&s_sq[g0 + 1], lq[1]);
  }
  __syncthreads();
  if (threadIdx.x < G) {
    atomicAdd(&stats[2 * threadIdx.x], (double)s_sum[threadIdx.x]);
    atomicAdd(&stats[2 * threadIdx.x + 1], (double)s_sq[threadIdx.x]);
  }
}

template <bool SILU>
__global__ __launch_bounds__(256) void gn_apply_kernel(const bf16_t* x, bf16_t* y, long rows, int C, int G,
                                                       const double* stats, const bf16_t* gamma,
                                                       const bf16_t* beta, float eps) {
  const int cg = C / G;
  const double n = (double)rows * cg;
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
        const double mean = stats[2 * g] / n;
        const double var = fmax(stats[2 * g + 1] / n - mean * mean, 0.0);
        const float rstd = (float)(1.0 / sqrt(var + (double)eps));
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

// row softmax: P[r][:] = softmax(scale * S[r][:]) (fp32 in, bf16 out), one workgroup per row
__global__ __launch_bounds__(256) void softmax_rows_kernel(const float* S, bf16_t* P, int L, float scale) {
  __shared__ float red[8];
  const float* s = S + (long)blockIdx.x * L;
  bf16_t* pr = P + (long)blockIdx.x * L;
  float m = -INFINITY;
  for (int i = threadIdx.x * 4; i < L; i += 1024) {
    const f32x4 v = *(const f32x4*)(s + i);
    m = fmaxf(m, fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])));
  }
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])) * scale;
  __syncthreads();
  float sum = 0.f;
  for (int i = threadIdx.x * 4; i < L; i += 1024) {
    const f32x4 v = *(const f32x4*)(s + i);
#pragma unroll
    for (int j = 0; j < 4; ++j) sum += __expf(v[j] * scale - m);
  }
  sum = wave_sum(sum);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sum;
  __syncthreads();
  const float inv = 1.f / (red[0] + red[1] + red[2] + red[3]);
  for (int i = threadIdx.x * 4; i < L; i += 1024) {
    const f32x4 v = *(const f32x4*)(s + i);
    u32x2 w;
    w.x = pack2bf(__expf(v[0] * scale - m) * inv, __expf(v[1] * scale - m) * inv);
    w.y = pack2bf(__expf(v[2] * scale - m) * inv, __expf(v[3] * scale - m) * inv);
    *(u32x2*)(pr + i) = w;
  }
}

// bf16 transpose [R, C] -> [C, R] through a 64x64 LDS tile
__global__ __launch_bounds__(256) void transpose_kernel(const bf16_t* x, bf16_t* y, int R, int C) {
  __shared__ bf16_t t[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int r = i / 64, c = i % 64;
    if (r0 + r < R && c0 + c < C) t[r][c] = x[(long)(r0 + r) * C + c0 + c];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int c = i / 64, r = i % 64;
    if (r0 + r < R && c0 + c < C) y[(long)(c0 + c) * R + r0 + r] = t[r][c];
  }
}

// latents (fp32 [C, h, w] of one image) -> NHWC bf16 [h*w, Cpad]: z / scaling + shift (pipeline.py:304)
__global__ __launch_bounds__(256) void latent_to_nhwc_kernel(const float* z, bf16_t* x, int C, int Cpad, int hw,
                                                             float inv_scale, float shift) {
  const long total = (long)hw * Cpad;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cpad);
    const long p = i / Cpad;
    x[i] = c < C ? f2bf(z[(long)c * hw + p] * inv_scale + shift) : (bf16_t)0;
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
  FLITE_REQUIRE(C % G == 0 && C % 8 == 0 && C / G >= 4 && (C / G) % 4 == 0, "group_norm: unsupported channels");
  FLITE_REQUIRE(G <= 64, "group_norm: at most 64 groups");
  FLITE_HIP_CHECK(hipMemsetAsync(stats, 0, 2 * G * sizeof(double), s));
  const long vecs = rows * (C / 8);
  // the grid stride (blocks * 256) must be a multiple of C/8 so that each thread stays on one channel vector
  FLITE_REQUIRE(256 % (C / 8) == 0, "group_norm: C/8 must divide 256");
  const int blocks = std::min(1024, grid_of(vecs));
  hipLaunchKernelGGL(gn_stats_kernel, dim3(blocks), dim3(256), 0, s, x, rows, C, G, stats);
  if (silu)
    hipLaunchKernelGGL(gn_apply_kernel<true>, dim3(grid_of(vecs)), dim3(256), 0, s, x, y, rows, C, G, stats, gamma,
                       beta, eps);
  else
    hipLaunchKernelGGL(gn_apply_kernel<false>, dim3(grid_of(vecs)), dim3(256), 0, s, x, y, rows, C, G, stats, gamma,
                       beta, eps);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int softmax_rows(const float* S, bf16_t* P, int R, int L, float scale, hipStream_t s) {
  FLITE_REQUIRE(L % 4 == 0, "softmax_rows: L must be a multiple of 4");
  hipLaunchKernelGGL(softmax_rows_kernel, dim3(R), dim3(256), 0, s, S, P, L, scale);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int transpose_bf16(const bf16_t* x, bf16_t* y, int R, int C, hipStream_t s) {
  hipLaunchKernelGGL(transpose_kernel, dim3((C + 63) / 64, (R + 63) / 64), dim3(256), 0, s, x, y, R, C);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int latent_to_nhwc(const float* z, bf16_t* x, int C, int Cpad, int hw, float scaling, float shift, hipStream_t s) {
  hipLaunchKernelGGL(latent_to_nhwc_kernel, dim3(grid_of((long)hw * Cpad)), dim3(256), 0, s, z, x, C, Cpad, hw,
                     1.0f / scaling, shift);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int to_uint8(const float* o, int ld, unsigned char* img, long hw, hipStream_t s) {
  hipLaunchKernelGGL(to_uint8_kernel, dim3(grid_of(hw * 3)), dim3(256), 0, s, o, ld, img, hw);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int pack_conv_weight(const bf16_t* w, bf16_t* o, int Cout, int Cin, int Cpad, hipStream_t s) {
  hipLaunchKernelGGL(pack_conv_kernel, dim3(grid_of((long)Cout * 9 * Cpad)), dim3(256), 0, s, w, o, Cout, Cin, Cpad);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace flite
