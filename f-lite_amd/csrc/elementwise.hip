// HBM-bound kernels of the DiT step (gfx950). Every kernel reads/writes each element once, vectorised
// 16 B per lane; reductions are one wave per row with __shfl_xor.
#include <math.h>

#include "common.h"
#include "fp8.h"
#include "kernels.h"

namespace flite {

namespace {

// ------------------------------------------------------------------------------------------------
// RMSNorm (+ weight) (+ adaLN modulate) -> bf16.
//   y = rmsnorm(x) * w * (1 + scale[seg]) + shift[seg]
// Reference: LigerRMSNorm (model.py:238,248,260,437) / own RMSNorm (model.py:92-108, final_norm),
// then `norm_x * (1 + scale) + shift` (model.py:284,293,300,580). Computed in fp32, one rounding.
// One wave per output row; the input row of output row m is (m / in_seg) * in_stride + in_off + m % in_seg.
// ------------------------------------------------------------------------------------------------
// 4 consecutive outputs o of row m at column n: bf16, or (OUT8) MXFP8 -- the 8 lanes of an aligned group hold the
// 32 columns of one scale block (both norm kernels put 4 consecutive columns on consecutive lanes).
template <bool OUT8>
__device__ __forceinline__ void norm_store4(const NormModParams& p, long m, int n, const float (&o)[4]) {
  if constexpr (OUT8) {
    float amax = fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3])));
    amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
    amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
    amax = fmaxf(amax, __shfl_xor(amax, 4, 64));
    const int e = mx_exp(amax);
    *(unsigned*)(p.y8 + m * p.ldy + n) = pack4_fp8(o, mx_inv(e));
    if ((n & 31) == 0) {
      const int blk = n >> 5;
      p.ysc[((long)(blk >> 2) * p.ysc_rows_pad + m) * 4 + (blk & 3)] = (uint8_t)(e + 127);
    }
  } else {
    u32x2 st;
    st.x = pack2bf(o[0], o[1]);
    st.y = pack2bf(o[2], o[3]);
    *(u32x2*)(p.y + m * p.ldy + n) = st;
  }
}

template <bool IN_BF16, int NCH, bool OUT8 = false>
__global__ __launch_bounds__(256) void rmsnorm_mod_kernel(NormModParams p) {
  const int lane = threadIdx.x & 63;
  const long m = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= p.rows) return;
  const long seg = p.in_seg > 0 ? m / p.in_seg : 0;
  const long in_row = p.in_seg > 0 ? seg * p.in_stride + p.in_off + (m % p.in_seg) : m;
  const int D = p.D;
  // D == 256 * NCH: lane handles 4 consecutive elements of every 256-wide chunk (registers, static index)
  float v[4 * NCH];
  constexpr int nch = NCH;
  float ss = 0.f;
  if constexpr (IN_BF16) {
    const bf16_t* xr = (const bf16_t*)p.x + in_row * p.ldx;
#pragma unroll
    for (int c = 0; c < nch; ++c) {
      const u32x2 w = *(const u32x2*)(xr + c * 256 + lane * 4);
      v[4 * c + 0] = __uint_as_float(w.x << 16);
      v[4 * c + 1] = __uint_as_float(w.x & 0xffff0000u);
      v[4 * c + 2] = __uint_as_float(w.y << 16);
      v[4 * c + 3] = __uint_as_float(w.y & 0xffff0000u);
    }
  } else {
    const float* xr = (const float*)p.x + in_row * p.ldx;
#pragma unroll
    for (int c = 0; c < nch; ++c) {
      const f32x4 w = *(const f32x4*)(xr + c * 256 + lane * 4);
      v[4 * c + 0] = w[0];
      v[4 * c + 1] = w[1];
      v[4 * c + 2] = w[2];
      v[4 * c + 3] = w[3];
    }
  }
#pragma unroll
  for (int i = 0; i < 4 * nch; ++i) ss += v[i] * v[i];
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / (float)D + p.eps);
  const float* shift = p.shift ? p.shift + seg * p.mod_seg_stride : nullptr;
  const float* scale = p.scale ? p.scale + seg * p.mod_seg_stride : nullptr;
#pragma unroll
  for (int c = 0; c < nch; ++c) {
    const int n = c * 256 + lane * 4;
    float o[4];
    float wgt[4] = {1.f, 1.f, 1.f, 1.f};
    if (p.w) {
      const u32x2 ww = *(const u32x2*)(p.w + n);
      wgt[0] = __uint_as_float(ww.x << 16);
      wgt[1] = __uint_as_float(ww.x & 0xffff0000u);
      wgt[2] = __uint_as_float(ww.y << 16);
      wgt[3] = __uint_as_float(ww.y & 0xffff0000u);
    }
    f32x4 sc = {0.f, 0.f, 0.f, 0.f}, sh = {0.f, 0.f, 0.f, 0.f};
    if (scale) sc = *(const f32x4*)(scale + n);
    if (shift) sh = *(const f32x4*)(shift + n);
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = v[4 * c + j] * r * wgt[j] * (1.f + sc[j]) + sh[j];
    norm_store4<OUT8>(p, m, n, o);
  }
}

// Same operation, one 256-thread workgroup per output row, for D = 1024 * NQ (the DiT width 3072: NQ = 3).
// Thread t holds elements q*1024 + 4t .. +3 (q < NQ): 12 fp32 registers of x instead of 48, so 8 waves per
// SIMD stay resident and every wave has all of its row loads in flight at once; the row sum of squares is
// a wave reduction plus 4 partials through LDS.
// PF: the weight read-ahead below is compiled in; the PF = false instantiation is the plain kernel (the
// read-ahead's registers and loads had cost every launch ~8 us, round-2 VERDICT item 4).
// BC: the deferred broadcast residual of NormModParams (bc_*), applied to the row (fp32 or, IN_BF16, the bf16
// residual stream) before the reduction.
template <bool IN_BF16, int NQ, bool OUT8 = false, bool PF = false, bool BC = false>
__global__ __launch_bounds__(256) void rmsnorm_mod_row_kernel(NormModParams p) {
  __shared__ float part[4];
  const int t = threadIdx.x;
  const long m = blockIdx.x;
  const long seg = p.in_seg > 0 ? m / p.in_seg : 0;
  const long in_row = p.in_seg > 0 ? seg * p.in_stride + p.in_off + (m % p.in_seg) : m;
  float v[4 * NQ];
  if constexpr (IN_BF16) {
    const bf16_t* xr = (const bf16_t*)p.x + in_row * p.ldx;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const u32x2 w = *(const u32x2*)(xr + q * 1024 + t * 4);
      v[4 * q + 0] = __uint_as_float(w.x << 16);
      v[4 * q + 1] = __uint_as_float(w.x & 0xffff0000u);
      v[4 * q + 2] = __uint_as_float(w.y << 16);
      v[4 * q + 3] = __uint_as_float(w.y & 0xffff0000u);
    }
    if constexpr (BC) {  // bf16 residual stream (DitEngine resid16): the same fma, one rounding, written back
      if (m < p.bc_rows) {
        const long bs = m / p.bc_rows_per_seg;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const int n = q * 1024 + t * 4;
          const f32x4 cv = *(const f32x4*)(p.bc_c + bs * (long)(1024 * NQ) + n);
          const f32x4 gv = *(const f32x4*)(p.bc_gate + bs * p.bc_gate_stride + n);
          float nv[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) nv[j] = __builtin_fmaf(cv[j], gv[j], v[4 * q + j]);
          const u32x2 st = {pack2bf(nv[0], nv[1]), pack2bf(nv[2], nv[3])};
          *(u32x2*)((bf16_t*)p.x + in_row * p.ldx + n) = st;
          v[4 * q + 0] = __uint_as_float(st.x << 16);  // normalise what the stream now holds
          v[4 * q + 1] = __uint_as_float(st.x & 0xffff0000u);
          v[4 * q + 2] = __uint_as_float(st.y << 16);
          v[4 * q + 3] = __uint_as_float(st.y & 0xffff0000u);
        }
      }
    }
  } else {
    const float* xr = (const float*)p.x + in_row * p.ldx;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const f32x4 w = *(const f32x4*)(xr + q * 1024 + t * 4);
      v[4 * q + 0] = w[0];
      v[4 * q + 1] = w[1];
      v[4 * q + 2] = w[2];
      v[4 * q + 3] = w[3];
    }
    if constexpr (BC) {
      if (m < p.bc_rows) {  // uniform over the workgroup (one row)
        const long bs = m / p.bc_rows_per_seg;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const int n = q * 1024 + t * 4;
          const f32x4 cv = *(const f32x4*)(p.bc_c + bs * (long)(1024 * NQ) + n);
          const f32x4 gv = *(const f32x4*)(p.bc_gate + bs * p.bc_gate_stride + n);
          f32x4 nv;
#pragma unroll
          for (int j = 0; j < 4; ++j) nv[j] = v[4 * q + j] = __builtin_fmaf(cv[j], gv[j], v[4 * q + j]);
          *(f32x4*)((float*)p.x + in_row * p.ldx + n) = nv;  // ctx_bcast_resid_kernel's fma, in place
        }
      }
    }
  }
  // weight, scale and shift (L2-resident, shared by all rows) are loaded before the reduction, so the row's
  // two memory round trips overlap instead of running back to back
  const float* shift = p.shift ? p.shift + seg * p.mod_seg_stride : nullptr;
  const float* scale = p.scale ? p.scale + seg * p.mod_seg_stride : nullptr;
  float wgt[NQ][4];
  f32x4 sc[NQ], sh[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int n = q * 1024 + t * 4;
    wgt[q][0] = wgt[q][1] = wgt[q][2] = wgt[q][3] = 1.f;
    if (p.w) {
      const u32x2 ww = *(const u32x2*)(p.w + n);
      wgt[q][0] = __uint_as_float(ww.x << 16);
      wgt[q][1] = __uint_as_float(ww.x & 0xffff0000u);
      wgt[q][2] = __uint_as_float(ww.y << 16);
      wgt[q][3] = __uint_as_float(ww.y & 0xffff0000u);
    }
    sc[q] = scale ? *(const f32x4*)(scale + n) : f32x4{0.f, 0.f, 0.f, 0.f};
    sh[q] = shift ? *(const f32x4*)(shift + n) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 4 * NQ; ++i) ss += v[i] * v[i];
  ss = wave_sum(ss);
  if ((t & 63) == 0) part[t >> 6] = ss;
  __syncthreads();
  ss = part[0] + part[1] + part[2] + part[3];
  const float r = rsqrtf(ss / (float)(1024 * NQ) + p.eps);
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int n = q * 1024 + t * 4;
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = v[4 * q + j] * r * wgt[q][j] * (1.f + sc[q][j]) + sh[q][j];
    norm_store4<OUT8>(p, m, n, o);
  }
  // Read-ahead of the next GEMM's weights, after this row's stores: workgroup b touches the 4 KiB pieces b,
  // b + grid, ... (at most PF per range) of each range, all issued before any is consumed; the xor only keeps
  // the loads alive (the store never happens: pf_bytes >= 0).
  if constexpr (PF) {
    constexpr int NPF = 6;
    unsigned pf_acc = 0;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      if (p.pf[r] == nullptr) continue;
      const long pieces = p.pf_bytes[r] >> 12;
      u32x4 v[NPF];
#pragma unroll
      for (int k = 0; k < NPF; ++k) {
        const long i = m + (long)k * gridDim.x;
        v[k] = i < pieces ? ((const u32x4*)((const char*)p.pf[r] + (i << 12)))[t] : u32x4{0u, 0u, 0u, 0u};
      }
#pragma unroll
      for (int k = 0; k < NPF; ++k) pf_acc ^= v[k].x ^ v[k].w;
    }
    if (p.pf_bytes[0] < 0 && pf_acc == 0x9e3779b9u) part[0] = 0.f;
  }
}

// ------------------------------------------------------------------------------------------------
// RoPE (2-D, rotate-half pairs (j, j+128), rotation by -theta) + per-head RMSNorm (no weight), in place
// on bf16 heads of 256. Reference: apply_rotary_emb (model.py:403-414) then QKNorm (model.py:115-126,180,197).
// ------------------------------------------------------------------------------------------------
// 16 B per lane: a half-wave per head, two heads per wave. Lane s = lane & 31 of its half
// holds elements 8(s&15) .. +7 of head half (s>>4), so its rotation partner is lane ^ 16 and the head's sum of
// squares is a 32-lane reduction.
__global__ __launch_bounds__(256) void rope_qknorm16_kernel(RopeNormParams p) {
  const int lane = threadIdx.x & 63;
  const long item = (long)blockIdx.x * 4 + (threadIdx.x >> 6);  // (row, head pair)
  const int pairs = (p.heads + 1) >> 1;
  const long total = (long)p.rows * pairs;
  if (item >= total) return;
  const long row = item / pairs;
  const int head = (int)(item % pairs) * 2 + (lane >> 5);
  const int s = lane & 31;
  const int part = s >> 4;
  const int j0 = 8 * (s & 15);  // angle index of this lane's first element
  const bool live = head < p.heads;
  bf16_t* xp = p.x + row * p.ldx + (long)min(head, p.heads - 1) * 256 + 128 * part + j0;
  const u32x4 w = *(const u32x4*)xp;
  float v[8];
  v[0] = __uint_as_float(w.x << 16);
  v[1] = __uint_as_float(w.x & 0xffff0000u);
  v[2] = __uint_as_float(w.y << 16);
  v[3] = __uint_as_float(w.y & 0xffff0000u);
  v[4] = __uint_as_float(w.z << 16);
  v[5] = __uint_as_float(w.z & 0xffff0000u);
  v[6] = __uint_as_float(w.w << 16);
  v[7] = __uint_as_float(w.w & 0xffff0000u);
  if (p.cos != nullptr && head < p.rope_heads) {
    const long tok = row % p.tokens_per_seq;
    const f32x4 c0 = *(const f32x4*)(p.cos + tok * 128 + j0);
    const f32x4 c1 = *(const f32x4*)(p.cos + tok * 128 + j0 + 4);
    const f32x4 s0 = *(const f32x4*)(p.sin + tok * 128 + j0);
    const f32x4 s1 = *(const f32x4*)(p.sin + tok * 128 + j0 + 4);
    const float c[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
    const float sn[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float partner = __shfl_xor(v[i], 16, 64);
      // first half holds x1 (y1 = x1 c + x2 s); second half holds x2 (y2 = -x1 s + x2 c)
      o[i] = part == 0 ? (v[i] * c[i] + partner * sn[i]) : (-partner * sn[i] + v[i] * c[i]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = o[i];
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) ss += v[i] * v[i];
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  const float r = rsqrtf(ss * (1.f / 256.f) + p.eps);
  if (!live) return;
  u32x4 st;
  st.x = pack2bf(v[0] * r, v[1] * r);
  st.y = pack2bf(v[2] * r, v[3] * r);
  st.z = pack2bf(v[4] * r, v[5] * r);
  st.w = pack2bf(v[6] * r, v[7] * r);
  *(u32x4*)xp = st;
}

// ------------------------------------------------------------------------------------------------
// Patchify (PatchEmbed conv k=s=p as a GEMM, model.py:318-331): latents [Bi, C, H, W] (fp32 or bf16)
// -> patches bf16 [dup*Bi*(H/p)*(W/p), C*p*p] with columns in (c, p1, p2) order (= conv weight layout).
// Copy `d` of image i lands at batch index d*Bi + i (CFG batch = cat([latents]*2), pipeline.py:264).
// ------------------------------------------------------------------------------------------------
template <bool IN_BF16>
__global__ __launch_bounds__(256) void patchify_kernel(const void* lat, bf16_t* out, int Bi, int C, int H, int W,
                                                       int P, int dup) {
  const int hp = H / P, wp = W / P;
  const int K = C * P * P;
  const long total = (long)dup * Bi * hp * wp * K;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int k = (int)(idx % K);
    const long row = idx / K;
    const int x = (int)(row % wp);
    const int y = (int)((row / wp) % hp);
    const long b = row / ((long)wp * hp);
    const int i = (int)(b % Bi);
    const int c = k / (P * P);
    const int p1 = (k / P) % P;
    const int p2 = k % P;
    const long src = (((long)i * C + c) * H + (y * P + p1)) * W + (x * P + p2);
    float v;
    if constexpr (IN_BF16)
      v = bf2f(((const bf16_t*)lat)[src]);
    else
      v = ((const float*)lat)[src];
    out[idx] = f2bf(v);
  }
}

// register tokens into rows [0, R) of every sequence of the residual stream (fp32, or bf16 when X16)
template <bool X16>
__global__ __launch_bounds__(256) void fill_registers_kernel(void* x, const bf16_t* reg, int B, int T, int R, int D) {
  const long total = (long)B * R * D;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int d = (int)(idx % D);
    const long r = (idx / D) % R;
    const long b = idx / ((long)D * R);
    if constexpr (X16)
      ((bf16_t*)x)[(b * T + r) * D + d] = reg[r * D + d];
    else
      ((float*)x)[(b * T + r) * D + d] = bf2f(reg[r * D + d]);
  }
}

// x[b][t] += positional_embedding[t] for every row t of every sample (use_rope = False, model.py:546)
template <bool X16>
__global__ __launch_bounds__(256) void add_pos_embed_kernel(void* x, const bf16_t* pos, int B, int T, int D) {
  const long total = (long)B * T * D;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    if constexpr (X16)
      ((bf16_t*)x)[idx] = f2bf(bf2f(((bf16_t*)x)[idx]) + bf2f(pos[idx % ((long)T * D)]));
    else
      ((float*)x)[idx] += bf2f(pos[idx % ((long)T * D)]);
  }
}

// ------------------------------------------------------------------------------------------------
// Unpatchify + classifier-free guidance + Euler update (pipeline.py:274,290,296-297; model.py:583-590).
//   out rows = [dup*Bi*HW, C*p*p] fp32 with columns (p1, p2, c); image i uses rows of copy 0 (uncond)
//   and copy 1 (cond): v = u + g (c - u); acc[i] += dt * v  (fp32 accumulator, [Bi, C, H, W])
// With guidance disabled (dup == 1) v = out.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void cfg_euler_kernel(const float* out, float* acc, int Bi, int C, int H, int W,
                                                        int P, int dup, float g, float dt) {
  const int hp = H / P, wp = W / P;
  const long HW = (long)hp * wp;
  const long total = (long)Bi * C * H * W;
  const int K = C * P * P;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int x = (int)(idx % W);
    const int y = (int)((idx / W) % H);
    const int c = (int)((idx / ((long)W * H)) % C);
    const long i = idx / ((long)W * H * C);
    const long prow = (long)(y / P) * wp + (x / P);
    const int col = ((y % P) * P + (x % P)) * C + c;
    float v;
    if (dup == 2) {
      const float u = out[(i * HW + prow) * K + col];
      const float cc = out[((Bi + i) * HW + prow) * K + col];
      v = u + g * (cc - u);
    } else {
      v = out[(i * HW + prow) * K + col];
    }
    acc[idx] += dt * v;
  }
}

// CFG + Euler over NCHW branch outputs, for the CFG-parallel mode where the uncond and cond branches run on
// two ranks and their [Bi, C, H, W] outputs are exchanged before the update. The fp32 expressions are those
// of cfg_euler_kernel, so equal branch outputs give a bit-identical accumulator.
__global__ __launch_bounds__(256) void cfg_euler_nchw_kernel(const float* u, const float* c, float* acc, long n,
                                                             float g, float dt, int use_cfg) {
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (long)gridDim.x * blockDim.x) {
    float v;
    if (use_cfg) {
      const float uu = u[idx];
      const float cc = c[idx];
      v = uu + g * (cc - uu);
    } else {
      v = c[idx];
    }
    acc[idx] += dt * v;
  }
}

// ------------------------------------------------------------------------------------------------
// Adaptive projected guidance (APG, pipeline.py:276-287) + Euler update. The reference reduces over the
// WHOLE batch tensor, so one 1024-thread workgroup does the three passes (sums, std, update) in-launch.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float block_sum_1024(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = (threadIdx.x < 16) ? red[threadIdx.x] : 0.f;
  if (w == 0) t = wave_sum(t);
  if (threadIdx.x == 0) red[16] = t;
  __syncthreads();
  return red[16];
}

__global__ __launch_bounds__(1024) void apg_euler_kernel(const float* out, float* acc, int Bi, int C, int H, int W,
                                                         int P, float g, float thr, float dt) {
  __shared__ float red[32];
  const int wp = W / P;
  const long HW = (long)(H / P) * wp;
  const long n = (long)Bi * C * H * W;
  const int K = C * P * P;
  auto uc = [&](long idx, float& u, float& c) {
    const int x = (int)(idx % W);
    const int y = (int)((idx / W) % H);
    const int ch = (int)((idx / ((long)W * H)) % C);
    const long i = idx / ((long)W * H * C);
    const long prow = (long)(y / P) * wp + (x / P);
    const int col = ((y % P) * P + (x % P)) * C + ch;
    u = out[(i * HW + prow) * K + col];
    c = out[((Bi + i) * HW + prow) * K + col];
  };
  float s_dd = 0.f, s_yy = 0.f;
  for (long idx = threadIdx.x; idx < n; idx += blockDim.x) {
    float u, c;
    uc(idx, u, c);
    s_dd += c * (c - u);
    s_yy += c * c;
  }
  const float dydd = block_sum_1024(s_dd, red);
  const float dyy = block_sum_1024(s_yy, red);
  const float k = dyy > 0.f ? dydd / dyy : 0.f;
  float s1 = 0.f, s2 = 0.f;
  for (long idx = threadIdx.x; idx < n; idx += blockDim.x) {
    float u, c;
    uc(idx, u, c);
    const float o = (c - u) - k * c;
    s1 += o;
    s2 += o * o;
  }
  const float so = block_sum_1024(s1, red);
  const float soo = block_sum_1024(s2, red);
  const float mean = so / (float)n;
  const float var = n > 1 ? fmaxf(soo - mean * so, 0.f) / (float)(n - 1) : 0.f;
  const float sd = sqrtf(var);
  const float sc = sd > 0.f ? fminf(1.f, thr / sd) : 1.f;
  for (long idx = threadIdx.x; idx < n; idx += blockDim.x) {
    float u, c;
    uc(idx, u, c);
    const float o = (c - u) - k * c;
    acc[idx] += dt * (c + (g - 1.f) * sc * o);
  }
}

// APG split into its two batch-global reductions and the update, over NCHW fp32 branch outputs, for the modes
// where the uncond / cond outputs are exchanged between ranks (CFG-parallel) or the images of one reference
// batch live on different ranks (data parallel: the partial sums are all-reduced between the phases, SURVEY
// §8e). Same expressions and the same thread-strided summation order as apg_euler_kernel, so one rank holding
// the whole batch gets bit-identical sums.
//   phase 0: out = [sum c (c - u), sum c^2]            (dy = c, dd = c - u: pipeline.py:278-281)
//   phase 1: out = [sum o, sum o^2], o = (c - u) - k c  (orthogonal part, for its std: pipeline.py:282-284)
// Uniform-context collapse (dit.cpp set_context / run_block). bad[s] = 1 when a row of context sequence s differs
// (bit for bit) from its first row. Grid (nseq, chunks): chunk c compares rows first + 1 + c, + chunks, ...; a
// mismatch is recorded by plain stores of 1 (any number of lanes may store it; the host zeroes bad first).
__global__ __launch_bounds__(256) void rows_uniform_kernel(const unsigned* x, long ld_words, const int* cu,
                                                           int cols_words, int* bad) {
  const int s = blockIdx.x;
  const int r0 = cu[s], r1 = cu[s + 1];
  const unsigned* first = x + (long)r0 * ld_words;
  int diff = 0;
  for (long r = r0 + 1 + blockIdx.y; r < r1; r += gridDim.y) {
    const unsigned* row = x + r * ld_words;
    for (int c = threadIdx.x; c < cols_words; c += blockDim.x) diff |= row[c] != first[c];
  }
  if (diff) bad[s] = 1;
}

// Collapsed rows r < rows (sequences whose cross-attention keys are all equal): the attention output of every such
// row is the sequence's one V row, so the gated residual of its cross-proj is the step-invariant c[seq] = V.Wproj^T
// (made once per set_context): x[r][n] += gate[seq][n] * c[seq][n] -- the cross-proj epilogue's own expression.
// (X16: the bf16 residual stream, one rounding of the fp32 fma; rmsnorm_mod_row_kernel's BC form, bit for bit)
template <bool X16>
__global__ __launch_bounds__(256) void ctx_bcast_resid_kernel(void* x, const float* c, const float* gate,
                                                              long gate_seg_stride, int rows_per_seg, long rows,
                                                              int D) {
  const int d4 = D / 4;
  const long n4 = rows * d4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const long r = i / d4;
    const int n = (int)(i - r * d4) * 4;
    const long seq = r / rows_per_seg;
    f32x4 xv;
    if constexpr (X16) {
      const u32x2 w = *(const u32x2*)((const bf16_t*)x + r * D + n);
      xv = f32x4{__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u), __uint_as_float(w.y << 16),
                 __uint_as_float(w.y & 0xffff0000u)};
    } else {
      xv = *(const f32x4*)((const float*)x + r * D + n);
    }
    const f32x4 cv = *(const f32x4*)(c + seq * D + n);
    const f32x4 gv = *(const f32x4*)(gate + seq * gate_seg_stride + n);
#pragma unroll
    for (int j = 0; j < 4; ++j) xv[j] = __builtin_fmaf(cv[j], gv[j], xv[j]);
    if constexpr (X16)
      *(u32x2*)((bf16_t*)x + r * D + n) = u32x2{pack2bf(xv[0], xv[1]), pack2bf(xv[2], xv[3])};
    else
      *(f32x4*)((float*)x + r * D + n) = xv;
  }
}

// Device-resident scalars (flite_apg_sums_dev / flite_apg_euler_dev): ws[0..1] = the phase-0 sums, ws[2..3] = the
// phase-1 sums, each after any all-reduce between the ranks; k and the orthogonal scale are derived where they are
// used, with apg_euler_kernel's fp32 expressions, so a multi-rank APG step needs no host round trip.
__device__ __forceinline__ float apg_k_of(const float* ws) { return ws[1] > 0.f ? ws[0] / ws[1] : 0.f; }
__device__ __forceinline__ float apg_scale_of(const float* ws, long n, float thr) {
  const float so = ws[2], soo = ws[3];
  const float mean = so / (float)n;
  const float var = n > 1 ? fmaxf(soo - mean * so, 0.f) / (float)(n - 1) : 0.f;
  const float sd = sqrtf(var);
  return sd > 0.f ? fminf(1.f, thr / sd) : 1.f;
}

__global__ __launch_bounds__(1024) void apg_sums_kernel(const float* u, const float* c, long n, float k, int phase,
                                                        const float* ws_k, float* out) {
  __shared__ float red[32];
  if (ws_k != nullptr) k = apg_k_of(ws_k);
  float a = 0.f, b = 0.f;
  for (long idx = threadIdx.x; idx < n; idx += blockDim.x) {
    const float uu = u[idx], cc = c[idx];
    if (phase == 0) {
      a += cc * (cc - uu);
      b += cc * cc;
    } else {
      const float o = (cc - uu) - k * cc;
      a += o;
      b += o * o;
    }
  }
  a = block_sum_1024(a, red);
  b = block_sum_1024(b, red);
  if (threadIdx.x == 0) {
    out[0] = a;
    out[1] = b;
  }
}

// acc += dt * (dy + (g - 1) * sc * orth)   (pipeline.py:285-286,296); with ws, k and sc come from the device sums
__global__ __launch_bounds__(256) void apg_update_nchw_kernel(const float* u, const float* c, float* acc, long n,
                                                              float g, float k, float sc, float dt, const float* ws,
                                                              long n_total, float thr) {
  if (ws != nullptr) {
    k = apg_k_of(ws);
    sc = apg_scale_of(ws, n_total, thr);
  }
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (long)gridDim.x * blockDim.x) {
    const float uu = u[idx], cc = c[idx];
    const float o = (cc - uu) - k * cc;
    acc[idx] += dt * (cc + (g - 1.f) * sc * o);
  }
}

// unpatchify only (DiT.forward output, model.py:583-590): out rows [B*HW, C*p*p] -> y [B, C, H, W]
template <bool OUT_BF16>
__global__ __launch_bounds__(256) void unpatchify_kernel(const float* out, void* y, int B, int C, int H, int W,
                                                         int P) {
  const int hp = H / P, wp = W / P;
  const long HW = (long)hp * wp;
  const long total = (long)B * C * H * W;
  const int K = C * P * P;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int x = (int)(idx % W);
    const int yy = (int)((idx / W) % H);
    const int c = (int)((idx / ((long)W * H)) % C);
    const long i = idx / ((long)W * H * C);
    const long prow = (long)(yy / P) * wp + (x / P);
    const int col = ((yy % P) * P + (x % P)) * C + c;
    const float v = out[(i * HW + prow) * K + col];
    if constexpr (OUT_BF16)
      ((bf16_t*)y)[idx] = f2bf(v);
    else
      ((float*)y)[idx] = v;
  }
}

// ------------------------------------------------------------------------------------------------
// Timestep embedding (model.py:20-28, 551) with the reference bf16 quantisation of the bf16 pipeline:
//   t_q = bf16(bf16(t) * 1000) (pipeline.py:260 + model.py:551), emb = [cos(t_q f), sin(t_q f)], f_j =
//   exp(-ln(1e4) j / half); the embedding is cast to bf16 (model.py:551 .to(dtype)).
// quantize = 0 reproduces the fp32 model (t * 1000 in fp32).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void timestep_embed_kernel(const float* t, bf16_t* emb, int n, int D,
                                                             int quantize) {
  const int half = D / 2;
  const long total = (long)n * D;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int j = (int)(idx % D);
    const long i = idx / D;
    float tv = t[i];
    if (quantize) {
      tv = bf2f(f2bf(tv));
      tv = bf2f(f2bf(tv * 1000.f));
    } else {
      tv = tv * 1000.f;
    }
    const int jj = j < half ? j : j - half;
    const float freq = expf(-9.210340371976184f * (float)jj / (float)half);
    const float a = tv * freq;
    emb[idx] = f2bf(j < half ? cosf(a) : sinf(a));
  }
}

// ------------------------------------------------------------------------------------------------
// 2-D RoPE tables (TwoDimRotary, model.py:334-386): rows [0, R) are registers (cos 1, sin 0); token
// R + y*w + x gets cat(y * inv_freq, x * inv_freq); values rounded to bf16 when the model is bf16
// (buffers are cast by .to(bf16)). inv_freq (64 fp32) comes from the host (double math).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void rope_table_kernel(const float* inv_freq, float* cos_t, float* sin_t, int hh,
                                                         int ww, int R, int round_bf16) {
  const long total = (long)(R + hh * ww) * 128;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int j = (int)(idx % 128);
    const long tok = idx / 128;
    float c = 1.f, s = 0.f;
    if (tok >= R) {
      const long q = tok - R;
      const int y = (int)(q / ww), x = (int)(q % ww);
      const float pos = j < 64 ? (float)y : (float)x;
      const float a = pos * inv_freq[j & 63];
      c = cosf(a);
      s = sinf(a);
      if (round_bf16) {
        c = bf2f(f2bf(c));
        s = bf2f(f2bf(s));
      }
    }
    cos_t[idx] = c;
    sin_t[idx] = s;
  }
}

// gather rows (context compaction by the attention mask, model.py:31-64)
__global__ __launch_bounds__(256) void gather_rows_kernel(const bf16_t* src, bf16_t* dst, const int* idx, long n,
                                                          int cols) {
  const long total = n * cols / 8;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / (cols / 8);
    const int c = (int)(i % (cols / 8));
    ((u32x4*)dst)[r * (cols / 8) + c] = ((const u32x4*)src)[(long)idx[r] * (cols / 8) + c];
  }
}

int grid_for(long total, int per_block = 256) {
  long g = (total + per_block - 1) / per_block;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

int rmsnorm_mod(const NormModParams& p, bool in_bf16, hipStream_t s) {
  FLITE_REQUIRE(p.ldx % 4 == 0 && p.ldy % 4 == 0, "rmsnorm: strides must be multiples of 4");
  FLITE_REQUIRE(p.bc_rows <= 0 || (p.D == 3072 && p.rows < (1L << 31)),
                "rmsnorm: the deferred broadcast residual is implemented for the D = 3072 row kernel only");
  if (p.rows <= 0) return 0;
  if (p.y8 != nullptr) {  // MXFP8 output (fp8 DiT path): fp32 or bf16 residual rows
    FLITE_REQUIRE(p.ysc != nullptr && p.ysc_rows_pad >= mx_rows_pad(p.rows) && p.D % 128 == 0 && p.ldy % 16 == 0,
                  "rmsnorm(fp8 out): scales for the padded rows, D % 128, 16-B row stride");
    if (p.D == 3072) {
      if (p.bc_rows > 0) {
        FLITE_REQUIRE(p.in_seg == p.in_stride && p.in_off == 0 && p.bc_c && p.bc_gate && p.bc_rows_per_seg > 0,
                      "rmsnorm(fp8 out): the deferred broadcast residual needs the rows in place");
        if (in_bf16)
          hipLaunchKernelGGL((rmsnorm_mod_row_kernel<true, 3, true, false, true>), dim3((unsigned)p.rows), dim3(256),
                             0, s, p);
        else
          hipLaunchKernelGGL((rmsnorm_mod_row_kernel<false, 3, true, false, true>), dim3((unsigned)p.rows), dim3(256),
                             0, s, p);
      } else if (in_bf16) {
        hipLaunchKernelGGL((rmsnorm_mod_row_kernel<true, 3, true>), dim3((unsigned)p.rows), dim3(256), 0, s, p);
      } else {
        hipLaunchKernelGGL((rmsnorm_mod_row_kernel<false, 3, true>), dim3((unsigned)p.rows), dim3(256), 0, s, p);
      }
    } else {
      const int grid8 = (int)((p.rows + 3) / 4);
#define FLITE_NORM8_CASE(N)                                                                        \
  case N:                                                                                           \
    if (in_bf16)                                                                                    \
      hipLaunchKernelGGL((rmsnorm_mod_kernel<true, N, true>), dim3(grid8), dim3(256), 0, s, p);     \
    else                                                                                            \
      hipLaunchKernelGGL((rmsnorm_mod_kernel<false, N, true>), dim3(grid8), dim3(256), 0, s, p);    \
    break;
      switch (p.D / 256) {
        FLITE_NORM8_CASE(1)
        FLITE_NORM8_CASE(2)
        FLITE_NORM8_CASE(4)
        default: FLITE_REQUIRE(false, "rmsnorm(fp8 out): D must be 256, 512, 1024 or 3072");
      }
#undef FLITE_NORM8_CASE
    }
    FLITE_HIP_CHECK(hipGetLastError());
    return 0;
  }
  if (p.D == 3072 && p.rows < (1L << 31)) {  // the DiT width: one workgroup per row
    const bool pf = p.pf[0] != nullptr || p.pf[1] != nullptr;
    if (p.bc_rows > 0) {
      FLITE_REQUIRE(!pf && p.in_seg == p.in_stride && p.in_off == 0 && p.bc_c && p.bc_gate && p.bc_rows_per_seg > 0,
                    "rmsnorm: the deferred broadcast residual needs the rows in place, no read-ahead");
      if (in_bf16)
        hipLaunchKernelGGL((rmsnorm_mod_row_kernel<true, 3, false, false, true>), dim3((unsigned)p.rows), dim3(256), 0,
                           s, p);
      else
        hipLaunchKernelGGL((rmsnorm_mod_row_kernel<false, 3, false, false, true>), dim3((unsigned)p.rows), dim3(256),
                           0, s, p);
    } else if (in_bf16 && pf)
      hipLaunchKernelGGL((rmsnorm_mod_row_kernel<true, 3, false, true>), dim3((unsigned)p.rows), dim3(256), 0, s, p);
    else if (in_bf16)
      hipLaunchKernelGGL((rmsnorm_mod_row_kernel<true, 3>), dim3((unsigned)p.rows), dim3(256), 0, s, p);
    else if (pf)
      hipLaunchKernelGGL((rmsnorm_mod_row_kernel<false, 3, false, true>), dim3((unsigned)p.rows), dim3(256), 0, s,
                         p);
    else
      hipLaunchKernelGGL((rmsnorm_mod_row_kernel<false, 3>), dim3((unsigned)p.rows), dim3(256), 0, s, p);
    FLITE_HIP_CHECK(hipGetLastError());
    return 0;
  }
  const int grid = (int)((p.rows + 3) / 4);
#define FLITE_NORM_CASE(N)                                                                      \
  case N:                                                                                        \
    if (in_bf16)                                                                                 \
      hipLaunchKernelGGL((rmsnorm_mod_kernel<true, N>), dim3(grid), dim3(256), 0, s, p);         \
    else                                                                                         \
      hipLaunchKernelGGL((rmsnorm_mod_kernel<false, N>), dim3(grid), dim3(256), 0, s, p);        \
    break;
  FLITE_REQUIRE(p.D % 256 == 0, "rmsnorm: D must be a multiple of 256");
  switch (p.D / 256) {
    FLITE_NORM_CASE(1)
    FLITE_NORM_CASE(2)
    FLITE_NORM_CASE(3)
    FLITE_NORM_CASE(4)
    FLITE_NORM_CASE(6)
    FLITE_NORM_CASE(8)
    FLITE_NORM_CASE(12)
    FLITE_NORM_CASE(16)
    default:
      FLITE_REQUIRE(false, "rmsnorm: unsupported D (256 x {1,2,3,4,6,8,12,16})");
  }
#undef FLITE_NORM_CASE
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int rope_qknorm(const RopeNormParams& p, hipStream_t s) {
  FLITE_REQUIRE(p.ldx % 4 == 0, "rope_qknorm: stride must be a multiple of 4");
  if (p.cos) FLITE_REQUIRE(p.tokens_per_seq > 0, "rope_qknorm: tokens_per_seq must be > 0");
  const long items = (long)p.rows * ((p.heads + 1) / 2);
  if (items <= 0) return 0;
  FLITE_REQUIRE(p.ldx % 8 == 0 && ((uintptr_t)p.x & 15) == 0, "rope_qknorm: rows must be 16-B aligned");
  hipLaunchKernelGGL(rope_qknorm16_kernel, dim3((unsigned)((items + 3) / 4)), dim3(256), 0, s, p);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int patchify(const void* lat, bool in_bf16, bf16_t* out, int Bi, int C, int H, int W, int P, int dup,
             hipStream_t s) {
  const long total = (long)dup * Bi * C * H * W;
  if (in_bf16)
    hipLaunchKernelGGL(patchify_kernel<true>, dim3(grid_for(total)), dim3(256), 0, s, lat, out, Bi, C, H, W, P, dup);
  else
    hipLaunchKernelGGL(patchify_kernel<false>, dim3(grid_for(total)), dim3(256), 0, s, lat, out, Bi, C, H, W, P,
                       dup);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int fill_registers(void* x, bool x16, const bf16_t* reg, int B, int T, int R, int D, hipStream_t s) {
  if (x16)
    hipLaunchKernelGGL(fill_registers_kernel<true>, dim3(grid_for((long)B * R * D)), dim3(256), 0, s, x, reg, B, T,
                       R, D);
  else
    hipLaunchKernelGGL(fill_registers_kernel<false>, dim3(grid_for((long)B * R * D)), dim3(256), 0, s, x, reg, B, T,
                       R, D);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int add_pos_embed(void* x, bool x16, const bf16_t* pos, int B, int T, int D, hipStream_t s) {
  FLITE_REQUIRE(pos != nullptr, "add_pos_embed: positional_embedding not bound");
  if (x16)
    hipLaunchKernelGGL(add_pos_embed_kernel<true>, dim3(grid_for((long)B * T * D)), dim3(256), 0, s, x, pos, B, T, D);
  else
    hipLaunchKernelGGL(add_pos_embed_kernel<false>, dim3(grid_for((long)B * T * D)), dim3(256), 0, s, x, pos, B, T,
                       D);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int cfg_euler(const float* out, float* acc, int Bi, int C, int H, int W, int P, int dup, float g, float dt,
              hipStream_t s) {
  hipLaunchKernelGGL(cfg_euler_kernel, dim3(grid_for((long)Bi * C * H * W)), dim3(256), 0, s, out, acc, Bi, C, H,
                     W, P, dup, g, dt);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int cfg_euler_nchw(const float* u, const float* c, float* acc, long n, float g, float dt, int use_cfg,
                   hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(cfg_euler_nchw_kernel, dim3(grid_for(n)), dim3(256), 0, s, u, c, acc, n, g, dt, use_cfg);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int apg_euler(const float* out, float* acc, int Bi, int C, int H, int W, int P, float g, float thr, float dt,
              hipStream_t s) {
  hipLaunchKernelGGL(apg_euler_kernel, dim3(1), dim3(1024), 0, s, out, acc, Bi, C, H, W, P, g, thr, dt);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int rows_uniform(const void* x, int cols, const int* cu, int nseq, int* bad, hipStream_t s) {
  FLITE_REQUIRE(cols % 2 == 0 && nseq > 0, "rows_uniform: bf16 rows of even width");
  hipLaunchKernelGGL(rows_uniform_kernel, dim3(nseq, 32), dim3(256), 0, s, (const unsigned*)x, (long)cols / 2, cu,
                     cols / 2, bad);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int ctx_bcast_resid(void* x, bool x16, const float* c, const float* gate, long gate_seg_stride, int rows_per_seg,
                    long rows, int D, hipStream_t s) {
  if (rows <= 0) return 0;
  FLITE_REQUIRE(D % 4 == 0, "ctx_bcast_resid: D must be a multiple of 4");
  if (x16)
    hipLaunchKernelGGL(ctx_bcast_resid_kernel<true>, dim3(grid_for(rows * (D / 4))), dim3(256), 0, s, x, c, gate,
                       gate_seg_stride, rows_per_seg, rows, D);
  else
    hipLaunchKernelGGL(ctx_bcast_resid_kernel<false>, dim3(grid_for(rows * (D / 4))), dim3(256), 0, s, x, c, gate,
                       gate_seg_stride, rows_per_seg, rows, D);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int apg_sums(const float* u, const float* c, long n, float k, int phase, float* out2, hipStream_t s) {
  FLITE_REQUIRE(phase == 0 || phase == 1, "apg_sums: phase must be 0 or 1");
  hipLaunchKernelGGL(apg_sums_kernel, dim3(1), dim3(1024), 0, s, u, c, n, k, phase, (const float*)nullptr, out2);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int apg_sums_dev(const float* u, const float* c, long n, int phase, float* ws4, hipStream_t s) {
  FLITE_REQUIRE(phase == 0 || phase == 1, "apg_sums_dev: phase must be 0 or 1");
  hipLaunchKernelGGL(apg_sums_kernel, dim3(1), dim3(1024), 0, s, u, c, n, 0.f, phase,
                     phase == 1 ? (const float*)ws4 : (const float*)nullptr, ws4 + 2 * phase);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int apg_update_nchw(const float* u, const float* c, float* acc, long n, float g, float k, float sc, float dt,
                    hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(apg_update_nchw_kernel, dim3(grid_for(n)), dim3(256), 0, s, u, c, acc, n, g, k, sc, dt,
                     (const float*)nullptr, 0L, 0.f);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int apg_update_nchw_dev(const float* u, const float* c, float* acc, long n, float g, float thr, long n_total,
                        const float* ws4, float dt, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(apg_update_nchw_kernel, dim3(grid_for(n)), dim3(256), 0, s, u, c, acc, n, g, 0.f, 1.f, dt, ws4,
                     n_total, thr);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int unpatchify(const float* out, void* y, bool out_bf16, int B, int C, int H, int W, int P, hipStream_t s) {
  const long total = (long)B * C * H * W;
  if (out_bf16)
    hipLaunchKernelGGL(unpatchify_kernel<true>, dim3(grid_for(total)), dim3(256), 0, s, out, y, B, C, H, W, P);
  else
    hipLaunchKernelGGL(unpatchify_kernel<false>, dim3(grid_for(total)), dim3(256), 0, s, out, y, B, C, H, W, P);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int timestep_embed(const float* t, bf16_t* emb, int n, int D, int quantize, hipStream_t s) {
  FLITE_REQUIRE(D % 2 == 0, "timestep_embed: D must be even");
  hipLaunchKernelGGL(timestep_embed_kernel, dim3(grid_for((long)n * D)), dim3(256), 0, s, t, emb, n, D, quantize);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

// [1 + hh + ww][64][2]: row 0 = (1, 0), rows 1 + y and 1 + hh + x = (cos, sin) of pos * inv_freq, rounded as
// rope_table does (RopeAxes, common.h)
__global__ __launch_bounds__(256) void rope_axes_kernel(const float* inv_freq, float* cs, int hh, int ww,
                                                        int round_bf16) {
  const int total = (1 + hh + ww) * 64;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const int row = idx / 64, j = idx % 64;
    float c = 1.f, s = 0.f;
    if (row > 0) {
      const float pos = (float)(row <= hh ? row - 1 : row - 1 - hh);
      const float a = pos * inv_freq[j];
      c = cosf(a);
      s = sinf(a);
      if (round_bf16) {
        c = bf2f(f2bf(c));
        s = bf2f(f2bf(s));
      }
    }
    cs[2 * idx] = c;
    cs[2 * idx + 1] = s;
  }
}

int rope_axes_table(const float* inv_freq, float* cs, int hh, int ww, int round_bf16, hipStream_t s) {
  FLITE_REQUIRE(hh > 0 && ww > 0, "rope_axes_table: empty grid");
  hipLaunchKernelGGL(rope_axes_kernel, dim3((unsigned)(((1 + hh + ww) * 64 + 255) / 256)), dim3(256), 0, s, inv_freq,
                     cs, hh, ww, round_bf16);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int rope_table(const float* inv_freq, float* cos_t, float* sin_t, int hh, int ww, int R, int round_bf16,
               hipStream_t s) {
  const long total = (long)(R + hh * ww) * 128;
  hipLaunchKernelGGL(rope_table_kernel, dim3(grid_for(total)), dim3(256), 0, s, inv_freq, cos_t, sin_t, hh, ww, R,
                     round_bf16);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int gather_rows(const bf16_t* src, bf16_t* dst, const int* idx, long n, int cols, hipStream_t s) {
  FLITE_REQUIRE(cols % 8 == 0, "gather_rows: cols must be a multiple of 8");
  if (n <= 0) return 0;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_for(n * cols / 8)), dim3(256), 0, s, src, dst, idx, n, cols);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace flite
