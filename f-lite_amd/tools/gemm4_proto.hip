// Prototype (tools only, never shipped): bf16 GEMM C = A . W^T with 4 waves per 256x256 tile, each wave owning a
// 128x128 block of C (8x8 v_mfma_f32_16x16x32_bf16 accumulators = 256 registers, meant for the AGPR half of the
// register file at one wave per SIMD). Same LDS image, swizzle and LDS-DMA staging as gemm.hip; two barriers per
// 64-deep k-tile. Question it answers: does halving the waves (and cutting LDS fragment reads by a third) beat the
// product kernel's 8 x (128x64) layout on the DiT shapes? Build: tools/gemm4_bench.py.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "common.h"

using namespace flite;

namespace {

constexpr int BM = 256, BN = 256, BK = 64, NT = 256;
constexpr int TILE_BYTES = BM * BK * 2;
constexpr int W_REGION = 2 * TILE_BYTES;
constexpr int LDS_BYTES = 4 * TILE_BYTES;

typedef __attribute__((ext_vector_type(4))) int i32x4;

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ i32x4 make_rsrc(const void* base, unsigned bytes) {
  const unsigned long long a = (unsigned long long)base;
  i32x4 r;
  r.x = __builtin_amdgcn_readfirstlane((int)(a & 0xffffffffu));
  r.y = __builtin_amdgcn_readfirstlane((int)(a >> 32));
  r.z = __builtin_amdgcn_readfirstlane((int)bytes);
  r.w = 0x00020000;
  return r;
}

__device__ __forceinline__ unsigned lds_addr_of(const void* p) {
  return (unsigned)(unsigned long long)(const LDS_AS char*)p;
}

// one LDS-DMA piece (64 lanes x 16 B); skip != 0 (uniform) issues nothing
__device__ __forceinline__ void dma1(const i32x4& rs, unsigned so, unsigned voff, unsigned lds, unsigned skip) {
  unsigned keep;
  asm volatile(
      "s_cmp_eq_u32 %[skip], 0\n\t"
      "s_cbranch_scc0 .Lskip1_%=\n\t"
      "s_mov_b32 %[keep], m0\n\t"
      "s_mov_b32 m0, %[lds]\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %[v], %[rs], %[so] offen lds\n\t"
      "s_mov_b32 m0, %[keep]\n"
      ".Lskip1_%=:"
      : [keep] "=&s"(keep)
      : [skip] "s"(skip), [lds] "s"(lds), [rs] "s"(rs), [so] "s"(so), [v] "v"(voff)
      : "memory", "scc");
}

struct P {
  const bf16_t* A;
  const bf16_t* W;
  bf16_t* C;
  int M, N, K;
};

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

__device__ __forceinline__ void tile_origin(int L, int num_m, int num_n, int& m0, int& n0) {
  constexpr int GROUP = 6;
  const int group_size = GROUP * num_n;
  const int gid = L / group_size;
  const int first_m = gid * GROUP;
  const int gm = min(num_m - first_m, GROUP);
  const int rem = L - gid * group_size;
  m0 = (first_m + rem % gm) * BM;
  n0 = (rem / gm) * BN;
}

// MFMA with the accumulator pinned to AGPRs (hipcc otherwise moves the 256 accumulator registers between the
// register files at every basic-block edge). Operands come from ds_reads only (no VALU producer: no hazard nops).
__device__ __forceinline__ void mfma_acc(f32x4& acc, const bf16x8& w, const bf16x8& a) {
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(w), "v"(a));
}
// MFMA write -> v_accvgpr_read wait states for the last MFMAs of the loop (in-order issue: older ones are done)
__device__ __forceinline__ void acc_fence(f32x4 (&t)[8]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3"
               : "+a"(t[0]), "+a"(t[1]), "+a"(t[2]), "+a"(t[3]), "+a"(t[4]), "+a"(t[5]), "+a"(t[6]), "+a"(t[7]));
}
// s_waitcnt vmcnt(16) when `more` (the next tile's 16 copies are in flight behind the awaited ones), else vmcnt(0);
// branch inside the asm so the k-loop stays one basic block
__device__ __forceinline__ void wait_tile(unsigned more) {
  asm volatile(
      "s_cmp_eq_u32 %0, 0\n\t"
      "s_cbranch_scc1 .Lw0_%=\n\t"
      "s_waitcnt vmcnt(16)\n\t"
      "s_branch .Lw1_%=\n"
      ".Lw0_%=:\n\t"
      "s_waitcnt vmcnt(0)\n"
      ".Lw1_%=:" ::"s"(more)
      : "memory", "scc");
}

__global__ __launch_bounds__(NT, 1) void gemm4_kernel(P p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wave_m = wave >> 1, wave_n = wave & 1;
  const int lr = lane & 15, lk = lane >> 4;
  const unsigned lds0 = (unsigned)__builtin_amdgcn_readfirstlane((int)lds_addr_of(smem));
  const int num_m = (p.M + BM - 1) / BM, num_n = (p.N + BN - 1) / BN, nk = p.K / BK;
  int m0, n0;
  tile_origin(xcd_remap(blockIdx.x, gridDim.x), num_m, num_n, m0, n0);
  const i32x4 a_rs = make_rsrc(p.A, (unsigned)((long)p.M * p.K * 2));
  const i32x4 w_rs = make_rsrc(p.W, (unsigned)((long)p.N * p.K * 2));
  unsigned a_off[8], w_off[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = (wave * 8 + i) * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ swz(row);
    a_off[i] = (unsigned)(((long)min(m0 + row, p.M - 1) * p.K + chunk * 8) * 2);
    w_off[i] = (unsigned)(((long)min(n0 + row, p.N - 1) * p.K + chunk * 8) * 2);
  }
  unsigned ab[2], wb[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const unsigned coff = ((4 * s + lk) ^ swz(lr)) << 4;
    ab[s] = lds0 + (wave_m * 128 + lr) * 128 + coff;
    wb[s] = lds0 + W_REGION + (wave_n * 128 + lr) * 128 + coff;
  }
  auto dma = [&](int kt, int buf, int q) {  // piece q: 0..7 A, 8..15 W
    const unsigned skip = (unsigned)__builtin_amdgcn_readfirstlane(kt >= nk ? 1 : 0);
    const unsigned so = (unsigned)__builtin_amdgcn_readfirstlane(kt * BK * 2);
    if (q < 8)
      dma1(a_rs, so, a_off[q], lds0 + buf * TILE_BYTES + (wave * 8 + q) * 1024, skip);
    else
      dma1(w_rs, so, w_off[q - 8], lds0 + W_REGION + buf * TILE_BYTES + (wave * 8 + q - 8) * 1024, skip);
  };
  auto rd = [&](unsigned base) { return *(const LDS_AS bf16x8*)(base); };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int q = 0; q < 16; ++q) dma(0, 0, q);
#pragma unroll
  for (int q = 0; q < 16; ++q) dma(1, 1, q);
  if (nk > 1)
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  bf16x8 ca[8], cw[8], na[8], nw[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    ca[i] = rd(ab[0] + i * 2048);
    cw[i] = rd(wb[0] + i * 2048);
  }

  auto group = [&](const bf16x8(&a)[8], const bf16x8(&w)[8], int g) {
    const int mi = g >> 1, nb = (g & 1) * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) mfma_acc(acc[mi][nb + j], w[nb + j], a[mi]);
  };

  // one 64-deep k-tile from buffer BUF: step 0 = MFMA(ca, cw) | read step 1 (na, nw); B1; step 1 first half =
  // MFMA(na, nw) | DMA tile kt + 2 into BUF; B2 (tile kt + 1 landed); second half | read step 0 of kt + 1
  auto ktile2 = [&](auto buf_, int kt) {
    constexpr int BUF = decltype(buf_)::value;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      group(ca, cw, g);
      if (g < 8)
        na[g] = rd(ab[1] + BUF * TILE_BYTES + g * 2048);
      else
        nw[g - 8] = rd(wb[1] + BUF * TILE_BYTES + (g - 8) * 2048);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      group(na, nw, g);
      __builtin_amdgcn_sched_barrier(0);
      dma(kt + 2, BUF, 2 * g);
      dma(kt + 2, BUF, 2 * g + 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    wait_tile((unsigned)__builtin_amdgcn_readfirstlane(kt + 2 < nk ? 1 : 0));
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int g = 8; g < 16; ++g) {
      group(na, nw, g);
      const int q = 2 * (g - 8);  // two reads per group: A and W fragment (g - 8)
      ca[q >> 1] = rd(ab[0] + (BUF ^ 1) * TILE_BYTES + (q >> 1) * 2048);
      cw[q >> 1] = rd(wb[0] + (BUF ^ 1) * TILE_BYTES + (q >> 1) * 2048);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    ktile2(I0{}, kt);
    ktile2(I1{}, kt + 1);
  }
  if (kt < nk) ktile2(I0{}, kt);
  acc_fence(acc[7]);

  // store bf16: lane holds C[m][n..n+3], m = m0 + wave_m*128 + mi*16 + lr, n = n0 + wave_n*128 + ni*16 + lk*4
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
    const int m = m0 + wave_m * 128 + mi * 16 + lr;
    if (m >= p.M) continue;
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) {
      const int n = n0 + wave_n * 128 + ni * 16 + lk * 4;
      if (n >= p.N) continue;
      u32x2 v;
      v.x = pack2bf(acc[mi][ni][0], acc[mi][ni][1]);
      v.y = pack2bf(acc[mi][ni][2], acc[mi][ni][3]);
      *(u32x2*)(p.C + (long)m * p.N + n) = v;
    }
  }
}

}  // namespace

extern "C" int gemm4_proto(const void* A, const void* W, void* C, int M, int N, int K, void* stream) {
  if (K % BK || N % 4) return 2;
  static bool init = false;
  if (!init) {
    if (hipFuncSetAttribute((const void*)gemm4_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES))
      return 1;
    init = true;
  }
  P p{(const bf16_t*)A, (const bf16_t*)W, (bf16_t*)C, M, N, K};
  const int T = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL(gemm4_kernel, dim3(T), dim3(NT), LDS_BYTES, (hipStream_t)stream, p);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
