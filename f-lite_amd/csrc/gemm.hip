// bf16 MFMA GEMM for gfx950 with fused epilogues.
//
//   C[M,N] = A[M,K] . W[N,K]^T (+ bias[N])           -- nn.Linear layout: both operands K-contiguous
//
// Replaces every nn.Linear on the DiT hot path (reference f_lite/model.py:151-156 qkv/q/context_kv/proj,
// model.py:261-267 LigerSwiGLUMLP gate/up/down, model.py:436 context_proj, model.py:448-456 time/adaLN,
// model.py:475 final_proj) and the patch-embed Conv2d (model.py:321, k=s=2 == GEMM over 64-vectors).
//
// Tile 256x256x64, 512 threads = 8 waves laid out 2(M) x 4(N), each wave owns 128x64 of C.
// Operands are staged HBM->LDS with global_load_lds (16 B/lane, lane-linear LDS image), double-buffered;
// the bank-conflict XOR swizzle is applied on the per-lane SOURCE address and undone on the ds_read.
// MFMA v_mfma_f32_16x16x32_bf16 is issued with W as the "A" operand and the activations as "B", so each
// lane's accumulator holds 4 consecutive output COLUMNS of one output row: the epilogue stores 8/16 B
// contiguous per lane and fused row-wise epilogues (gate, SwiGLU pairs) need no shuffles.
#include "common.h"
#include "kernels.h"

namespace flite {

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int NT = 512;
constexpr int TILE_BYTES = BM * BK * 2;          // 32 KiB per operand tile
constexpr int STAGE_BYTES = 2 * TILE_BYTES;      // A + W
constexpr int LDS_BYTES = 2 * STAGE_BYTES;       // double buffer = 128 KiB

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ void glds16(const void* gsrc, void* ldst) {
  __builtin_amdgcn_global_load_lds((const GLB_AS void*)gsrc, (LDS_AS void*)ldst, 16, 0, 0);
}

__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t r, unsigned voff, void* ldst) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS_AS void*)ldst, 16, voff, 0, 0, 0);
}

// CONV = implicit-GEMM 3x3 convolution (pad 1) over an NHWC bf16 input: A row m = output pixel, k = (tap, c)
// with tap = ky*3+kx. Each 64-wide k-tile is one tap and 64 consecutive channels (128 contiguous bytes of
// one input pixel) -> staged by buffer_load ... lds, whose range check returns 0 for the padding pixels.
// `upsample` folds nearest-2x interpolation into the addressing (Upsample2D + conv).
template <int EPI, bool CONV>
__global__ __launch_bounds__(NT, 2) void gemm_bf16_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wave_m = wave >> 2;  // 0..1
  const int wave_n = wave & 3;   // 0..3

  // ---- tile scheduling: XCD-aware bijective remap, then grouped (M-fastest) ordering ----
  const int num_m = (p.M + BM - 1) / BM;
  const int num_n = (p.N + BN - 1) / BN;
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  int wg;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  constexpr int GROUP = 8;
  const int group_size = GROUP * num_n;
  const int gid = wg / group_size;
  const int first_m = gid * GROUP;
  const int gm = min(num_m - first_m, GROUP);
  const int rem = wg - gid * group_size;
  const int tile_m = first_m + rem % gm;
  const int tile_n = rem / gm;
  const int m0 = tile_m * BM;
  const int n0 = tile_n * BN;

  // ---- per-lane staging sources (4 rows of A and 4 rows of W per wave per k-tile) ----
  // glds instruction q (0..31) covers tile rows 8q..8q+7; lane -> row 8q + lane/8, 16-B chunk (lane&7)^swz.
  const bf16_t* a_src[4];
  const bf16_t* w_src[4];
  int cy[4], cx[4];
  unsigned cbase[4];  // element offset of (batch, chunk) for CONV
  __amdgpu_buffer_rsrc_t crs;
  if constexpr (CONV) crs = __builtin_amdgcn_make_buffer_rsrc((void*)p.conv_in, 0, (int)p.conv_in_bytes, 0x00020000);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = wave * 4 + i;
    const int row = q * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ swz(row);
    const int am = min(m0 + row, p.M - 1);
    if constexpr (CONV) {
      const int hw = p.conv_oh * p.conv_ow;
      const int b = am / hw;
      const int r = am - b * hw;
      cy[i] = r / p.conv_ow;
      cx[i] = r - cy[i] * p.conv_ow;
      cbase[i] = (unsigned)((long)b * p.conv_ih * p.conv_iw * p.conv_c + chunk * 8);
      a_src[i] = nullptr;
    } else {
      a_src[i] = p.A + (long)am * p.lda + chunk * 8;
    }
    const int wn = min(n0 + row, p.N - 1);
    const bf16_t* wbase;
    long wrow;
    if constexpr (EPI == EPI_SWIGLU_BF16) {
      // virtual row wn: 16-row sub-tiles alternate gate (W) / up (W2) rows of the same output columns
      const int sub = wn >> 4;
      wrow = (long)(sub >> 1) * 16 + (wn & 15);
      wbase = (sub & 1) ? p.W2 : p.W;
    } else {
      wrow = wn;
      wbase = p.W;
    }
    w_src[i] = wbase + wrow * p.ldw + chunk * 8;
  }

  auto stage = [&](int kt, int buf) {
    char* base = smem + buf * STAGE_BYTES;
    const int koff = kt * BK;
    if constexpr (CONV) {
      const int tap = koff / p.conv_c;
      const int c0 = koff - tap * p.conv_c;
      const int ky = tap / 3 - 1, kx = tap % 3 - 1;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = wave * 4 + i;
        const int iy = cy[i] + ky, ix = cx[i] + kx;
        const bool ok = iy >= 0 && iy < p.conv_oh && ix >= 0 && ix < p.conv_ow;
        const int sy = p.conv_up ? (iy >> 1) : iy;
        const int sx = p.conv_up ? (ix >> 1) : ix;
        const unsigned e = cbase[i] + (unsigned)((sy * p.conv_iw + sx) * p.conv_c + c0);
        blds16(crs, ok ? e * 2u : 0x80000000u, base + q * 1024);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = wave * 4 + i;
        glds16(a_src[i] + koff, base + q * 1024);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = wave * 4 + i;
      glds16(w_src[i] + koff, base + TILE_BYTES + q * 1024);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / BK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // per-lane LDS read offsets (row = base16 + (lane&15); chunk = kk*4 + (lane>>4), swizzled)
  const int lr = lane & 15;
  const int lsw = (lr >> 1) & 7;
  const int lk = lane >> 4;

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    const char* As = smem + cur * STAGE_BYTES;
    const char* Ws = As + TILE_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int coff = (((kk * 4 + lk) ^ lsw) << 4);
      bf16x8 wf[4], af[8];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int row = wave_n * 64 + ni * 16 + lr;
        wf[ni] = *(const bf16x8*)(Ws + row * 128 + coff);
      }
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) {
        const int row = wave_m * 128 + mi * 16 + lr;
        af[mi] = *(const bf16x8*)(As + row * 128 + coff);
      }
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ni], af[mi], acc[mi][ni], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: lane holds C[m][n..n+3] for m = m_base + mi*16 + (lane&15), n = n_base + ni*16 + 4*(lane>>4)
  const int m_base = m0 + wave_m * 128 + lr;
  const int n_base = n0 + wave_n * 64 + lk * 4;

  if constexpr (EPI == EPI_SWIGLU_BF16) {
    // pairs (ni=0 gate, ni=1 up), (ni=2 gate, ni=3 up) -> output column (n0/2 + wave_n*32 + pair*16 + 4*(lane>>4))
    const int F = p.N >> 1;
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      const int m = m_base + mi * 16;
      if (m >= p.M) continue;
      bf16_t* orow = (bf16_t*)p.out + (long)m * p.ldo;
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int oc = (n0 >> 1) + wave_n * 32 + pr * 16 + lk * 4;
        if (oc >= F) continue;
        const f32x4 g = acc[mi][2 * pr];
        const f32x4 u = acc[mi][2 * pr + 1];
        u32x2 v;
        v.x = pack2bf(silu_f(g[0]) * u[0], silu_f(g[1]) * u[1]);
        v.y = pack2bf(silu_f(g[2]) * u[2], silu_f(g[3]) * u[3]);
        *(u32x2*)(orow + oc) = v;
      }
    }
    return;
  } else {
    float bias[4][4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n_base + ni * 16 + r;
        bias[ni][r] = (p.bias != nullptr && n < p.N) ? bf2f(p.bias[n]) : 0.f;
      }
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      const int m = m_base + mi * 16;
      if (m >= p.M) continue;
      const long om = p.out_seg > 0 ? (m / p.out_seg) * p.out_seg_stride + p.out_seg_off + (m % p.out_seg) : m;
      const float* grow = nullptr;
      if constexpr (EPI == EPI_RESID_F32) {
        if (p.gate != nullptr) grow = p.gate + (long)(m / p.rows_per_seg) * p.gate_seg_stride;
      }
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int n = n_base + ni * 16;
        if (n >= p.N) continue;
        f32x4 v = acc[mi][ni];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += bias[ni][r];
        if (p.act == 1) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = silu_f(v[r]);
        }
        if constexpr (EPI == EPI_STORE_BF16) {
          bf16_t* o = (bf16_t*)p.out + om * p.ldo + n;
          if (p.resid != nullptr) {  // ResnetBlock2D / attention residual (x + h), same layout as out
            const bf16_t* rr = p.resid + om * p.ldo + n;
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (n + r < p.N) v[r] += bf2f(rr[r]);
          }
          if (n + 3 < p.N) {
            u32x2 w;
            w.x = pack2bf(v[0], v[1]);
            w.y = pack2bf(v[2], v[3]);
            *(u32x2*)o = w;
          } else {
            for (int r = 0; r < 4 && n + r < p.N; ++r) o[r] = f2bf(v[r]);
          }
        } else if constexpr (EPI == EPI_STORE_F32) {
          float* o = (float*)p.out + om * p.ldo + n;
          if (n + 3 < p.N) {
            *(f32x4*)o = v;
          } else {
            for (int r = 0; r < 4 && n + r < p.N; ++r) o[r] = v[r];
          }
        } else if constexpr (EPI == EPI_RESID_F32) {
          float* o = (float*)p.out + om * p.ldo + n;
          f32x4 x = *(f32x4*)o;
          if (grow != nullptr) {
            const f32x4 g = *(const f32x4*)(grow + n);
#pragma unroll
            for (int r = 0; r < 4; ++r) x[r] += v[r] * g[r];
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) x[r] += v[r];
          }
          *(f32x4*)o = x;
        }
      }
    }
  }
}

template <int EPI>
int launch(const GemmParams& p, hipStream_t s) {
  const int num_m = (p.M + BM - 1) / BM;
  const int num_n = (p.N + BN - 1) / BN;
  const int grid = num_m * num_n;
  if (p.conv_in != nullptr)
    hipLaunchKernelGGL((gemm_bf16_kernel<EPI, true>), dim3(grid), dim3(NT), LDS_BYTES, s, p);
  else
    hipLaunchKernelGGL((gemm_bf16_kernel<EPI, false>), dim3(grid), dim3(NT), LDS_BYTES, s, p);
  return 0;
}

bool attrs_done = false;

template <int EPI>
hipError_t set_attrs() {
  hipError_t e = hipFuncSetAttribute((const void*)gemm_bf16_kernel<EPI, false>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute((const void*)gemm_bf16_kernel<EPI, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             LDS_BYTES);
}

}  // namespace

int gemm_init() {
  if (attrs_done) return 0;
  FLITE_HIP_CHECK(set_attrs<EPI_STORE_BF16>());
  FLITE_HIP_CHECK(set_attrs<EPI_STORE_F32>());
  FLITE_HIP_CHECK(set_attrs<EPI_RESID_F32>());
  FLITE_HIP_CHECK(set_attrs<EPI_SWIGLU_BF16>());
  attrs_done = true;
  return 0;
}

int gemm_bf16(const GemmParams& p, int epi, hipStream_t stream) {
  FLITE_REQUIRE(p.M > 0 && p.N > 0 && p.K > 0, "gemm: empty problem");
  FLITE_REQUIRE(p.K % BK == 0, "gemm: K must be a multiple of 64");
  FLITE_REQUIRE(p.ldw % 8 == 0, "gemm: ldw must be a multiple of 8 elements");
  FLITE_REQUIRE(((uintptr_t)p.W & 15) == 0, "gemm: W must be 16-B aligned");
  if (p.conv_in != nullptr) {
    FLITE_REQUIRE(p.conv_c % 64 == 0, "conv: input channels must be a multiple of 64");
    FLITE_REQUIRE(p.K == 9 * p.conv_c, "conv: K must be 9 * C_in");
    FLITE_REQUIRE(p.conv_oh == (p.conv_up ? 2 : 1) * p.conv_ih && p.conv_ow == (p.conv_up ? 2 : 1) * p.conv_iw,
                  "conv: output size must equal input size (x2 with upsample)");
    FLITE_REQUIRE(p.conv_in_bytes < (1L << 31), "conv: input must be < 2 GiB (32-bit buffer offsets)");
    FLITE_REQUIRE(epi == EPI_STORE_BF16 || epi == EPI_STORE_F32, "conv: store epilogues only");
  } else {
    FLITE_REQUIRE(p.lda % 8 == 0, "gemm: lda must be a multiple of 8 elements");
    FLITE_REQUIRE(((uintptr_t)p.A & 15) == 0, "gemm: A must be 16-B aligned");
  }
  if (gemm_init()) return 1;
  switch (epi) {
    case EPI_STORE_BF16:
      FLITE_REQUIRE(p.ldo % 4 == 0 || p.N < 4, "gemm: ldo must be a multiple of 4 (or N < 4)");
      launch<EPI_STORE_BF16>(p, stream);
      break;
    case EPI_STORE_F32:
      FLITE_REQUIRE(p.ldo % 4 == 0 || p.N < 4, "gemm: ldo must be a multiple of 4 (or N < 4)");
      launch<EPI_STORE_F32>(p, stream);
      break;
    case EPI_RESID_F32:
      FLITE_REQUIRE(p.N % 4 == 0 && p.ldo % 4 == 0, "gemm(resid): N, ldo must be multiples of 4");
      FLITE_REQUIRE(p.gate == nullptr || p.rows_per_seg > 0, "gemm(resid): rows_per_seg must be > 0");
      launch<EPI_RESID_F32>(p, stream);
      break;
    case EPI_SWIGLU_BF16:
      FLITE_REQUIRE(p.W2 != nullptr, "gemm(swiglu): up weight missing");
      FLITE_REQUIRE(p.N % 32 == 0, "gemm(swiglu): F must be a multiple of 16");
      FLITE_REQUIRE(p.bias == nullptr, "gemm(swiglu): bias not supported");
      launch<EPI_SWIGLU_BF16>(p, stream);
      break;
    default:
      FLITE_REQUIRE(false, "gemm: unknown epilogue");
  }
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace flite
