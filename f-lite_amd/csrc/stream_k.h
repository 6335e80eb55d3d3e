// Tile scheduling shared by the bf16 (gemm.hip) and MXFP8 (gemm_fp8.hip) GEMMs: XCD-aware block remap, grouped
// raster, and the stream-K + data-parallel persistent schedule with its launch-time cost model.
#pragma once
#include <algorithm>

#include "common.h"

namespace flite {
namespace sk {

// blockIdx -> XCD-contiguous index (bijective; the dispatcher places block b on XCD b % 8)
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// linear tile id -> (m0, n0): groups of 6 M-tiles, M-fastest inside a group (L2 reuse of W columns)
__device__ __forceinline__ void tile_origin(int L, int num_m, int num_n, int& m0, int& n0, int bm, int bn) {
  constexpr int GROUP = 6;  // kbench_gemm A/B on MI355X: 4-6 beat 8 by 1.5-2.5 % (gate/up, 8192^3), 2 and 16 lose
  const int group_size = GROUP * num_n;
  const int gid = L / group_size;
  const int first_m = gid * GROUP;
  const int gm = min(num_m - first_m, GROUP);
  const int rem = L - gid * group_size;
  m0 = (first_m + rem % gm) * bm;
  n0 = (rem / gm) * bn;
}

__device__ __forceinline__ long sk_start(int g, long I, int G) { return (long)g * I / G; }

// Stream-K + data-parallel (persistent grid G = one workgroup per CU) over 256x256 tiles. Tiles [0, sk_tiles)
// are cut into Gs contiguous, equal ranges of k-tile iterations (I / Gs < nk, so a range touches at most 2
// tiles); the remaining tiles are data parallel. A range's segment that ends inside its tile is a PARTIAL:
// written to workspace slot wg (fp32, lane-linear) and published with a flag. The segment that ends a tile
// FINISHES it: adds the partials of the lower-index workgroups that own the tile's earlier segments, in a fixed
// order, then runs the epilogue. Order per workgroup: data-parallel tiles, partial, finisher -- producers
// publish before any wait, so every wait is on work that never waits (no cycle).
// Cta: setup_tile(m0, n0), mainloop(acc, kb, kend), epilogue(acc, m0, n0), tid, p.{sk_ws, sk_flags, sk_tiles,
// sk_wgs}; NT threads, acc[8][4] per lane.
template <int NT, class Cta>
__device__ __forceinline__ void stream_k_body(Cta& c, f32x4 (&acc)[8][4], int num_m, int num_n, int nk, int wg) {
  constexpr int TILE = 256;
  int m0, n0;
  const int G = gridDim.x;
  const int Gs = c.p.sk_wgs;  // workgroups [0, Gs) share the stream-K iterations
  const int T = num_m * num_n;
  const long I = (long)c.p.sk_tiles * nk;
  const long it0 = wg < Gs ? sk_start(wg, I, Gs) : I, it1 = wg < Gs ? sk_start(wg + 1, I, Gs) : I;
  const int jf = (int)(it0 / nk);        // tile of the first segment
  const int jl = (int)((it1 - 1) / nk);  // tile of the last segment
  const bool has_range = it1 > it0;
  f32x4* slab = (f32x4*)c.p.sk_ws;
  int* flags = c.p.sk_flags;

  // (1) data-parallel tiles: every workgroup in step, so the XCD-local tile block shares A/W k-slices in L2
  for (int L = c.p.sk_tiles + wg; L < T; L += G) {
    tile_origin(L, num_m, num_n, m0, n0, TILE, TILE);
    c.setup_tile(m0, n0);
    c.mainloop(acc, 0, nk);
    c.epilogue(acc, m0, n0);
  }
  // (2) partial: the last segment when it does not reach its tile's end
  if (has_range) {
    const long t0 = (long)jl * nk;
    const int kb = (int)(max(it0, t0) - t0), kend = (int)(it1 - t0);
    if (kend < nk) {
      tile_origin(jl, num_m, num_n, m0, n0, TILE, TILE);
      c.setup_tile(m0, n0);
      c.mainloop(acc, kb, kend);
      // publish (MI355X guide §6 G16, R1): write-through (sc1) payload stores drained by every wave, then
      // one relaxed agent-scope flag store -- no release fence (it would write back the XCD's whole L2)
      const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(slab + (size_t)wg * (TILE * TILE / 4)), (short)0, TILE * TILE * 4, 0x00020000);
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[mi][ni]), srs,
                                                 ((mi * 4 + ni) * NT + c.tid) * 16, 0, 16 /* sc1 */);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (c.tid == 0) __hip_atomic_store(flags + wg, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // (3) finisher: the first segment when it reaches its tile's end
  if (has_range) {
    const long t0 = (long)jf * nk;
    const int kb = (int)(it0 - t0), kend = (int)(min(it1, t0 + nk) - t0);
    if (kend == nk) {
      tile_origin(jf, num_m, num_n, m0, n0, TILE, TILE);
      c.setup_tile(m0, n0);
      c.mainloop(acc, kb, kend);
      if (kb > 0) {
        // producers: workgroups h < wg whose range ends inside this tile
        int h_lo = wg;
        while (h_lo > 0 && sk_start(h_lo, I, Gs) > t0) --h_lo;
        if (c.tid == 0) {
          for (int h = h_lo; h < wg; ++h) {
            if (sk_start(h + 1, I, Gs) == sk_start(h, I, Gs)) continue;  // empty range: no partial
            long spins = 0;
            while (__hip_atomic_load(flags + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
              __builtin_amdgcn_s_sleep(2);
              if (++spins > (1L << 28)) __builtin_trap();  // never expected: all G workgroups are resident
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        for (int h = h_lo; h < wg; ++h) {
          if (sk_start(h + 1, I, Gs) == sk_start(h, I, Gs)) continue;
          const f32x4* src = slab + (size_t)h * (TILE * TILE / 4);
#pragma unroll
          for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) acc[mi][ni] += src[(mi * 4 + ni) * NT + c.tid];
        }
        __syncthreads();
        if (c.tid == 0)
          for (int h = h_lo; h < wg; ++h) __hip_atomic_store(flags + h, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      c.epilogue(acc, m0, n0);
    }
  }
}

// Stream-K split for a workspace-carrying launch of T 256x256 tiles on G resident workgroups, in units of one
// k-tile iteration of one workgroup (nk per tile):
//   data parallel  ceil(T / G) * nk
//   stream-K       floor(T / G) * nk + 1.1 * rem * nk / Gs + 24 + 5.5 * (ceil(Gs / rem) - 1)
// over Gs workgroups sharing the rem = T % G leftover tiles. The 1.1 and 24 (partial-slab write/read, two extra
// pipeline prologues, finisher epilogue) are fitted to round-1 timelines of the bf16 GEMM on MI355X (M = 8224,
// N = 3072: stream-K wins at K = 12288 (-11 %), loses at K = 3072 (+6 %)); 5.5 per extra partial a finisher adds
// is fitted to M = 16448, N = 3072 (12 leftover tiles cut 22 ways cost +230 us over the first two terms). An
// MXFP8 k-tile (128 deep) costs the same MFMA cycles and bytes as a bf16 one (64 deep), so the model carries
// over. Returns the tile count and sets *gs; taken only with a 3 % margin.
inline int choose_sk_tiles(int T, int nk_tiles, int G, int* gs) {
  *gs = 0;
  if (G <= 0) return 0;
  const int rem = T % G;
  if (rem == 0) return 0;
  const double nk = nk_tiles;
  const double dp = (double)(T / G + 1) * nk;
  double best = 0.97 * dp;
  for (int f = 2;; ++f) {  // Gs = f * rem: each leftover tile cut into about f ranges
    const int Gs = std::min(G, f * rem);
    if (rem * nk < 2.0 * Gs) break;  // ranges of at least 2 k-tiles
    const int fan = (Gs + rem - 1) / rem;
    const double sk = (double)(T / G) * nk + 1.1 * rem * nk / Gs + 24.0 + 5.5 * (fan - 1);
    if (sk < best) {
      best = sk;
      *gs = Gs;
    }
    if (Gs == G) break;
  }
  return *gs ? rem : 0;
}

}  // namespace sk
}  // namespace flite
