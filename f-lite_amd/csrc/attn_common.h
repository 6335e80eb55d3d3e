// Device helpers shared by the gfx950 flash-attention kernels (attention.hip: 128 query rows per workgroup;
// attention_q256.hip: 256). CDNA4 only: 64-lane waves, v_mfma_f32_32x32x16_bf16, LDS-DMA, ds_read_b64_tr_b16.
#pragma once
#include "common.h"

namespace flite {
namespace {

__device__ __forceinline__ s16x4 ds_tr16(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(p));
}

typedef __attribute__((ext_vector_type(4))) int i32x4;

// Buffer descriptor (raw, stride 0) from wave-uniform values (readfirstlane makes uniformity provable).
__device__ __forceinline__ i32x4 make_rsrc(const void* base, unsigned bytes) {
  const unsigned long long a = (unsigned long long)base;
  i32x4 r;
  r.x = __builtin_amdgcn_readfirstlane((int)(a & 0xffffffffu));
  r.y = __builtin_amdgcn_readfirstlane((int)(a >> 32));
  r.z = __builtin_amdgcn_readfirstlane((int)bytes);
  r.w = 0x00020000;
  return r;
}

// 16-B-per-lane LDS-DMA: LDS[m0 + lane*16] = buffer[voff] (0 when voff is out of range). Inline asm on
// purpose: hipcc counts a builtin LDS-DMA in vmcnt and then waits for it (vmcnt(0)) before every later
// ds_read, serialising the next tile's prefetch with this tile's compute; the waits are placed by hand
// (vmcnt(0) + barrier at the end of each tile).
__device__ __forceinline__ void blds16(const i32x4& rsrc, unsigned voff, unsigned lds_addr) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rsrc), "s"(__builtin_amdgcn_readfirstlane(lds_addr))
      : "memory");
}

// O^T += V^T . P^T with the accumulator pinned to AGPRs. Left to itself hipcc keeps O (128 registers per lane)
// in VGPRs inside the key loop and copies it to and from AGPRs every tile (~300 v_accvgpr moves per tile,
// an issue-bound loop). An MFMA reads its srcC from AGPRs directly. The asm is opaque to the hazard
// recognizer, so the VALU write -> MFMA srcA/B read distance of the P operand must hold by construction. Both
// kernels use only the no-NOP form, under this invariant: every P register is written by the softmax VALU before
// a workgroup barrier or a sched_barrier(0)-fenced block of at least VAHEAD transposed V reads (two ds_read each;
// VAHEAD >= 1 is static_asserted at each kernel), all issued before the first PV MFMA that reads it. In the key
// loop a whole phase A (32 MFMAs) also lies in between; on the last tile (no phase A) and on the single-tile path
// (prologue softmax, barrier, phase B) the barrier and the read-ahead block alone provide the distance. Every
// reader of O after the loop waits behind o_acc_fence() (MFMA write -> read). The NOP form (`s_nop 1`, and a
// "+v" pk that orders later readers after it) is kept for a P produced right before its MFMA.
template <bool NOP>
__device__ __forceinline__ void mfma_o(f32x16& acc, const bf16x8& v, bf16x8& pk) {
  if constexpr (NOP)
    asm("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %2, %1, %0" : "+a"(acc), "+v"(pk) : "v"(v));
  else
    asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(v), "v"(pk));
}
// S^T = K . Q^T with Q^T pinned to AGPRs (loop-invariant; hipcc otherwise shuttles it between the register files
// every tile) and S in VGPRs for the softmax VALU.
__device__ __forceinline__ void mfma_s_first(f32x16& acc, const bf16x8& k, const bf16x8& q) {
  asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(k), "a"(q));
}
__device__ __forceinline__ void mfma_s(f32x16& acc, const bf16x8& k, const bf16x8& q) {
  asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(k), "a"(q));
}
// Wait states between an asm MFMA's write and a VALU / v_accvgpr read of its result (XDL 32x32: 18). The
// fence "redefines" the results, so no reader can be scheduled above it.
__device__ __forceinline__ void mfma_read_fence(f32x16& a, f32x16& b) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ void o_acc_fence(f32x16 (&o)[8]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3"
               : "+a"(o[0]), "+a"(o[1]), "+a"(o[2]), "+a"(o[3]), "+a"(o[4]), "+a"(o[5]), "+a"(o[6]), "+a"(o[7]));
}

__device__ __forceinline__ unsigned lds_addr_of(const void* p) {
  return (unsigned)(unsigned long long)(const LDS_AS char*)p;
}

// blockIdx -> XCD-contiguous index (bijective; the dispatcher deals blocks round-robin over the 8 XCDs)
__device__ __forceinline__ int xcd_remap(int bid, int n) {
  const int xcd = bid & 7, q8 = n >> 3, r8 = n & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
}

// S^T = K . Q^T with Q^T in VGPRs (the 256-row kernel: its O accumulators take all 256 AGPRs)
__device__ __forceinline__ void mfma_sv_first(f32x16& acc, const bf16x8& k, const bf16x8& q) {
  asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(k), "v"(q));
}
__device__ __forceinline__ void mfma_sv(f32x16& acc, const bf16x8& k, const bf16x8& q) {
  asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(k), "v"(q));
}

}  // namespace
}  // namespace flite
