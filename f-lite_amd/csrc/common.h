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
