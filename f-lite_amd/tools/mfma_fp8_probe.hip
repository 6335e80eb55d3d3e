// Probe of the gfx950 block-scaled fp8 MFMA (v_mfma_scale_f32_16x16x128_f8f6f4) operand / scale lane maps.
// One wave: D[16x16] = sum_k A_l(bytes) * B_l(bytes) under the hardware's lane maps; the host (mfma_fp8_probe.py)
// tests layout hypotheses against exact small-integer data. Diagnostic tool, not part of libflite_hip.so.
#include <hip/hip_runtime.h>

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__global__ void probe_kernel(const int* a, const int* b, const int* sa, const int* sb, float* d) {
  const int l = threadIdx.x;
  i32x8 av, bv;
  for (int i = 0; i < 8; ++i) {
    av[i] = a[l * 8 + i];
    bv[i] = b[l * 8 + i];
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, acc, 0, 0, 0, sa[l], 0, sb[l]);
  for (int r = 0; r < 4; ++r) d[l * 4 + r] = acc[r];
}

extern "C" int mfma_fp8_probe(const int* a, const int* b, const int* sa, const int* sb, float* d) {
  hipLaunchKernelGGL(probe_kernel, dim3(1), dim3(64), 0, 0, a, b, sa, sb, d);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
