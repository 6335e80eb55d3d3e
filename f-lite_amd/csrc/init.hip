// Deterministic synthetic parameters/inputs on the device (counter-based splitmix64 hash).
// Bit-identical to the CPU generator used by the oracle (oracle/weights.py): weights are never shipped,
// both sides regenerate them from (seed, parameter name, element index).
#include "common.h"
#include "kernels.h"

namespace flite {

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <bool OUT_BF16>
__global__ __launch_bounds__(256) void hash_uniform_kernel(void* out, long n, uint64_t base, float scale) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t bits = splitmix64(base + (uint64_t)i);
    const long s = (long)(bits >> 40) - (1L << 23);
    const float v = (float)(2 * s + 1) * scale;
    if constexpr (OUT_BF16)
      ((bf16_t*)out)[i] = f2bf(v);
    else
      ((float*)out)[i] = v;
  }
}

__global__ __launch_bounds__(256) void fill_kernel(bf16_t* out, long n, bf16_t v) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = v;
}

uint64_t host_splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

}  // namespace

uint64_t fnv1a64(const char* s) {
  uint64_t h = 0xCBF29CE484222325ull;
  for (; *s; ++s) {
    h ^= (unsigned char)*s;
    h *= 0x100000001B3ull;
  }
  return h;
}

int hash_init(void* out, int out_bf16, long n, const char* name, uint64_t seed, double std, hipStream_t s) {
  if (n <= 0) return 0;
  const uint64_t base = host_splitmix64(seed ^ fnv1a64(name));
  const float scale = (float)(std * 1.7320508075688772 / 16777216.0);
  long grid = (n + 255) / 256;
  if (grid > 16384) grid = 16384;
  if (out_bf16)
    hipLaunchKernelGGL(hash_uniform_kernel<true>, dim3((unsigned)grid), dim3(256), 0, s, out, n, base, scale);
  else
    hipLaunchKernelGGL(hash_uniform_kernel<false>, dim3((unsigned)grid), dim3(256), 0, s, out, n, base, scale);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

int fill_bf16(bf16_t* out, long n, float v, hipStream_t s) {
  if (n <= 0) return 0;
  long grid = (n + 255) / 256;
  if (grid > 16384) grid = 16384;
  const float vv = v;
  const uint32_t u = *(const uint32_t*)&vv;
  const bf16_t h = (bf16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
  hipLaunchKernelGGL(fill_kernel, dim3((unsigned)grid), dim3(256), 0, s, out, n, h);
  FLITE_HIP_CHECK(hipGetLastError());
  return 0;
}

}  // namespace flite
