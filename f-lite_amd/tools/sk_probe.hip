// Diagnostic build of the GEMM with per-workgroup stream-K phase stamps (FLITE_SK_STAMPS); not part of the
// product library. Built by f-lite_amd/tools/sk_probe.py into f-lite_amd/tools/sk_probe.so.
#define FLITE_SK_STAMPS 1
#include "../csrc/gemm.hip"

namespace flite {
static std::string g_err;
void set_last_error(const std::string& msg) { g_err = msg; }
}  // namespace flite

extern "C" int sk_probe_gemm(void* stream, int M, int N, int K, const void* A, const void* W, void* out,
                             void* workspace, unsigned long long* stamps) {
  using namespace flite;
  GemmParams p;
  p.A = (const bf16_t*)A;
  p.lda = K;
  p.W = (const bf16_t*)W;
  p.ldw = K;
  p.out = out;
  p.ldo = N;
  p.M = M;
  p.N = N;
  p.K = K;
  const int G = gemm_sk_workspace_cus();
  if (workspace) {
    p.sk_ws = (float*)workspace;
    p.sk_flags = (int*)((char*)workspace + (size_t)G * 256 * 256 * 4);
  }
  p.sk_stamps = stamps;
  return gemm_bf16(p, EPI_STORE_F32, (hipStream_t)stream);
}
