// Diagnostic build of the attention kernel with per-workgroup timeline stamps (FLITE_ATTN_STAMPS); not part of
// the product library. Built by f-lite_amd/tools/attn_probe.py into f-lite_amd/tools/attn_probe.so.
#define FLITE_ATTN_STAMPS 1
#include "../csrc/attention.hip"

namespace flite {
static std::string g_err;
void set_last_error(const std::string& msg) { g_err = msg; }
}  // namespace flite

extern "C" int attn_probe(void* stream, int T, int Lk, int H, const void* q, const void* k, const void* v, void* o,
                          const int* cu_q, const int* cu_k, void* ws, long ws_bytes, unsigned long long* stamps) {
  using namespace flite;
  AttnParams a;
  a.q = (const bf16_t*)q;
  a.k = (const bf16_t*)k;
  a.v = (const bf16_t*)v;
  a.o = (bf16_t*)o;
  a.q_row_stride = a.o_row_stride = (long)H * 256;
  a.k_row_stride = a.v_row_stride = (long)H * 256;
  a.q_head_stride = a.k_head_stride = a.v_head_stride = a.o_head_stride = 256;
  a.cu_q = cu_q;
  a.cu_k = cu_k;
  a.B = 2;
  a.H = H;
  a.head_dim = 256;
  a.max_q = T;
  a.max_k = Lk;
  a.scale = 1.f / 16.f;
  a.max_score = 16.5f;
  a.split_ws = ws;
  a.split_ws_bytes = ws_bytes;
  a.stamps = stamps;
  return attn_fwd(a, (hipStream_t)stream);
}
