// T5 encoder launchers (t5.hip). Host side; not part of the C ABI.
#pragma once
#include "common.h"

namespace flite {

struct T5AttnParams {
  const bf16_t* q = nullptr;  // [B*L, >= H*64] rows (head h at column h*64)
  const bf16_t* k = nullptr;
  const bf16_t* v = nullptr;
  bf16_t* o = nullptr;
  long ldq = 0, ldk = 0, ldv = 0, ldo = 0;  // row strides (elements)
  const int* bucket = nullptr;         // int32 [2L-1]: relative-position bucket of (key - query) + L - 1
  const bf16_t* rel_weight = nullptr;  // relative_attention_bias.weight [num_buckets, H] (bf16)
  const float* mask = nullptr;         // additive key mask [B, L] (0 / -inf) or null
  int B = 0, L = 0, H = 0;
};

int t5_attention(const T5AttnParams& p, hipStream_t s);
int embed_rows_f32(const bf16_t* table, const int* ids, float* out, long n, int cols, long vocab, hipStream_t s);

}  // namespace flite
