// Host-side validation of the C ABI, built with AddressSanitizer + UndefinedBehaviorSanitizer on the host code
// (tests/native/build_asan.sh; tests/test_capi_sanitizers.py runs it). No GPU is needed or touched: every call
// here must be refused by argument / bind validation BEFORE any device work, with status 2 and a message in
// flite_last_error(), and the sanitizers watch the string handling, the bind tables and the engine's
// bookkeeping while it happens. The DiT engine is constructed directly (flite_dit_create would first
// initialise the GEMM / attention kernels on a device).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "dit.h"

static int failures = 0;

#define EXPECT_ERR(call, substr)                                                                          \
  do {                                                                                                    \
    const int st_ = (call);                                                                               \
    const char* e_ = flite_last_error();                                                                  \
    if (st_ == 0 || e_ == nullptr || strstr(e_, substr) == nullptr) {                                     \
      fprintf(stderr, "FAIL %s:%d: %s -> status %d, error '%s' (want '%s')\n", __FILE__, __LINE__, #call, \
              st_, e_ ? e_ : "(null)", substr);                                                           \
      ++failures;                                                                                         \
    }                                                                                                     \
  } while (0)

#define EXPECT_OK(call)                                                                                  \
  do {                                                                                                   \
    const int st_ = (call);                                                                              \
    if (st_ != 0) {                                                                                      \
      fprintf(stderr, "FAIL %s:%d: %s -> status %d, error '%s'\n", __FILE__, __LINE__, #call, st_,      \
              flite_last_error());                                                                       \
      ++failures;                                                                                        \
    }                                                                                                    \
  } while (0)

// the state-dict inventory of a DiT (model.py:417-479 / model_v2.py layout), name -> element count
static std::vector<std::pair<std::string, long>> inventory(const flite_dit_config& c) {
  const long D = c.hidden_size, F = c.mlp_hidden, CC = c.cross_attn_input_size;
  const long cpp = (long)c.in_channels * c.patch_size * c.patch_size;
  std::vector<std::pair<std::string, long>> v = {
      {"context_proj.weight", CC * D}, {"context_proj.bias", D}, {"context_norm.weight", D},
      {"patch_embed.patch_proj.weight", cpp * D}, {"patch_embed.patch_proj.bias", D},
      {"register_tokens", 16 * D}, {"time_embed.0.weight", 4 * D * D}, {"time_embed.0.bias", 4 * D},
      {"time_embed.2.weight", 4 * D * D}, {"time_embed.2.bias", D},
      {"final_modulation.1.weight", 2 * D * D}, {"final_modulation.1.bias", 2 * D},
      {"final_proj.weight", cpp * D}, {"final_proj.bias", cpp}};
  if (c.train_bias_and_rms) v.push_back({"final_norm.weight", D});
  if (!c.per_block_adaln) {
    v.push_back({"adaLN_modulation.1.weight", 9 * D * D});
    v.push_back({"adaLN_modulation.1.bias", 9 * D});
  }
  for (int i = 0; i < c.depth; ++i) {
    const std::string b = "blocks." + std::to_string(i) + ".";
    const bool cross = c.per_block_adaln || i % 4 == 0 || i < 8;
    v.push_back({b + "norm1.weight", D});
    v.push_back({b + "self_attn.qkv.weight", 3 * D * D});
    if (c.train_bias_and_rms) v.push_back({b + "self_attn.qkv.bias", 3 * D});
    v.push_back({b + "self_attn.proj.weight", D * D});
    if (cross) {
      v.push_back({b + "norm2.weight", D});
      v.push_back({b + "cross_attn.q.weight", D * D});
      v.push_back({b + "cross_attn.context_kv.weight", 2 * D * D});
      if (c.train_bias_and_rms) {
        v.push_back({b + "cross_attn.q.bias", D});
        v.push_back({b + "cross_attn.context_kv.bias", 2 * D});
      }
      v.push_back({b + "cross_attn.proj.weight", D * D});
    }
    v.push_back({b + "norm3.weight", D});
    v.push_back({b + "mlp.gate_proj.weight", F * D});
    v.push_back({b + "mlp.up_proj.weight", F * D});
    v.push_back({b + "mlp.down_proj.weight", F * D});
    if (c.per_block_adaln) {
      v.push_back({b + "adaLN_modulation.1.weight", 9 * D * D});
      v.push_back({b + "adaLN_modulation.1.bias", 9 * D});
    }
  }
  return v;
}

static void engine_binds(int per_block, int bias) {
  flite_dit_config c{};
  c.in_channels = 16;
  c.patch_size = 2;
  c.hidden_size = 512;
  c.depth = 10;
  c.num_heads = 2;
  c.mlp_hidden = 2048;
  c.cross_attn_input_size = 128;
  c.train_bias_and_rms = bias;
  c.per_block_adaln = per_block;
  c.n_register_tokens = 16;
  c.rope_base = 10000.f;
  c.bf16_timestep_quant = 1;
  c.bf16_rope_tables = 1;
  c.use_rope = 1;
  flite::DitEngine eng(c);
  // one 16-B aligned host arena stands in for the device storage: bind only records pointers
  alignas(16) static char arena[64];
  const void* p = arena;
  EXPECT_ERR(eng.check_bound(), "unbound");
  EXPECT_ERR(eng.enable_fp8(nullptr, true), "unbound");
  EXPECT_ERR(eng.bind("blocks.3.mlp.gate_proj.weight", nullptr, 2048L * 512), "null pointer");
  EXPECT_ERR(eng.bind("blocks.3.mlp.gate_proj.weight", arena + 2, 2048L * 512), "16-B aligned");
  EXPECT_ERR(eng.bind("blocks.3.mlp.gate_proj.weight", p, 7), "expected");
  EXPECT_ERR(eng.bind("blocks.99.norm1.weight", p, 512), "out of range");
  EXPECT_ERR(eng.bind("blocks.-1.norm1.weight", p, 512), "out of range");
  EXPECT_ERR(eng.bind("blocks.0.no_such.weight", p, 512), "unknown block parameter");
  EXPECT_ERR(eng.bind("no_such_parameter", p, 512), "unknown parameter");
  EXPECT_ERR(eng.bind("blocks.", p, 512), "unknown parameter");
  EXPECT_ERR(eng.bind("blocks.7", p, 512), "unknown parameter");
  const std::string longname(4096, 'x');
  EXPECT_ERR(eng.bind(longname, p, 512), "unknown parameter");
  const auto inv = inventory(c);
  for (size_t i = 0; i + 1 < inv.size(); ++i) EXPECT_OK(eng.bind(inv[i].first, p, inv[i].second));
  EXPECT_ERR(eng.check_bound(), "unbound");  // the last tensor is still missing
  EXPECT_OK(eng.bind(inv.back().first, p, inv.back().second));
  EXPECT_OK(eng.check_bound());
  EXPECT_OK(eng.bind(inv[0].first, p, inv[0].second));  // rebinding the same storage is accepted
  EXPECT_OK(eng.weights_updated(nullptr));               // bf16 mode: nothing derived
  const int blks[2] = {0, c.depth};
  EXPECT_ERR(eng.set_fp8_bf16_blocks(blks, 2), "out of range");
  EXPECT_ERR(eng.set_fp8_bf16_blocks(nullptr, 1), "bad block list");
  EXPECT_OK(eng.set_fp8_bf16_blocks(blks, 1));
  EXPECT_OK(eng.set_fp8_bf16_blocks(nullptr, 0));
  std::vector<int> masks(c.depth, 63);
  EXPECT_ERR(eng.set_fp8_block_classes(masks.data(), c.depth - 1), "one mask per block");
  EXPECT_ERR(eng.set_fp8_block_classes(nullptr, c.depth), "one mask per block");
  masks[0] = 64;
  EXPECT_ERR(eng.set_fp8_block_classes(masks.data(), c.depth), "outside FLITE_FP8_ALL");
  masks[0] = 0;
  EXPECT_OK(eng.set_fp8_block_classes(masks.data(), c.depth));
  EXPECT_OK(eng.set_fp8_block_classes(nullptr, 0));
  EXPECT_OK(eng.set_residual_bf16(false));
  if (eng.residual_bf16()) {
    fprintf(stderr, "FAIL residual_bf16 after set_residual_bf16(false)\n");
    ++failures;
  }
  EXPECT_OK(eng.set_residual_bf16(true));
  EXPECT_ERR(eng.forward(nullptr, p, false, 1, 2, 0, 0), "prepare first");
  EXPECT_ERR(eng.unpatchify_out(nullptr, nullptr, false), "prepare first");
  long a = 0, b = 0;
  EXPECT_ERR(eng.sp_buffer_bytes(&a, &b), "prepare first");
  EXPECT_ERR(eng.set_sequence_parallel(0, 2, nullptr, nullptr), "callback missing");
  EXPECT_ERR(eng.sp_bind_buffers(nullptr, nullptr, nullptr, nullptr), "null buffer");
  float ms[4];
  int n = 0;
  (void)eng.read_probe(ms, 4, &n);
}

int main() {
  EXPECT_ERR(flite_dit_create(nullptr, nullptr), "null");
  flite_dit_config bad{};
  flite_dit* d = nullptr;
  EXPECT_ERR(flite_dit_create(&bad, &d), "bad config");
  EXPECT_ERR(flite_dit_bind(nullptr, "x", nullptr, 0), "null");
  EXPECT_ERR(flite_dit_prepare(nullptr, 1, 8, 8, 1, 1), "null");
  EXPECT_ERR(flite_dit_forward(nullptr, nullptr, nullptr, 0, 1, 0, 0, nullptr, 0), "null");
  EXPECT_ERR(flite_dit_sample(nullptr, nullptr, nullptr, 1, 1, nullptr, nullptr, 6.f, 1, 0, 0.03f, 1), "null");
  EXPECT_ERR(flite_dit_enable_fp8(nullptr, nullptr, 1), "null");
  EXPECT_ERR(flite_dit_weights_updated(nullptr, nullptr), "null");
  EXPECT_ERR(flite_vae_create(nullptr, nullptr), "null");
  flite_vae_config vbad{};
  flite_vae* v = nullptr;
  EXPECT_ERR(flite_vae_create(&vbad, &v), "unsupported config");
  EXPECT_ERR(flite_vae_bind(nullptr, "x", nullptr, 0), "null");
  EXPECT_ERR(flite_vae_weights_updated(nullptr), "null");
  EXPECT_ERR(flite_cfg_euler(nullptr, nullptr, nullptr, nullptr, 4, 6.f, 0.1f, 1), "null");
  alignas(16) static float f[8];
  EXPECT_ERR(flite_cfg_euler(nullptr, f, f, f, -1, 6.f, 0.1f, 1), "negative");
  EXPECT_ERR(flite_apg_sums(nullptr, nullptr, f, 4, 0.f, 0, f), "null");
  EXPECT_ERR(flite_apg_sums(nullptr, f, f, 4, 0.f, 2, f), "phase");
  EXPECT_ERR(flite_apg_euler(nullptr, f, f, nullptr, 4, 6.f, 0.f, 1.f, 0.1f), "null");
  EXPECT_ERR(flite_apg_sums_dev(nullptr, f, f, 4, 0, nullptr), "null");
  EXPECT_ERR(flite_apg_sums_dev(nullptr, f, f, -1, 0, f), "negative");
  EXPECT_ERR(flite_apg_sums_dev(nullptr, f, f, 4, 3, f), "phase");
  EXPECT_ERR(flite_apg_euler_dev(nullptr, f, f, f, 4, 6.f, 0.03f, 4, nullptr, 0.1f), "null");
  EXPECT_ERR(flite_apg_euler_dev(nullptr, f, f, f, 8, 6.f, 0.03f, 4, f, 0.1f), "element counts");
  EXPECT_ERR(flite_dit_set_fp8_bf16_blocks(nullptr, nullptr, 0), "null");
  EXPECT_ERR(flite_dit_set_fp8_block_classes(nullptr, nullptr, 0), "null");
  EXPECT_ERR(flite_dit_set_residual_bf16(nullptr, 1), "null");
  if (flite_dit_residual_bf16(nullptr) != -1) {
    fprintf(stderr, "FAIL flite_dit_residual_bf16(nullptr) != -1\n");
    ++failures;
  }
  // GEMM shape / stride / alignment validation happens before any kernel initialisation
  alignas(16) static char g[256];
  EXPECT_ERR(flite_gemm_bf16(nullptr, 0, 64, 64, g, 64, g, 64, nullptr, nullptr, 0, g, 64, nullptr, 0, 0), "empty");
  EXPECT_ERR(flite_gemm_bf16(nullptr, 8, 64, 60, g, 64, g, 64, nullptr, nullptr, 0, g, 64, nullptr, 0, 0),
             "multiple of 64");
  EXPECT_ERR(flite_gemm_bf16(nullptr, 8, 64, 64, g, 64, g + 2, 64, nullptr, nullptr, 0, g, 64, nullptr, 0, 0),
             "16-B aligned");
  EXPECT_ERR(flite_gemm_bf16(nullptr, 8, 64, 64, g, 60, g, 64, nullptr, nullptr, 0, g, 64, nullptr, 0, 0),
             "lda");
  EXPECT_ERR(flite_gemm_bf16(nullptr, 8, 64, 64, g, 64, g, 60, nullptr, nullptr, 0, g, 64, nullptr, 0, 0),
             "ldw");
  for (int pb = 0; pb < 2; ++pb)
    for (int bias = 0; bias < 2; ++bias) engine_binds(pb, bias);
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("capi_validation: all checks passed\n");
  return 0;
}
