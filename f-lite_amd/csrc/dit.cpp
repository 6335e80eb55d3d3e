// Native DiT engine (host side). See dit.h.
#include "dit.h"

#include <cstdlib>

#include <math.h>
#include <stdio.h>
#include <string.h>

namespace flite {

constexpr long kPosEmbRows = 2048;  // DiT.positional_embedding rows (model.py:444)

namespace {
constexpr int HEAD_DIM = 256;
// q and k are RMS-normalised per head before every DiT attention (QKNorm, model.py:180,197): |q|,|k| <= 16
// (+ bf16 rounding), so |q.k| / sqrt(256) <= 16; 16.5 leaves margin for the rounding of q and k.
constexpr float kQKNormScoreBound = 16.5f;

// RoPE + QK-norm fused into the qkv / cross-q GEMM epilogue (gemm.hip EPI_QKV_NORM_BF16); FLITE_NO_QK_FUSION=1
// runs the separate rope_qknorm kernel instead (A/B switch for measurements)
bool fuse_qk_norm() {
  static const bool on = getenv("FLITE_NO_QK_FUSION") == nullptr;
  return on;
}

// The norm passes read the next GEMM's weights ahead (NormModParams::pf); FLITE_NO_WPREFETCH=1 turns it off (A/B)
bool w_prefetch() {
  static const bool on = getenv("FLITE_NO_WPREFETCH") == nullptr;
  return on;
}

// Block 0 of a CFG batch runs its self-attention sub-block once per image instead of once per CFG copy (forward);
// FLITE_NO_CFG_DEDUP=1 runs it on every copy (A/B switch for measurements)
bool cfg_dedup() {
  static const bool on = getenv("FLITE_NO_CFG_DEDUP") == nullptr;
  return on;
}

// the norm2 pass reading the cross-q weights ahead (NormModParams::pf); FLITE_NO_NORM_PF=1 turns only it off
bool norm_prefetch() {
  static const bool on = w_prefetch() && getenv("FLITE_NO_NORM_PF") == nullptr;
  return on;
}

// Uniform-context collapse: a sequence whose context rows are all equal (the pipeline's zero negative prompt) has
// equal cross-attention keys and values, so its cross-attention output is the V row for every query, and the whole
// cross-attention sub-block reduces to x += gate_ca * (V . Wproj^T), step-invariant (set_context makes it once).
// FLITE_NO_CTX_COLLAPSE=1 computes those rows like any other (A/B switch and test reference).
bool ctx_collapse() {
  static const bool on = getenv("FLITE_NO_CTX_COLLAPSE") == nullptr;
  return on;
}

bool parse_block(const std::string& name, int* idx, std::string* rest) {
  if (name.rfind("blocks.", 0) != 0) return false;
  const size_t dot = name.find('.', 7);
  if (dot == std::string::npos) return false;
  *idx = atoi(name.substr(7, dot - 7).c_str());
  *rest = name.substr(dot + 1);
  return true;
}
}  // namespace

DitEngine::DitEngine(const flite_dit_config& c) : cfg(c) {
  D = c.hidden_size;
  H = c.num_heads;
  F = c.mlp_hidden;
  R = c.n_register_tokens;
  P = c.patch_size;
  C = c.in_channels;
  w_.blocks.resize(c.depth);
  // residual-stream storage: bf16 by default since round 6 (the reference's own storage type, model.py:289; +1.55 %
  // images/s against fp32 in a same-box A/B, profiles/r06b); FLITE_RESID_BF16=0 makes fp32 the default (A/B switch)
  const char* x16 = getenv("FLITE_RESID_BF16");
  x16_ = !(x16 != nullptr && x16[0] == '0');
  for (int i = 0; i < c.depth; ++i)
    w_.blocks[i].cross = c.per_block_adaln ? true : (i % 4 == 0 || i < 8);  // model.py:464 / model_v2.py:468
}

DitEngine::~DitEngine() {
  drop_graph();
  free_fp8_weights();
  free_ws();
  if (gstream_) hipStreamDestroy(gstream_);
  if (ev_in_) hipEventDestroy(ev_in_);
  if (ev_out_) hipEventDestroy(ev_out_);
  if (xstream_) hipStreamDestroy(xstream_);
  if (ev_kv_) hipEventDestroy(ev_kv_);
  if (ev_x_) hipEventDestroy(ev_x_);
  for (int i = 0; i < 2; ++i) {
    if (ev_ring_[i]) hipEventDestroy(ev_ring_[i]);
    if (ev_used_[i]) hipEventDestroy(ev_used_[i]);
  }
}

// Destroy the cached graph once every replay of it has finished (a replay may still be in flight on gstream_).
void DitEngine::drop_graph() {
  if (!gexec_) return;
  if (gstream_) hipStreamSynchronize(gstream_);
  hipGraphExecDestroy(gexec_);
  gexec_ = nullptr;
}

void DitEngine::free_ws() {
  for (void* p : allocs_) hipFree(p);
  allocs_.clear();
  ctx_kv_.clear();
  sk_ws_ = nullptr;
  sk_flags_ = nullptr;
  attn_ws_ = nullptr;
  attn_ws_bytes_ = 0;
  nbuf8_ = nbuf8_s_ = obuf8_ = obuf8_s_ = hbuf8_ = hbuf8_s_ = nullptr;
  x_ = nullptr;
  kv_full_ = nullptr;
  cu_full_ = nullptr;
  part_o_ = part_l_ = nullptr;
  kend_loc_ = cu_rem_ = kend_all_ = nullptr;
  rope_axes_ = nullptr;
}

RopeAxes DitEngine::rope_axes() const {
  RopeAxes r;
  r.cs = rope_axes_;
  r.tokens = Tl_;
  r.tok0 = sp_rank_ * Tl_;  // the rows held here start at this token of the sequence
  r.reg = R;
  r.h = Hl_ / P;
  r.w = Wl_ / P;
  r.inv_w = 1.f / (float)r.w;
  return r;
}

void DitEngine::free_fp8_weights() {
  for (void* p : w8_allocs_) hipFree(p);
  w8_allocs_.clear();
  w8_.clear();
}

// every GEMM of the engine may use the stream-K workspace (launches on the engine's streams are ordered)
int DitEngine::gemm(GemmParams& g, int epi, hipStream_t s) {
  static const bool no_sk = getenv("FLITE_GEMM_NO_STREAM_K") != nullptr;  // A/B switch for measurements
  g.sk_ws = no_sk ? nullptr : sk_ws_;
  g.sk_flags = no_sk ? nullptr : sk_flags_;
  return gemm_bf16(g, epi, s);
}

int DitEngine::alloc(void** p, size_t bytes) {
  if (bytes == 0) bytes = 16;
  FLITE_HIP_CHECK(hipMalloc(p, bytes));
  allocs_.push_back(*p);
  return 0;
}

int DitEngine::bind(const std::string& name, const void* ptr, long numel) {
  FLITE_REQUIRE(ptr != nullptr, "bind: null pointer for " + name);
  FLITE_REQUIRE(((uintptr_t)ptr & 15) == 0, "bind: parameter " + name + " is not 16-B aligned");
  // a captured graph bakes every weight pointer into its kernel arguments: rebinding to new storage
  // invalidates it (the next sample() recaptures)
  auto old = bound_.find(name);
  if (old == bound_.end() || old->second.first != ptr) {
    drop_graph();
    // the fp8 copies were quantised from the old storage: fp8 mode stays on and the next forward / sample
    // requantises them (into the same buffers) before it runs
    w8_stale_ = true;
    ctx_stale_ = true;  // the context K/V were projected with the old weights
  }
  bound_[name] = {ptr, numel};
  const bf16_t* p = (const bf16_t*)ptr;
  const long DD = (long)D * D;
  auto expect = [&](long n) -> int {
    FLITE_REQUIRE(numel == n, "bind: " + name + " has " + std::to_string(numel) + " elements, expected " +
                                  std::to_string(n));
    return 0;
  };
  int blk;
  std::string rest;
  if (parse_block(name, &blk, &rest)) {
    FLITE_REQUIRE(blk >= 0 && blk < cfg.depth, "bind: block index out of range in " + name);
    BlockW& b = w_.blocks[blk];
    if (rest == "norm1.weight") { if (expect(D)) return 2; b.norm1 = p; }
    else if (rest == "self_attn.qkv.weight") { if (expect(3 * DD)) return 2; b.qkv_w = p; }
    else if (rest == "self_attn.qkv.bias") { if (expect(3L * D)) return 2; b.qkv_b = p; }
    else if (rest == "self_attn.proj.weight") { if (expect(DD)) return 2; b.proj_w = p; }
    else if (rest == "norm2.weight") { if (expect(D)) return 2; b.norm2 = p; }
    else if (rest == "cross_attn.q.weight") { if (expect(DD)) return 2; b.cq_w = p; }
    else if (rest == "cross_attn.q.bias") { if (expect(D)) return 2; b.cq_b = p; }
    else if (rest == "cross_attn.context_kv.weight") { if (expect(2 * DD)) return 2; b.ckv_w = p; }
    else if (rest == "cross_attn.context_kv.bias") { if (expect(2L * D)) return 2; b.ckv_b = p; }
    else if (rest == "cross_attn.proj.weight") { if (expect(DD)) return 2; b.cproj_w = p; }
    else if (rest == "norm3.weight") { if (expect(D)) return 2; b.norm3 = p; }
    else if (rest == "mlp.gate_proj.weight") { if (expect((long)F * D)) return 2; b.gate_w = p; }
    else if (rest == "mlp.up_proj.weight") { if (expect((long)F * D)) return 2; b.up_w = p; }
    else if (rest == "mlp.down_proj.weight") { if (expect((long)F * D)) return 2; b.down_w = p; }
    else if (rest == "adaLN_modulation.1.weight") { if (expect(9 * DD)) return 2; b.ada_w = p; }
    else if (rest == "adaLN_modulation.1.bias") { if (expect(9L * D)) return 2; b.ada_b = p; }
    else FLITE_REQUIRE(false, "bind: unknown block parameter " + name);
    return 0;
  }
  const long CC = cfg.cross_attn_input_size;
  const long cpp = (long)C * P * P;
  if (name == "context_proj.weight") { if (expect(CC * D)) return 2; w_.ctx_proj_w = p; }
  else if (name == "context_proj.bias") { if (expect(D)) return 2; w_.ctx_proj_b = p; }
  else if (name == "context_norm.weight") { if (expect(D)) return 2; w_.ctx_norm = p; }
  else if (name == "patch_embed.patch_proj.weight") { if (expect(cpp * D)) return 2; w_.patch_w = p; }
  else if (name == "patch_embed.patch_proj.bias") { if (expect(D)) return 2; w_.patch_b = p; }
  else if (name == "register_tokens") { if (expect((long)R * D)) return 2; w_.registers = p; }
  else if (name == "positional_embedding" && !cfg.use_rope) { if (expect(kPosEmbRows * D)) return 2; w_.pos_emb = p; }
  else if (name == "time_embed.0.weight") { if (expect(4 * DD)) return 2; w_.te0_w = p; }
  else if (name == "time_embed.0.bias") { if (expect(4L * D)) return 2; w_.te0_b = p; }
  else if (name == "time_embed.2.weight") { if (expect(4 * DD)) return 2; w_.te2_w = p; }
  else if (name == "time_embed.2.bias") { if (expect(D)) return 2; w_.te2_b = p; }
  else if (name == "adaLN_modulation.1.weight") { if (expect(9 * DD)) return 2; w_.ada_w = p; }
  else if (name == "adaLN_modulation.1.bias") { if (expect(9L * D)) return 2; w_.ada_b = p; }
  else if (name == "final_modulation.1.weight") { if (expect(2 * DD)) return 2; w_.fmod_w = p; }
  else if (name == "final_modulation.1.bias") { if (expect(2L * D)) return 2; w_.fmod_b = p; }
  else if (name == "final_norm.weight") { if (expect(D)) return 2; w_.fnorm = p; }
  else if (name == "final_proj.weight") { if (expect(cpp * D)) return 2; w_.fproj_w = p; }
  else if (name == "final_proj.bias") { if (expect(cpp)) return 2; w_.fproj_b = p; }
  else FLITE_REQUIRE(false, "bind: unknown parameter " + name);
  return 0;
}

int DitEngine::check_bound() {
  const bool bias = cfg.train_bias_and_rms != 0;
  FLITE_REQUIRE(w_.ctx_proj_w && w_.ctx_proj_b && w_.ctx_norm, "unbound: context_proj/context_norm");
  FLITE_REQUIRE(w_.patch_w && w_.patch_b && w_.registers, "unbound: patch_embed/register_tokens");
  FLITE_REQUIRE(cfg.use_rope || w_.pos_emb, "unbound: positional_embedding (use_rope = 0)");
  FLITE_REQUIRE(w_.te0_w && w_.te0_b && w_.te2_w && w_.te2_b, "unbound: time_embed");
  FLITE_REQUIRE(w_.fmod_w && w_.fmod_b && w_.fproj_w && w_.fproj_b, "unbound: final stage");
  FLITE_REQUIRE(!bias || w_.fnorm, "unbound: final_norm.weight");
  if (!cfg.per_block_adaln) FLITE_REQUIRE(w_.ada_w && w_.ada_b, "unbound: adaLN_modulation");
  for (int i = 0; i < cfg.depth; ++i) {
    const BlockW& b = w_.blocks[i];
    const std::string pre = "unbound: blocks." + std::to_string(i) + ".";
    FLITE_REQUIRE(b.norm1 && b.qkv_w && b.proj_w && b.norm3 && b.gate_w && b.up_w && b.down_w, pre + "*");
    FLITE_REQUIRE(!bias || b.qkv_b, pre + "self_attn.qkv.bias");
    if (b.cross) {
      FLITE_REQUIRE(b.norm2 && b.cq_w && b.ckv_w && b.cproj_w, pre + "cross_attn.*");
      FLITE_REQUIRE(!bias || (b.cq_b && b.ckv_b), pre + "cross_attn biases");
    }
    if (cfg.per_block_adaln) FLITE_REQUIRE(b.ada_w && b.ada_b, pre + "adaLN_modulation");
  }
  return 0;
}

int DitEngine::prepare(int B, int Hl, int Wl, int n_ctx_max, int n_t_max) {
  FLITE_REQUIRE(D % 256 == 0 && D / H == HEAD_DIM, "config: hidden_size / num_heads must be 256");
  FLITE_REQUIRE(F % 256 == 0 || F % 16 == 0, "config: mlp hidden must be a multiple of 16");
  FLITE_REQUIRE(Hl % P == 0 && Wl % P == 0, "prepare: latent H, W must be multiples of patch_size");
  FLITE_REQUIRE(Hl / P <= 512 && Wl / P <= 512, "prepare: RoPE tables cover at most 512x512 patches");
  FLITE_REQUIRE(cfg.use_rope || R + (Hl / P) * (Wl / P) <= kPosEmbRows,
                "prepare: the learned positional embedding covers at most 2048 rows (registers + patches)");
  FLITE_REQUIRE(cfg.cross_attn_input_size % 64 == 0, "config: cross_attn_input_size must be a multiple of 64");
  if (check_bound()) return 2;
  FLITE_REQUIRE(sp_n_ == 1 || (!fp8_ && cfg.use_rope),
                "prepare: sequence parallelism runs the bf16 RoPE path only (no fp8, no positional_embedding)");
  if (B == B_ && Hl == Hl_ && Wl == Wl_ && n_ctx_max <= nctx_max_ && n_t_max <= ntmax_) return 0;
  drop_graph();
  free_ws();
  B_ = B;
  Hl_ = Hl;
  Wl_ = Wl;
  HW_ = (Hl / P) * (Wl / P);
  T_ = R + HW_;
  Tl_ = (T_ + sp_n_ - 1) / sp_n_;
  FLITE_REQUIRE(Tl_ >= R, "prepare: sequence parallelism needs at least 16 rows per rank");
  M_ = (long)B * Tl_;
  sp_kv_send_ = sp_kv_recv_ = nullptr;  // caller buffers are sized per shape: bind again after prepare
  sp_out_send_ = sp_out_recv_ = nullptr;
  nctx_max_ = n_ctx_max;
  ntmax_ = n_t_max;
  const int cpp = C * P * P;
  if (alloc((void**)&x_, M_ * D * 4)) return 1;
  if (alloc((void**)&nbuf_, M_ * D * 2)) return 1;
  if (alloc((void**)&qkv_, M_ * 3 * D * 2)) return 1;
  if (alloc((void**)&obuf_, M_ * D * 2)) return 1;
  if (alloc((void**)&hbuf_, M_ * (long)F * 2)) return 1;
  if (alloc((void**)&patches_, (long)B * HW_ * cpp * 2)) return 1;
  if (alloc((void**)&fout_, (long)B * HW_ * cpp * 4)) return 1;
  if (alloc((void**)&acc_, (long)B * HW_ * cpp * 4)) return 1;
  {
    const int G = gemm_sk_workspace_cus();
    if (G > 0) {
      if (alloc((void**)&sk_ws_, (size_t)G * 256 * 256 * 4)) return 1;
      if (alloc((void**)&sk_flags_, (size_t)G * 4)) return 1;
      FLITE_HIP_CHECK(hipMemset(sk_flags_, 0, (size_t)G * 4));
    }
  }
  attn_ws_bytes_ = attn_workspace_bytes(B, H, Tl_, T_);  // self-attention: Tl_ queries over T_ keys
  if (attn_ws_bytes_ > 0) {
    if (alloc(&attn_ws_, (size_t)attn_ws_bytes_)) return 1;
    FLITE_HIP_CHECK(hipMemset(attn_ws_, 0, (size_t)attn_ws_bytes_));
  }
  if (alloc((void**)&cu_self_, (B + 1) * 4)) return 1;
  if (alloc((void**)&cu_ctx_, (B + 1) * 4)) return 1;
  if (alloc((void**)&ctx_c_, (long)cfg.depth * B * D * 4)) return 1;
  if (alloc((void**)&ctx_vrow_, (long)B * D * 2)) return 1;
  if (alloc((void**)&ctx_bad_, (long)B * 4)) return 1;
  if (alloc((void**)&ctx_c8_, (long)cfg.depth * B * D * 4)) return 1;
  if (alloc((void**)&ctx_vrow8_, (long)B * D)) return 1;
  // the collapse's M = U <= B rows: scale rows padded to the GEMM's 256-row tiles, however many sequences
  vrow8_rows_pad_ = mx_rows_pad(B);
  if (alloc((void**)&ctx_vrow8_s_, (long)(D / 128) * vrow8_rows_pad_ * 4)) return 1;
  ctx_uni_ = 0;
  ctx_c8_stale_ = true;
  // RoPE tables for every row a rank may hold (the last rank's padding rows read zeros)
  if (alloc((void**)&cos_, (long)sp_n_ * Tl_ * 128 * 4)) return 1;
  if (alloc((void**)&sin_, (long)sp_n_ * Tl_ * 128 * 4)) return 1;
  FLITE_HIP_CHECK(hipMemset(cos_, 0, (size_t)sp_n_ * Tl_ * 128 * 4));
  FLITE_HIP_CHECK(hipMemset(sin_, 0, (size_t)sp_n_ * Tl_ * 128 * 4));
  if (sp_n_ > 1) {
    if (alloc((void**)&kv_full_, (long)B * T_ * 2 * D * 2)) return 1;
    if (alloc((void**)&cu_full_, (B + 1) * 4)) return 1;
    std::vector<int> cuf(B + 1);
    for (int i = 0; i <= B; ++i) cuf[i] = i * T_;
    FLITE_HIP_CHECK(hipMemcpy(cu_full_, cuf.data(), (B + 1) * 4, hipMemcpyHostToDevice));
    // overlapped exchange: local keys [b*Tl, b*Tl + v) of the rank's own rows, remote keys packed per sequence
    const int v = std::max(0, std::min(T_, (sp_rank_ + 1) * Tl_) - sp_rank_ * Tl_);
    std::vector<int> kend(B), cur(B + 1);
    for (int i = 0; i < B; ++i) kend[i] = i * Tl_ + v;
    for (int i = 0; i <= B; ++i) cur[i] = i * (T_ - v);
    if (alloc((void**)&part_o_, M_ * D * 4)) return 1;
    if (alloc((void**)&part_l_, M_ * H * 4)) return 1;
    if (alloc((void**)&kend_loc_, B * 4)) return 1;
    if (alloc((void**)&cu_rem_, (B + 1) * 4)) return 1;
    FLITE_HIP_CHECK(hipMemcpy(kend_loc_, kend.data(), B * 4, hipMemcpyHostToDevice));
    FLITE_HIP_CHECK(hipMemcpy(cu_rem_, cur.data(), (B + 1) * 4, hipMemcpyHostToDevice));
    std::vector<int> ka((size_t)sp_n_ * B);
    for (int q = 0; q < sp_n_; ++q)
      for (int i = 0; i < B; ++i) ka[(size_t)q * B + i] = i * Tl_ + std::max(0, std::min(T_, (q + 1) * Tl_) - q * Tl_);
    if (alloc((void**)&kend_all_, (long)sp_n_ * B * 4)) return 1;
    FLITE_HIP_CHECK(hipMemcpy(kend_all_, ka.data(), (size_t)sp_n_ * B * 4, hipMemcpyHostToDevice));
    if (!xstream_) {
      FLITE_HIP_CHECK(hipStreamCreateWithFlags(&xstream_, hipStreamNonBlocking));
      FLITE_HIP_CHECK(hipEventCreateWithFlags(&ev_kv_, hipEventDisableTiming));
      FLITE_HIP_CHECK(hipEventCreateWithFlags(&ev_x_, hipEventDisableTiming));
      for (int i = 0; i < 2; ++i) {
        FLITE_HIP_CHECK(hipEventCreateWithFlags(&ev_ring_[i], hipEventDisableTiming));
        FLITE_HIP_CHECK(hipEventCreateWithFlags(&ev_used_[i], hipEventDisableTiming));
      }
    }
    const char* no = getenv("FLITE_SP_NO_OVERLAP");  // A/B switch: gather every key first, one attention
    sp_overlap_ = !(no && no[0] == '1');
  }
  if (alloc((void**)&inv_freq_, 64 * 4)) return 1;
  if (alloc((void**)&rope_axes_, (long)(1 + Hl / P + Wl / P) * 128 * 4)) return 1;
  if (alloc((void**)&ctx_p_, (long)std::max(n_ctx_max, 1) * D * 2)) return 1;
  ctx_kv_.assign(cfg.depth, nullptr);
  for (int i = 0; i < cfg.depth; ++i)
    if (w_.blocks[i].cross)
      if (alloc((void**)&ctx_kv_[i], (long)std::max(n_ctx_max, 1) * 2 * D * 2)) return 1;
  if (alloc((void**)&tdev_, std::max(n_t_max, 1) * 4)) return 1;
  if (alloc((void**)&temb_, (long)std::max(n_t_max, 1) * D * 2)) return 1;
  if (alloc((void**)&th_, (long)std::max(n_t_max, 1) * 4 * D * 2)) return 1;
  if (alloc((void**)&tsilu_, (long)std::max(n_t_max, 1) * D * 2)) return 1;
  mod_t_stride_ = (long)(cfg.per_block_adaln ? cfg.depth : 1) * 9 * D;
  if (alloc((void**)&mod_, std::max(n_t_max, 1) * mod_t_stride_ * 4)) return 1;
  if (alloc((void**)&fmod_, (long)std::max(n_t_max, 1) * 2 * D * 4)) return 1;

  // self-attention cu_seqlens [0, T, 2T, ...] (prepare_flash_attention_inputs with no mask, model.py:549)
  std::vector<int> cu(B + 1);
  for (int i = 0; i <= B; ++i) cu[i] = i * Tl_;  // queries held here
  FLITE_HIP_CHECK(hipMemcpy(cu_self_, cu.data(), (B + 1) * 4, hipMemcpyHostToDevice));
  // RoPE inv_freq in double like the reference's python list (model.py:342), then fp32
  const int rdim = D / (2 * H);  // 128
  FLITE_REQUIRE(rdim == 128, "config: RoPE dim must be 128");
  float inv[64];
  for (int i = 0; i < 64; ++i) inv[i] = (float)(1.0 / pow((double)cfg.rope_base, (double)(2 * i) / (double)rdim));
  FLITE_HIP_CHECK(hipMemcpy(inv_freq_, inv, sizeof(inv), hipMemcpyHostToDevice));
  if (rope_table(inv_freq_, cos_, sin_, Hl / P, Wl / P, R, cfg.bf16_rope_tables, 0)) return 1;
  if (rope_axes_table(inv_freq_, rope_axes_, Hl / P, Wl / P, cfg.bf16_rope_tables, 0)) return 1;
  if (fp8_ && alloc_fp8_act()) return 1;
  FLITE_HIP_CHECK(hipDeviceSynchronize());
  nctx_ = 0;
  nt_ = 0;
  return 0;
}

int DitEngine::set_context(hipStream_t s, const void* ctx, const int* cu_host, int nseq) {
  FLITE_REQUIRE(x_ != nullptr, "set_context: call prepare first");
  FLITE_REQUIRE(nseq == B_, "set_context: number of context sequences must equal the batch");
  const int n = cu_host[nseq];
  FLITE_REQUIRE(n <= nctx_max_, "set_context: context longer than prepared");
  for (int i = 0; i < nseq; ++i) FLITE_REQUIRE(cu_host[i + 1] >= cu_host[i], "set_context: bad cu_seqlens");
  // stale until the last K/V projection below has been issued: a failure part-way leaves the cache refused
  ctx_stale_ = true;
  FLITE_HIP_CHECK(hipMemcpyAsync(cu_ctx_, cu_host, (nseq + 1) * 4, hipMemcpyHostToDevice, s));
  nctx_ = n;
  nseq_ctx_ = nseq;
  ctx_max_len_ = 0;
  for (int i = 0; i < nseq; ++i) ctx_max_len_ = std::max(ctx_max_len_, cu_host[i + 1] - cu_host[i]);
  if (n == 0) {
    // no keys at all: every sequence takes the zero-key cross-attention, so no row may keep an earlier call's
    // collapse (x += gate * c of the old context) and a cached graph holding its launch shapes must go
    if (ctx_uni_ != 0) drop_graph();
    ctx_uni_ = 0;
    ctx_row0_.clear();
    ctx_c8_stale_ = true;
    ctx_stale_ = false;
    return 0;
  }
  // context_proj (model.py:527) -> LigerRMSNorm (model.py:528)
  GemmParams g;
  g.A = (const bf16_t*)ctx;
  g.lda = cfg.cross_attn_input_size;
  g.W = w_.ctx_proj_w;
  g.ldw = cfg.cross_attn_input_size;
  g.bias = w_.ctx_proj_b;
  g.out = ctx_p_;
  g.ldo = D;
  g.M = n;
  g.N = D;
  g.K = cfg.cross_attn_input_size;
  if (gemm(g, EPI_STORE_BF16, s)) return 1;
  NormModParams nm;
  nm.x = ctx_p_;
  nm.ldx = D;
  nm.y = ctx_p_;
  nm.ldy = D;
  nm.w = w_.ctx_norm;
  nm.rows = n;
  nm.D = D;
  if (rmsnorm_mod(nm, true, s)) return 1;
  // step-invariant cross-attention K/V (model.py:189-197): context_kv then key QK-norm, cached per block
  for (int i = 0; i < cfg.depth; ++i) {
    const BlockW& b = w_.blocks[i];
    if (!b.cross) continue;
    GemmParams k;
    k.A = ctx_p_;
    k.lda = D;
    k.W = b.ckv_w;
    k.ldw = D;
    k.bias = b.ckv_b;
    k.out = ctx_kv_[i];
    k.ldo = 2L * D;
    k.M = n;
    k.N = 2 * D;
    k.K = D;
    if (gemm(k, EPI_STORE_BF16, s)) return 1;
    RopeNormParams rn;
    rn.x = ctx_kv_[i];
    rn.ldx = 2L * D;
    rn.rows = n;
    rn.heads = H;
    rn.rope_heads = 0;
    if (rope_qknorm(rn, s)) return 1;
  }
  // uniform-context collapse: the leading sequences whose rows are all equal, and their c = V . Wproj^T per block
  int uni = 0;
  if (ctx_collapse() && sp_n_ == 1) {
    FLITE_HIP_CHECK(hipMemsetAsync(ctx_bad_, 0, (size_t)nseq * 4, s));
    if (rows_uniform(ctx, cfg.cross_attn_input_size, cu_ctx_, nseq, ctx_bad_, s)) return 1;
    std::vector<int> bad(nseq);
    FLITE_HIP_CHECK(hipMemcpyAsync(bad.data(), ctx_bad_, (size_t)nseq * 4, hipMemcpyDeviceToHost, s));
    FLITE_HIP_CHECK(hipStreamSynchronize(s));
    while (uni < nseq && cu_host[uni + 1] > cu_host[uni] && !bad[uni]) ++uni;
  }
  if (uni != ctx_uni_) drop_graph();  // a cached graph holds the other launch shapes
  ctx_uni_ = uni;
  ctx_row0_.assign(cu_host, cu_host + uni);
  ctx_c8_stale_ = true;
  for (int i = 0; i < cfg.depth && uni > 0; ++i) {
    const BlockW& b = w_.blocks[i];
    if (!b.cross) continue;
    for (int q = 0; q < uni; ++q)  // the sequence's V row (model.py:189-196: every key of it has this value)
      FLITE_HIP_CHECK(hipMemcpyAsync(ctx_vrow_ + (long)q * D, ctx_kv_[i] + (long)cu_host[q] * 2 * D + D,
                                     (size_t)D * 2, hipMemcpyDeviceToDevice, s));
    GemmParams g;
    g.A = ctx_vrow_;
    g.lda = D;
    g.W = b.cproj_w;
    g.ldw = D;
    g.out = ctx_c_ + (long)i * B_ * D;
    g.ldo = D;
    g.M = uni;
    g.N = D;
    g.K = D;
    if (gemm(g, EPI_STORE_F32, s)) return 1;
  }
  ctx_stale_ = false;
  return 0;
}

int DitEngine::set_timesteps(hipStream_t s, const float* t_dev, int n, int quantize) {
  FLITE_REQUIRE(x_ != nullptr, "set_timesteps: call prepare first");
  FLITE_REQUIRE(n >= 1 && n <= ntmax_, "set_timesteps: too many timesteps for the prepared workspace");
  if (t_dev != tdev_) FLITE_HIP_CHECK(hipMemcpyAsync(tdev_, t_dev, n * 4, hipMemcpyDeviceToDevice, s));
  nt_ = n;
  // timestep_embedding (model.py:20-28,551) -> time_embed Linear-SiLU-Linear (model.py:448-452)
  if (timestep_embed(tdev_, temb_, n, D, quantize, s)) return 1;
  GemmParams g;
  g.A = temb_;
  g.lda = D;
  g.W = w_.te0_w;
  g.ldw = D;
  g.bias = w_.te0_b;
  g.out = th_;
  g.ldo = 4L * D;
  g.M = n;
  g.N = 4 * D;
  g.K = D;
  g.act = 1;
  if (gemm(g, EPI_STORE_BF16, s)) return 1;
  GemmParams g2;
  g2.A = th_;
  g2.lda = 4L * D;
  g2.W = w_.te2_w;
  g2.ldw = 4L * D;
  g2.bias = w_.te2_b;
  g2.out = tsilu_;  // t_emb only feeds SiLU->Linear heads (adaLN_modulation, final_modulation)
  g2.ldo = D;
  g2.M = n;
  g2.N = D;
  g2.K = 4 * D;
  g2.act = 1;
  if (gemm(g2, EPI_STORE_BF16, s)) return 1;
  // adaLN modulation rows (model.py:553-556; model_v2.py:275 per block), fp32
  auto ada = [&](const bf16_t* W, const bf16_t* b, float* out, long ldo) -> int {
    GemmParams a;
    a.A = tsilu_;
    a.lda = D;
    a.W = W;
    a.ldw = D;
    a.bias = b;
    a.out = out;
    a.ldo = ldo;
    a.M = n;
    a.N = 9 * D;
    a.K = D;
    return gemm(a, EPI_STORE_F32, s);
  };
  if (cfg.per_block_adaln) {
    for (int i = 0; i < cfg.depth; ++i)
      if (ada(w_.blocks[i].ada_w, w_.blocks[i].ada_b, mod_ + (long)i * 9 * D, mod_t_stride_)) return 1;
  } else {
    if (ada(w_.ada_w, w_.ada_b, mod_, mod_t_stride_)) return 1;
  }
  // final modulation (model.py:578): chunk order (shift, scale)
  GemmParams f;
  f.A = tsilu_;
  f.lda = D;
  f.W = w_.fmod_w;
  f.ldw = D;
  f.bias = w_.fmod_b;
  f.out = fmod_;
  f.ldo = 2L * D;
  f.M = n;
  f.N = 2 * D;
  f.K = D;
  if (gemm(f, EPI_STORE_F32, s)) return 1;
  return 0;
}

// One DiTBlock (model.py:270-303). mod points at this block's 9 modulation chunks for segment 0;
// segment b (= sample b of the CFG batch) reads mod + b * mseg.
int DitEngine::run_block(hipStream_t s, int blk, const float* mod, long mseg) {
  const BlockW& b = w_.blocks[blk];
  const float *shift_sa = mod, *scale_sa = mod + D, *gate_sa = mod + 2L * D;
  const float *shift_ca = mod + 3L * D, *scale_ca = mod + 4L * D, *gate_ca = mod + 5L * D;
  const float *shift_mlp = mod + 6L * D, *scale_mlp = mod + 7L * D, *gate_mlp = mod + 8L * D;

  // pf0/pf1: weights of the GEMM that reads this norm's output, read ahead into the Infinity Cache (w_prefetch)
  // sa_seqs_ > 0 (forward, block 0 of a CFG batch): the self-attention sub-block runs on the first sa_seqs_
  // sequences only, and its residual rows are then copied to the other CFG copies (they are identical until the
  // cross-attention, which sees each copy's own context)
  const int Bsa = sa_seqs_ > 0 ? sa_seqs_ : B_;
  const long Msa = (long)Bsa * Tl_;
  auto norm = [&](const bf16_t* w, const float* sh, const float* sc, const bf16_t* pf0 = nullptr, long pf0_n = 0,
                  const bf16_t* pf1 = nullptr, long pf1_n = 0, long rows = 0, const float* bc_c = nullptr,
                  const float* bc_gate = nullptr, long bc_rows = 0) -> int {
    NormModParams nm;
    nm.bc_c = bc_c;
    nm.bc_gate = bc_gate;
    nm.bc_gate_stride = mseg;
    nm.bc_rows = bc_rows;
    nm.bc_rows_per_seg = Tl_;
    if (norm_prefetch()) {
      nm.pf[0] = pf0;
      nm.pf_bytes[0] = pf0_n * 2;
      nm.pf[1] = pf1;
      nm.pf_bytes[1] = pf1_n * 2;
    }
    nm.x = x_;
    nm.ldx = D;
    nm.y = nbuf_;
    nm.ldy = D;
    nm.w = w;
    nm.shift = sh;
    nm.scale = sc;
    nm.mod_seg_stride = mseg;
    nm.rows = rows > 0 ? rows : M_;
    nm.D = D;
    nm.in_seg = Tl_;
    nm.in_stride = Tl_;
    nm.in_off = 0;
    return rmsnorm_mod(nm, x16_, s);
  };
  auto resid = [&](const bf16_t* A, long lda, const bf16_t* W, int K, const float* gate, long rows = 0) -> int {
    GemmParams g;
    g.A = A;
    g.lda = lda;
    g.W = W;
    g.ldw = K;
    g.out = x_;
    g.ldo = D;
    g.gate = gate;
    g.gate_seg_stride = mseg;
    g.rows_per_seg = Tl_;
    g.M = (int)(rows > 0 ? rows : M_);
    g.N = D;
    g.K = K;
    return gemm(g, epi_resid(), s);
  };
  const long rope_off = (long)sp_rank_ * Tl_ * 128;  // table rows of the tokens held here

  // --- self attention ---
  const bool probe_sa = Msa == M_;  // the kernel probes average full-batch launches only
  if (norm(b.norm1, shift_sa, scale_sa, nullptr, 0, nullptr, 0, Msa)) return 1;
  {
    GemmParams g;
    g.A = nbuf_;
    g.lda = D;
    g.W = b.qkv_w;
    g.ldw = D;
    g.bias = b.qkv_b;
    g.out = qkv_;
    g.ldo = 3L * D;
    if (w_prefetch()) {  // the proj weights, read after the attention, into the Infinity Cache
      g.pf = b.proj_w;
      g.pf_bytes = (long)D * D * 2;
    }
    g.M = (int)Msa;
    g.N = 3 * D;
    g.K = D;
    // RoPE + QK-norm of the q and k heads ("(k h d)" layout, model.py:163) in the GEMM epilogue
    g.rope = rope_axes();
    g.norm_cols = 2 * D;
    g.rope_cols = cfg.use_rope ? 2 * D : 0;
    if (probe_sa && probe_begin(s, FLITE_PROBE_GEMM_QKV)) return 1;
    if (gemm(g, fuse_qk_norm() ? EPI_QKV_NORM_BF16 : EPI_STORE_BF16, s)) return 1;
    if (probe_sa && probe_end(s, FLITE_PROBE_GEMM_QKV)) return 1;
  }
  if (!fuse_qk_norm()) {
    RopeNormParams rn;
    rn.x = qkv_;
    rn.ldx = 3L * D;
    rn.rows = Msa;
    rn.heads = 2 * H;  // q heads then k heads ("(k h d)" layout, model.py:163)
    rn.rope_heads = cfg.use_rope ? 2 * H : 0;
    rn.cos = cos_ + rope_off;
    rn.sin = sin_ + rope_off;
    rn.tokens_per_seq = Tl_;
    if (rope_qknorm(rn, s)) return 1;
  }
  // the ring needs a key in every rank's block ((N - 1) Tl < T); otherwise the all-gather exchange runs
  const bool sp_rng = sp_n_ > 1 && sp_ring_ && (long)(sp_n_ - 1) * Tl_ < T_;
  const bool sp_ovl = sp_n_ > 1 && sp_overlap_ && !sp_rng;
  if (sp_n_ > 1 && !sp_ovl && !sp_rng && sp_gather_kv(s)) return 1;  // every key of the sequence on every rank
  {
    AttnParams a;
    a.q = qkv_;
    a.k = sp_n_ > 1 ? kv_full_ : qkv_ + D;
    a.v = sp_n_ > 1 ? kv_full_ + D : qkv_ + 2L * D;
    a.o = obuf_;
    a.q_row_stride = 3L * D;
    a.k_row_stride = a.v_row_stride = sp_n_ > 1 ? 2L * D : 3L * D;
    a.o_row_stride = D;
    a.q_head_stride = a.k_head_stride = a.v_head_stride = a.o_head_stride = HEAD_DIM;
    a.cu_q = cu_self_;
    a.cu_k = sp_n_ > 1 ? cu_full_ : cu_self_;
    a.B = Bsa;
    a.H = H;
    a.head_dim = HEAD_DIM;
    a.max_q = Tl_;
    a.max_k = T_;
    a.scale = 1.0f / sqrtf((float)HEAD_DIM);
    a.max_score = kQKNormScoreBound;
    a.split_ws = attn_ws_;
    a.split_ws_bytes = attn_ws_bytes_;
    if (probe_sa && probe_begin(s, FLITE_PROBE_ATTN_SELF)) return 1;
    if (sp_rng ? sp_ring_attention(s, a) : sp_ovl ? sp_self_attention(s, a) : attn_fwd(a, s)) return 1;
    if (probe_sa && probe_end(s, FLITE_PROBE_ATTN_SELF)) return 1;
  }
  if (resid(obuf_, D, b.proj_w, D, gate_sa, Msa)) return 1;
  for (long r0 = Msa; r0 < M_; r0 += Msa)  // the other CFG copies of the residual rows
    FLITE_HIP_CHECK(hipMemcpyAsync(xrow(r0), x_, (size_t)Msa * D * xbytes(), hipMemcpyDeviceToDevice, s));

  // --- cross attention (model.py:291-297) ---
  // The first ctx_uni_ sequences have uniform context (set_context): their rows take the step-invariant
  // x += gate_ca * c; the norm, the cross-q GEMM, the attention and the cross-proj run on the other rows only.
  // Nothing reads the collapsed rows of x before norm3, so their update x += gate_ca * c is deferred into norm3's
  // read of those rows (one 50 MB fp32 read-modify-write pass fewer per block; the same fma, bit for bit).
  // (the D = 3072 row kernel takes the update; other widths keep the separate pass here)
  const int U = b.cross ? ctx_uni_ : 0;
  const long r0 = (long)U * Tl_;
  const bool bc_defer = U > 0 && D == 3072;
  const float* bc_c = bc_defer ? ctx_c_ + (long)blk * B_ * D : nullptr;
  if (U > 0 && !bc_defer && ctx_bcast_resid(x_, x16_, ctx_c_ + (long)blk * B_ * D, gate_ca, mseg, Tl_, r0, D, s))
    return 1;
  if (b.cross && r0 < M_) {
    {
      NormModParams nm;
      if (norm_prefetch()) {
        nm.pf[0] = b.cq_w;
        nm.pf_bytes[0] = (long)D * D * 2;
      }
      nm.x = xrow(r0);
      nm.ldx = D;
      nm.y = nbuf_ + r0 * D;
      nm.ldy = D;
      nm.w = b.norm2;
      nm.shift = shift_ca + U * mseg;
      nm.scale = scale_ca + U * mseg;
      nm.mod_seg_stride = mseg;
      nm.rows = M_ - r0;
      nm.D = D;
      nm.in_seg = Tl_;
      nm.in_stride = Tl_;
      nm.in_off = 0;
      if (rmsnorm_mod(nm, x16_, s)) return 1;
    }
    GemmParams g;
    g.A = nbuf_ + r0 * D;
    g.lda = D;
    g.W = b.cq_w;
    g.ldw = D;
    g.bias = b.cq_b;
    g.out = qkv_ + r0 * D;
    g.ldo = D;
    if (w_prefetch()) {  // the cross-proj weights, read after the cross-attention
      g.pf = b.cproj_w;
      g.pf_bytes = (long)D * D * 2;
    }
    g.M = (int)(M_ - r0);
    g.N = D;
    g.K = D;
    g.norm_cols = D;  // query QK-norm (model.py:197) in the epilogue
    if (gemm(g, fuse_qk_norm() ? EPI_QKV_NORM_BF16 : EPI_STORE_BF16, s)) return 1;
    if (!fuse_qk_norm()) {
      RopeNormParams rn;
      rn.x = qkv_ + r0 * D;
      rn.ldx = D;
      rn.rows = M_ - r0;
      rn.heads = H;
      rn.rope_heads = 0;
      if (rope_qknorm(rn, s)) return 1;
    }
    AttnParams a;
    a.q = qkv_;
    a.k = ctx_kv_[blk];
    a.v = ctx_kv_[blk] + D;
    a.o = obuf_;
    a.q_row_stride = D;
    a.k_row_stride = a.v_row_stride = 2L * D;
    a.o_row_stride = D;
    a.q_head_stride = a.k_head_stride = a.v_head_stride = a.o_head_stride = HEAD_DIM;
    a.cu_q = cu_self_ + U;  // absolute row offsets: the collapsed sequences are skipped, nothing else moves
    a.cu_k = cu_ctx_ + U;
    a.B = B_ - U;
    a.H = H;
    a.head_dim = HEAD_DIM;
    a.max_q = Tl_;
    a.max_k = ctx_max_len_;
    a.scale = 1.0f / sqrtf((float)HEAD_DIM);
    a.max_score = kQKNormScoreBound;
    a.split_ws = attn_ws_;
    a.split_ws_bytes = attn_ws_bytes_;
    if (attn_fwd(a, s)) return 1;
    GemmParams c;
    c.A = obuf_ + r0 * D;
    c.lda = D;
    c.W = b.cproj_w;
    c.ldw = D;
    c.out = xrow(r0);
    c.ldo = D;
    c.gate = gate_ca + U * mseg;
    c.gate_seg_stride = mseg;
    c.rows_per_seg = Tl_;
    c.M = (int)(M_ - r0);
    c.N = D;
    c.K = D;
    if (gemm(c, epi_resid(), s)) return 1;
  }

  // --- SwiGLU MLP (model.py:299-301) ---
  if (norm(b.norm3, shift_mlp, scale_mlp, nullptr, 0, nullptr, 0, 0, bc_c, gate_ca, bc_defer ? r0 : 0)) return 1;
  {
    GemmParams g;
    g.A = nbuf_;
    g.lda = D;
    g.W = b.gate_w;
    g.W2 = b.up_w;
    g.ldw = D;
    g.out = hbuf_;
    g.ldo = F;
    g.M = (int)M_;
    g.N = 2 * F;
    g.K = D;
    if (probe_begin(s, FLITE_PROBE_GEMM_GATEUP)) return 1;
    if (gemm(g, EPI_SWIGLU_BF16, s)) return 1;
    if (probe_end(s, FLITE_PROBE_GEMM_GATEUP)) return 1;
  }
  if (probe_begin(s, FLITE_PROBE_GEMM_DOWN)) return 1;
  if (resid(hbuf_, F, b.down_w, F, gate_mlp)) return 1;
  if (probe_end(s, FLITE_PROBE_GEMM_DOWN)) return 1;
  return 0;
}

int DitEngine::alloc_fp8_act() {
  if (nbuf8_ != nullptr || x_ == nullptr) return 0;
  // + 256: a GEMM over rows [r0, M) (the uniform-context collapse, run_block_fp8) stages 256-row tiles of scales
  // from row r0 on, i.e. up to row r0 + mx_rows_pad(M - r0) <= M + 255
  mpad_ = mx_rows_pad(M_) + 256;
  const size_t sd = (size_t)(D / 128) * mpad_ * 4, sf = (size_t)(F / 128) * mpad_ * 4;
  if (alloc((void**)&nbuf8_, (size_t)M_ * D)) return 1;
  if (alloc((void**)&obuf8_, (size_t)M_ * D)) return 1;
  if (alloc((void**)&hbuf8_, (size_t)M_ * F)) return 1;
  if (alloc((void**)&nbuf8_s_, sd)) return 1;
  if (alloc((void**)&obuf8_s_, sd)) return 1;
  if (alloc((void**)&hbuf8_s_, sf)) return 1;
  // pad rows of the scale arrays are staged by the GEMM (256-row tiles) but never written: zero = 2^-127
  FLITE_HIP_CHECK(hipMemset(nbuf8_s_, 0, sd));
  FLITE_HIP_CHECK(hipMemset(obuf8_s_, 0, sd));
  FLITE_HIP_CHECK(hipMemset(hbuf8_s_, 0, sf));
  return 0;
}

int DitEngine::enable_fp8(hipStream_t s, bool on) {
  drop_graph();
  if (!on) {
    fp8_ = false;
    return 0;
  }
  FLITE_REQUIRE(sp_n_ == 1, "enable_fp8: not with sequence parallelism");
  {
    const char* un = getenv("FLITE_FP8_ATTN_UNFUSED");  // A/B switch: bf16 attention output + quant_rows_fp8
    attn_mx_ = !(un && un[0] == '1');
  }
  if (check_bound()) return 2;
  FLITE_REQUIRE(D % 128 == 0 && F % 128 == 0, "fp8: hidden and MLP widths must be multiples of 128");
  // always from the current bf16 weights: they may have changed while fp8 mode was off
  w8_stale_ = true;
  if (quantise_fp8(s)) return 1;
  fp8_ = true;
  return alloc_fp8_act();
}

int DitEngine::set_fp8_bf16_blocks(const int* blocks, int n) {
  FLITE_REQUIRE(n >= 0 && (n == 0 || blocks != nullptr), "set_fp8_bf16_blocks: bad block list");
  std::vector<char> keep(cfg.depth, 0);
  for (int i = 0; i < n; ++i) {
    FLITE_REQUIRE(blocks[i] >= 0 && blocks[i] < cfg.depth, "set_fp8_bf16_blocks: block index out of range");
    keep[blocks[i]] = 1;
  }
  drop_graph();  // a cached graph holds the old per-block choice
  fp8_bf16_blk_.swap(keep);
  return 0;
}

int DitEngine::set_fp8_classes(int mask) {
  FLITE_REQUIRE(mask >= 0 && mask <= FLITE_FP8_ALL, "set_fp8_gemm_classes: mask outside FLITE_FP8_ALL");
  if (mask != fp8_classes_) drop_graph();  // a cached graph holds the old choice
  fp8_classes_ = mask;
  return 0;
}

int DitEngine::set_fp8_block_classes(const int* masks, int n) {
  FLITE_REQUIRE(n == 0 || (masks != nullptr && n == cfg.depth),
                "set_fp8_block_classes: pass one mask per block (n = depth), or n = 0 to clear");
  std::vector<int> m(masks, masks + n);
  for (int v : m) FLITE_REQUIRE(v >= 0 && v <= FLITE_FP8_ALL, "set_fp8_block_classes: mask outside FLITE_FP8_ALL");
  drop_graph();  // a cached graph holds the old per-block choice
  fp8_blk_mask_.swap(m);
  return 0;
}

int DitEngine::set_residual_bf16(bool on) {
  if (on != x16_) drop_graph();  // a cached graph holds the other launch shapes
  x16_ = on;
  return 0;
}

int DitEngine::weights_updated(hipStream_t s) {
  w8_stale_ = true;
  ctx_stale_ = true;
  return fp8_ ? quantise_fp8(s) : 0;
}

// (Re)quantise every block GEMM weight into the engine's MXFP8 copies (allocated once; the sizes depend only on
// the config). Never called inside a graph capture: forward / sample call it before they launch anything.
int DitEngine::quantise_fp8(hipStream_t s) {
  if (!w8_stale_) return 0;
  if (check_bound()) return 2;
  const bool fresh = w8_.empty();
  if (fresh) w8_.resize(cfg.depth);
  auto buf = [&](uint8_t** p, size_t bytes) -> int {
    if (!fresh) return 0;
    FLITE_HIP_CHECK(hipMalloc((void**)p, bytes));
    w8_allocs_.push_back(*p);
    return 0;
  };
  // weight [rows, K] -> fp8 + scales [K/128][rows][4] (rows are multiples of 256 for every DiT weight)
  auto q = [&](const bf16_t* w, long rows, int K, uint8_t** d, uint8_t** sc) -> int {
    FLITE_REQUIRE(rows % 256 == 0, "fp8: weight rows must be a multiple of 256");
    if (buf(d, (size_t)rows * K) || buf(sc, (size_t)(K / 128) * rows * 4)) return 1;
    return quant_rows_fp8(w, K, rows, K, *d, K, *sc, rows, s);
  };
  // fused RoPE epilogue: the q/k rows of the qkv weight in rope_perm order (gemm_fp8 EPI8_QKV_NORM_BF16)
  const long perm_rows = (fuse_qk_norm() && cfg.use_rope) ? 2L * D : 0;
  for (int i = 0; i < cfg.depth; ++i) {
    const BlockW& b = w_.blocks[i];
    Fp8W& f = w8_[i];
    if (buf(&f.qkv, (size_t)3 * D * D) || buf(&f.qkv_s, (size_t)(D / 128) * 3 * D * 4) ||
        quant_rows_fp8_perm(b.qkv_w, D, 3L * D, D, f.qkv, D, f.qkv_s, 3L * D, perm_rows, s))
      return 1;
    if (q(b.proj_w, D, D, &f.proj, &f.proj_s) || q(b.down_w, D, F, &f.down, &f.down_s)) return 1;
    if (b.cross && (q(b.cq_w, D, D, &f.cq, &f.cq_s) || q(b.cproj_w, D, D, &f.cproj, &f.cproj_s))) return 1;
    if (buf(&f.gu, (size_t)2 * F * D) || buf(&f.gu_s, (size_t)(D / 128) * 2 * F * 4)) return 1;
    if (quant_gateup_fp8(b.gate_w, b.up_w, D, F, D, f.gu, f.gu_s, s)) return 1;
  }
  FLITE_HIP_CHECK(hipStreamSynchronize(s));
  w8_stale_ = false;
  ctx_c8_stale_ = true;
  return 0;
}

// The fp8 blocks' collapsed cross-attention rows need the collapsed-row offset r0 = U * Tl to keep the MXFP8 scale
// arrays 16-B aligned (gemm_fp8: scales + r0 * 4 bytes); otherwise those blocks run the full computation.
int DitEngine::uni_fp8() const { return ((long)ctx_uni_ * Tl_) % 4 == 0 ? ctx_uni_ : 0; }

// c8[blk][q] = MX(V row) . MX(Wproj)^T: the fp8 path's own cross-proj arithmetic on the attention output the
// collapse replaces (run_block_fp8). Runs before forward / sample launch any block, never inside a capture.
int DitEngine::collapse_fp8(hipStream_t s) {
  if (!ctx_c8_stale_) return 0;
  const int U = uni_fp8();
  for (int i = 0; i < cfg.depth && U > 0; ++i) {
    const BlockW& b = w_.blocks[i];
    if (!b.cross) continue;
    for (int q = 0; q < U; ++q)
      FLITE_HIP_CHECK(hipMemcpyAsync(ctx_vrow_ + (long)q * D, ctx_kv_[i] + (long)ctx_row0_[q] * 2 * D + D,
                                     (size_t)D * 2, hipMemcpyDeviceToDevice, s));
    FLITE_REQUIRE(U <= vrow8_rows_pad_, "collapse_fp8: more collapsed sequences than scale rows");
    if (quant_rows_fp8(ctx_vrow_, D, U, D, ctx_vrow8_, D, ctx_vrow8_s_, vrow8_rows_pad_, s)) return 1;
    float* c8 = ctx_c8_ + (long)i * B_ * D;
    FLITE_HIP_CHECK(hipMemsetAsync(c8, 0, (size_t)U * D * 4, s));
    GemmFp8Params g;
    g.A = ctx_vrow8_;
    g.lda = D;
    g.As = ctx_vrow8_s_;
    g.a_rows_pad = vrow8_rows_pad_;
    g.W = w8_[i].cproj;
    g.ldw = D;
    g.Ws = w8_[i].cproj_s;
    g.w_rows_pad = D;
    g.out = c8;
    g.ldo = D;
    g.rows_per_seg = 1;  // no gate: c8 += acc
    g.M = U;
    g.N = D;
    g.K = D;
    if (gemm_fp8(g, EPI8_RESID_F32, s)) return 1;
  }
  ctx_c8_stale_ = false;
  return 0;
}

// One DiTBlock in fp8 (flite_dit_enable_fp8): the six block GEMMs on MXFP8 operands; attention, RoPE / QK-norm,
// the residual stream and the modulation stay as in run_block.
int DitEngine::run_block_fp8(hipStream_t s, int blk, const float* mod, long mseg, int cm) {
  const BlockW& b = w_.blocks[blk];
  const Fp8W& q = w8_[blk];
  const float *shift_sa = mod, *scale_sa = mod + D, *gate_sa = mod + 2L * D;
  const float *shift_ca = mod + 3L * D, *scale_ca = mod + 4L * D, *gate_ca = mod + 5L * D;
  const float *shift_mlp = mod + 6L * D, *scale_mlp = mod + 7L * D, *gate_mlp = mod + 8L * D;
  const int Bsa = sa_seqs_ > 0 ? sa_seqs_ : B_;  // as run_block: block 0 of a CFG batch, self-attention once
  const long Msa = (long)Bsa * Tl_;
  const bool probe_sa = Msa == M_;
  auto norm8 = [&](const bf16_t* w, const float* sh, const float* sc, long rows = 0, long r0 = 0,
                    const float* bc_c = nullptr, long bc_rows = 0) -> int {
    NormModParams nm;  // rows [r0, r0 + rows) of x; r0 % 4 == 0 keeps the scale rows 16-B aligned (uni_fp8)
    nm.x = xrow(r0);
    nm.ldx = D;
    nm.y8 = nbuf8_ + r0 * D;
    nm.ldy = D;
    nm.ysc = nbuf8_s_ + r0 * 4;
    nm.ysc_rows_pad = mpad_;
    nm.w = w;
    nm.shift = sh;
    nm.scale = sc;
    nm.mod_seg_stride = mseg;
    nm.rows = rows > 0 ? rows : M_ - r0;
    nm.D = D;
    nm.in_seg = Tl_;
    nm.in_stride = Tl_;
    nm.in_off = 0;
    nm.bc_c = bc_c;  // the collapsed rows' deferred update (norm3 only; run_block's note)
    nm.bc_gate = gate_ca;
    nm.bc_gate_stride = mseg;
    nm.bc_rows = bc_rows;
    nm.bc_rows_per_seg = Tl_;
    return rmsnorm_mod(nm, x16_, s);
  };
  auto g8 = [&](const uint8_t* A, const uint8_t* As, const uint8_t* W, const uint8_t* Ws, long w_rows, int N, int K,
                const bf16_t* bias, int epi, void* out, long ldo, const float* gate, int norm_cols = 0,
                int rope_cols = 0, long rows = 0) -> int {
    GemmFp8Params g;
    g.A = A;
    g.lda = K;
    g.As = As;
    g.a_rows_pad = mpad_;
    g.W = W;
    g.ldw = K;
    g.Ws = Ws;
    g.w_rows_pad = w_rows;
    g.bias = bias;
    g.out = out;
    g.ldo = ldo;
    g.gate = gate;
    g.gate_seg_stride = mseg;
    g.rows_per_seg = Tl_;
    g.M = (int)(rows > 0 ? rows : M_);
    g.N = N;
    g.K = K;
    if (epi == EPI8_SWIGLU_FP8) {
      g.out_sc = hbuf8_s_;
      g.out_rows_pad = mpad_;
    }
    if (epi == EPI8_QKV_NORM_BF16) {
      g.norm_cols = norm_cols;
      g.rope_cols = rope_cols;
      g.rope = rope_axes();
    }
    static const bool no_sk = getenv("FLITE_GEMM_NO_STREAM_K") != nullptr;  // A/B switch, as gemm()
    g.sk_ws = no_sk ? nullptr : sk_ws_;
    g.sk_flags = no_sk ? nullptr : sk_flags_;
    return gemm_fp8(g, epi, s);
  };
  auto attn = [&](bool mx, const bf16_t* qp, long ldq, const bf16_t* kp, const bf16_t* vp, long ldkv, const int* cu_k,
                  int max_k, int nseq = 0, int seq0 = 0) -> int {
    AttnParams a;
    a.q = qp;
    a.k = kp;
    a.v = vp;
    a.o = obuf_;
    a.q_row_stride = ldq;
    a.k_row_stride = a.v_row_stride = ldkv;
    a.o_row_stride = D;
    a.q_head_stride = a.k_head_stride = a.v_head_stride = a.o_head_stride = HEAD_DIM;
    a.cu_q = cu_self_ + seq0;
    a.cu_k = cu_k;
    a.B = nseq > 0 ? nseq : B_;
    a.H = H;
    a.head_dim = HEAD_DIM;
    a.max_q = Tl_;
    a.max_k = max_k;
    a.scale = 1.0f / sqrtf((float)HEAD_DIM);
    a.max_score = kQKNormScoreBound;
    a.split_ws = attn_ws_;
    a.split_ws_bytes = attn_ws_bytes_;
    if (mx) {  // the proj GEMM's MXFP8 A operand straight from the attention epilogue
      a.o8 = obuf8_;
      a.o8_scale = obuf8_s_;
      a.o8_rows_pad = mpad_;
    }
    return attn_fwd(a, s);
  };
  auto qk_norm = [&](long ldx, int heads, int rope_heads, long rows = 0, long r0 = 0) -> int {
    RopeNormParams rn;
    rn.x = qkv_ + r0 * ldx;
    rn.ldx = ldx;
    rn.rows = rows > 0 ? rows : M_;
    rn.heads = heads;
    rn.rope_heads = rope_heads;
    if (rope_heads > 0) {
      rn.cos = cos_;
      rn.sin = sin_;
      rn.tokens_per_seq = Tl_;
    }
    return rope_qknorm(rn, s);
  };
  // the GEMM classes on MXFP8 (flite_dit_set_fp8_gemm_classes); every other class runs its bf16 GEMM, and each
  // activation is produced in the format its consumer takes
  const bool f_qkv = cm & FLITE_FP8_QKV, f_proj = cm & FLITE_FP8_PROJ, f_cq = cm & FLITE_FP8_CROSS_Q,
             f_cproj = cm & FLITE_FP8_CROSS_PROJ, f_gu = cm & FLITE_FP8_GATE_UP, f_down = cm & FLITE_FP8_DOWN;
  auto norm16 = [&](const bf16_t* w, const float* sh, const float* sc, long rows = 0, long r0 = 0,
                    const float* bc_c = nullptr, long bc_rows = 0) -> int {
    NormModParams nm;
    nm.x = xrow(r0);
    nm.ldx = D;
    nm.y = nbuf_ + r0 * D;
    nm.ldy = D;
    nm.w = w;
    nm.shift = sh;
    nm.scale = sc;
    nm.mod_seg_stride = mseg;
    nm.rows = rows > 0 ? rows : M_ - r0;
    nm.D = D;
    nm.in_seg = Tl_;
    nm.in_stride = Tl_;
    nm.in_off = 0;
    nm.bc_c = bc_c;
    nm.bc_gate = gate_ca;
    nm.bc_gate_stride = mseg;
    nm.bc_rows = bc_rows;
    nm.bc_rows_per_seg = Tl_;
    return rmsnorm_mod(nm, x16_, s);
  };
  auto g16 = [&](const bf16_t* A, const bf16_t* W, int N, const bf16_t* bias, int epi, void* out, long ldo,
                 const float* gate, int norm_cols = 0, int rope_cols = 0, long rows = 0) -> int {
    GemmParams g;
    g.A = A;
    g.lda = D;
    g.W = W;
    g.ldw = D;
    g.bias = bias;
    g.out = out;
    g.ldo = ldo;
    g.gate = gate;
    g.gate_seg_stride = mseg;
    g.rows_per_seg = Tl_;
    g.M = (int)(rows > 0 ? rows : M_);
    g.N = N;
    g.K = D;
    g.rope = rope_axes();
    g.norm_cols = norm_cols;
    g.rope_cols = rope_cols;
    return gemm(g, epi, s);
  };
  const bool fused = fuse_qk_norm();  // RoPE + QK-norm in the GEMM epilogue (the weights were quantised to match)
  // --- self attention ---
  if (f_qkv ? norm8(b.norm1, shift_sa, scale_sa, Msa) : norm16(b.norm1, shift_sa, scale_sa, Msa)) return 1;
  if (probe_sa && probe_begin(s, FLITE_PROBE_GEMM_QKV)) return 1;
  if (f_qkv) {
    if (g8(nbuf8_, nbuf8_s_, q.qkv, q.qkv_s, 3L * D, 3 * D, D, b.qkv_b, fused ? EPI8_QKV_NORM_BF16 : EPI8_STORE_BF16,
           qkv_, 3L * D, nullptr, 2 * D, cfg.use_rope ? 2 * D : 0, Msa))
      return 1;
  } else if (g16(nbuf_, b.qkv_w, 3 * D, b.qkv_b, fused ? EPI_QKV_NORM_BF16 : EPI_STORE_BF16, qkv_, 3L * D, nullptr,
                 2 * D, cfg.use_rope ? 2 * D : 0, Msa)) {
    return 1;
  }
  if (probe_sa && probe_end(s, FLITE_PROBE_GEMM_QKV)) return 1;
  if (!fused && qk_norm(3L * D, 2 * H, cfg.use_rope ? 2 * H : 0, Msa)) return 1;
  if (probe_sa && probe_begin(s, FLITE_PROBE_ATTN_SELF)) return 1;
  if (attn(f_proj && attn_mx_, qkv_, 3L * D, qkv_ + D, qkv_ + 2L * D, 3L * D, cu_self_, Tl_, Bsa)) return 1;
  if (probe_sa && probe_end(s, FLITE_PROBE_ATTN_SELF)) return 1;
  if (f_proj) {
    if (!attn_mx_ && quant_rows_fp8(obuf_, D, Msa, D, obuf8_, D, obuf8_s_, mpad_, s)) return 1;
    if (g8(obuf8_, obuf8_s_, q.proj, q.proj_s, D, D, D, nullptr, epi8_resid(), x_, D, gate_sa, 0, 0, Msa)) return 1;
  } else if (g16(obuf_, b.proj_w, D, nullptr, epi_resid(), x_, D, gate_sa, 0, 0, Msa)) {
    return 1;
  }
  for (long r0 = Msa; r0 < M_; r0 += Msa)  // the other CFG copies of the residual rows
    FLITE_HIP_CHECK(hipMemcpyAsync(xrow(r0), x_, (size_t)Msa * D * xbytes(), hipMemcpyDeviceToDevice, s));
  // --- cross attention --- (uniform-context collapse as in run_block: the first U sequences' rows take
  // x += gate_ca * c8, the rest run the sub-block from row r0 on)
  // (an MXFP8 cross-q or cross-proj keeps the collapsed rows' r0 16-B aligned in the scale arrays: uni_fp8; a bf16
  // cross-proj takes the bf16 path's c = V . Wproj^T)
  const bool f_ca = f_cq || f_cproj;
  const int U = b.cross ? (f_ca ? uni_fp8() : ctx_uni_) : 0;
  const long r0 = (long)U * Tl_, rows = M_ - r0;
  // deferred into norm3's read of the collapsed rows at D = 3072, as in run_block
  const bool bc_defer = U > 0 && D == 3072;
  const float* bc_c = bc_defer ? (f_cproj ? ctx_c8_ : ctx_c_) + (long)blk * B_ * D : nullptr;
  if (U > 0 && !bc_defer &&
      ctx_bcast_resid(x_, x16_, (f_cproj ? ctx_c8_ : ctx_c_) + (long)blk * B_ * D, gate_ca, mseg, Tl_, r0, D, s))
    return 1;
  if (b.cross && rows > 0) {
    if (f_cq ? norm8(b.norm2, shift_ca + U * mseg, scale_ca + U * mseg, rows, r0)
             : norm16(b.norm2, shift_ca + U * mseg, scale_ca + U * mseg, rows, r0))
      return 1;
    if (f_cq) {
      if (g8(nbuf8_ + r0 * D, nbuf8_s_ + r0 * 4, q.cq, q.cq_s, D, D, D, b.cq_b,
             fused ? EPI8_QKV_NORM_BF16 : EPI8_STORE_BF16, qkv_ + r0 * D, D, nullptr, D, 0, rows))
        return 1;
    } else if (g16(nbuf_ + r0 * D, b.cq_w, D, b.cq_b, fused ? EPI_QKV_NORM_BF16 : EPI_STORE_BF16, qkv_ + r0 * D, D,
                   nullptr, D, 0, rows)) {
      return 1;
    }
    if (!fused && qk_norm(D, H, 0, rows, r0)) return 1;
    if (attn(f_cproj && attn_mx_, qkv_, D, ctx_kv_[blk], ctx_kv_[blk] + D, 2L * D, cu_ctx_ + U, ctx_max_len_, B_ - U,
             U))
      return 1;
    if (f_cproj) {
      if (!attn_mx_ && quant_rows_fp8(obuf_ + r0 * D, D, rows, D, obuf8_ + r0 * D, D, obuf8_s_ + r0 * 4, mpad_, s))
        return 1;
      if (g8(obuf8_ + r0 * D, obuf8_s_ + r0 * 4, q.cproj, q.cproj_s, D, D, D, nullptr, epi8_resid(), xrow(r0), D,
             gate_ca + U * mseg, 0, 0, rows))
        return 1;
    } else if (g16(obuf_ + r0 * D, b.cproj_w, D, nullptr, epi_resid(), xrow(r0), D, gate_ca + U * mseg, 0, 0,
                   rows)) {
      return 1;
    }
  }
  // --- SwiGLU MLP --- (an fp8 gate/up writes the SwiGLU output as MXFP8 for an fp8 down, bf16 for a bf16 down; a
  // bf16 gate/up feeding an fp8 down is quantised by quant_rows_fp8)
  if (f_gu ? norm8(b.norm3, shift_mlp, scale_mlp, 0, 0, bc_c, bc_defer ? r0 : 0)
           : norm16(b.norm3, shift_mlp, scale_mlp, 0, 0, bc_c, bc_defer ? r0 : 0))
    return 1;
  if (probe_begin(s, FLITE_PROBE_GEMM_GATEUP)) return 1;
  if (f_gu) {
    if (f_down ? g8(nbuf8_, nbuf8_s_, q.gu, q.gu_s, 2L * F, 2 * F, D, nullptr, EPI8_SWIGLU_FP8, hbuf8_, F, nullptr)
               : g8(nbuf8_, nbuf8_s_, q.gu, q.gu_s, 2L * F, 2 * F, D, nullptr, EPI8_SWIGLU_BF16, hbuf_, F, nullptr))
      return 1;
  } else {
    GemmParams g;
    g.A = nbuf_;
    g.lda = D;
    g.W = b.gate_w;
    g.W2 = b.up_w;
    g.ldw = D;
    g.out = hbuf_;
    g.ldo = F;
    g.M = (int)M_;
    g.N = 2 * F;
    g.K = D;
    if (gemm(g, EPI_SWIGLU_BF16, s)) return 1;
    if (f_down && quant_rows_fp8(hbuf_, F, M_, F, hbuf8_, F, hbuf8_s_, mpad_, s)) return 1;
  }
  if (probe_end(s, FLITE_PROBE_GEMM_GATEUP)) return 1;
  if (probe_begin(s, FLITE_PROBE_GEMM_DOWN)) return 1;
  if (f_down) {
    if (g8(hbuf8_, hbuf8_s_, q.down, q.down_s, D, D, F, nullptr, epi8_resid(), x_, D, gate_mlp)) return 1;
  } else {
    GemmParams g;
    g.A = hbuf_;
    g.lda = F;
    g.W = b.down_w;
    g.ldw = F;
    g.out = x_;
    g.ldo = D;
    g.gate = gate_mlp;
    g.gate_seg_stride = mseg;
    g.rows_per_seg = Tl_;
    g.M = (int)M_;
    g.N = D;
    g.K = F;
    if (gemm(g, epi_resid(), s)) return 1;
  }
  if (probe_end(s, FLITE_PROBE_GEMM_DOWN)) return 1;
  return 0;
}

int DitEngine::set_probe(int kind, int max_pairs) {
  for (hipEvent_t e : probe_ev_) hipEventDestroy(e);
  probe_ev_.clear();
  probe_n_ = 0;
  probe_kind_ = kind;
  drop_graph();  // a cached graph holds (or lacks) the old probe nodes
  if (kind < 0) return 0;
  FLITE_REQUIRE(max_pairs > 0 && max_pairs <= 100000, "set_probe: bad max_pairs");
  probe_ev_.resize(2 * (size_t)max_pairs);
  for (auto& e : probe_ev_) FLITE_HIP_CHECK(hipEventCreate(&e));
  return 0;
}

int DitEngine::probe_begin(hipStream_t s, int kind) {
  if (kind != probe_kind_ || probe_n_ * 2 + 1 >= (int)probe_ev_.size()) return 0;
  FLITE_HIP_CHECK(hipEventRecord(probe_ev_[2 * probe_n_], s));
  return 0;
}

int DitEngine::probe_end(hipStream_t s, int kind) {
  if (kind != probe_kind_ || probe_n_ * 2 + 1 >= (int)probe_ev_.size()) return 0;
  FLITE_HIP_CHECK(hipEventRecord(probe_ev_[2 * probe_n_ + 1], s));
  ++probe_n_;
  return 0;
}

int DitEngine::read_probe(float* ms, int cap, int* n) {
  *n = 0;
  for (int i = 0; i < probe_n_ && i < cap; ++i) {
    FLITE_HIP_CHECK(hipEventSynchronize(probe_ev_[2 * i + 1]));
    FLITE_HIP_CHECK(hipEventElapsedTime(&ms[i], probe_ev_[2 * i], probe_ev_[2 * i + 1]));
    *n = i + 1;
  }
  return 0;
}

int DitEngine::forward(hipStream_t s, const void* lat, bool lat_bf16, int Bi, int dup, int t_row0, int t_row_step) {
  FLITE_REQUIRE(x_ != nullptr, "forward: call prepare first");
  FLITE_REQUIRE(Bi * dup == B_, "forward: batch does not match the prepared workspace");
  FLITE_REQUIRE(nseq_ctx_ == B_, "forward: set_context must be called for this batch");
  FLITE_REQUIRE(!ctx_stale_, "forward: context K/V cache is stale (weights changed since set_context, or it "
                "failed): set the context again");
  FLITE_REQUIRE(t_row0 >= 0 && t_row0 + (B_ - 1) * t_row_step < nt_, "forward: timestep rows out of range");
  FLITE_REQUIRE(sp_n_ == 1 || (sp_kv_send_ && sp_kv_recv_ && sp_out_send_ && sp_out_recv_),
                "forward: sequence parallelism needs its exchange buffers (flite_dit_sp_bind_buffers)");
  if (fp8_ && w8_stale_ && quantise_fp8(s)) return 1;  // a weight was rebound since the fp8 copies were made
  if (fp8_ && collapse_fp8(s)) return 1;
  const int cpp = C * P * P;
  // patch embed (model.py:533) straight into the residual stream after the registers (model.py:535)
  if (patchify(lat, lat_bf16, patches_, Bi, C, Hl_, Wl_, P, dup, s)) return 1;
  if (sp_n_ > 1) {
    // rows [r0, r0 + Tl) of each sequence: patches [p0, p1) land at local rows p + R - r0
    const int r0 = sp_rank_ * Tl_, t_hi = std::min(T_, r0 + Tl_);
    const int p0 = std::max(r0 - R, 0), p1 = t_hi - R;
    if (t_hi < r0 + Tl_)  // padding rows of the last rank: keep them finite
      FLITE_HIP_CHECK(hipMemset2DAsync(xrow(t_hi - r0), (size_t)Tl_ * D * xbytes(), 0,
                                       (size_t)(r0 + Tl_ - t_hi) * D * xbytes(), B_, s));
    for (int b = 0; b < B_ && p1 > p0; ++b) {
      GemmParams g;
      g.A = patches_ + ((long)b * HW_ + p0) * cpp;
      g.lda = cpp;
      g.W = w_.patch_w;
      g.ldw = cpp;
      g.bias = w_.patch_b;
      g.out = xrow((long)b * Tl_ + (p0 + R - r0));
      g.ldo = D;
      g.M = p1 - p0;
      g.N = D;
      g.K = cpp;
      if (gemm(g, x16_ ? EPI_STORE_BF16 : EPI_STORE_F32, s)) return 1;
    }
    if (r0 == 0 && fill_registers(x_, x16_, w_.registers, B_, Tl_, R, D, s)) return 1;
  } else {
    GemmParams g;
    g.A = patches_;
    g.lda = cpp;
    g.W = w_.patch_w;
    g.ldw = cpp;
    g.bias = w_.patch_b;
    g.out = x_;
    g.ldo = D;
    g.M = B_ * HW_;
    g.N = D;
    g.K = cpp;
    g.out_seg = HW_;
    g.out_seg_stride = T_;
    g.out_seg_off = R;
    if (gemm(g, x16_ ? EPI_STORE_BF16 : EPI_STORE_F32, s)) return 1;
    if (fill_registers(x_, x16_, w_.registers, B_, T_, R, D, s)) return 1;
  }
  // use_rope = False: x + positional_embedding[:, :T] over the register + patch rows (model.py:546)
  if (!cfg.use_rope && add_pos_embed(x_, x16_, w_.pos_emb, B_, T_, D, s)) return 1;
  const long mseg = (long)t_row_step * mod_t_stride_;
  for (int i = 0; i < cfg.depth; ++i) {
    const float* mod = mod_ + (long)t_row0 * mod_t_stride_ + (cfg.per_block_adaln ? (long)i * 9 * D : 0);
    char name[32];
    snprintf(name, sizeof(name), "flite.block.%d", i);
    RoctxRange range(name);
    // CFG batch (dup copies of each latent, one timestep row): the copies' residual streams agree until block 0's
    // cross-attention, so block 0's self-attention sub-block runs once per image instead of once per copy (one
    // rank; bf16 and MXFP8 paths)
    sa_seqs_ = (i == 0 && dup > 1 && t_row_step == 0 && sp_n_ == 1 && cfg_dedup()) ? Bi : 0;
    const int cm = i < (int)fp8_blk_mask_.size() ? fp8_blk_mask_[i] : fp8_classes_;  // this block's MXFP8 classes
    const bool blk8 = fp8_ && cm != 0 && !(i < (int)fp8_bf16_blk_.size() && fp8_bf16_blk_[i]);
    const int rc = blk8 ? run_block_fp8(s, i, mod, mseg, cm) : run_block(s, i, mod, mseg);
    sa_seqs_ = 0;
    if (rc) return 1;
  }
  // final stage (model.py:575-581): drop registers, RMSNorm (fp32 weight multiply), modulate, project
  {
    NormModParams nm;
    nm.x = x_;
    nm.ldx = D;
    nm.y = nbuf_;
    nm.ldy = D;
    nm.w = cfg.train_bias_and_rms ? w_.fnorm : nullptr;
    nm.shift = fmod_ + (long)t_row0 * 2 * D;
    nm.scale = fmod_ + (long)t_row0 * 2 * D + D;
    nm.mod_seg_stride = (long)t_row_step * 2 * D;
    // sequence parallel: every row held here (registers and padding included, dropped by the gather)
    const bool sp = sp_n_ > 1;
    nm.rows = sp ? M_ : (long)B_ * HW_;
    nm.D = D;
    nm.in_seg = sp ? Tl_ : HW_;
    nm.in_stride = sp ? Tl_ : T_;
    nm.in_off = sp ? 0 : R;
    if (rmsnorm_mod(nm, x16_, s)) return 1;
    GemmParams g;
    g.A = nbuf_;
    g.lda = D;
    g.W = w_.fproj_w;
    g.ldw = D;
    g.bias = w_.fproj_b;
    g.out = sp ? sp_out_send_ : fout_;
    g.ldo = cpp;
    g.M = sp ? (int)M_ : B_ * HW_;
    g.N = cpp;
    g.K = D;
    if (gemm(g, EPI_STORE_F32, s)) return 1;
    if (sp && sp_gather_out(s)) return 1;
  }
  return 0;
}

// K/V rows of this rank -> every rank's, reordered into whole sequences [B][T][2D] (kv_full_)
int DitEngine::sp_gather_kv(hipStream_t s) {
  const size_t row = 2 * (size_t)D * 2;
  FLITE_HIP_CHECK(hipMemcpy2DAsync(sp_kv_send_, row, qkv_ + D, 3 * (size_t)D * 2, row, M_, hipMemcpyDeviceToDevice, s));
  FLITE_REQUIRE(sp_fn_(sp_user_, 0, (void*)s) == 0, "sequence parallel: K/V exchange failed");
  for (int q = 0; q < sp_n_; ++q) {
    const int valid = std::min(T_, (q + 1) * Tl_) - q * Tl_;
    if (valid <= 0) continue;
    FLITE_HIP_CHECK(hipMemcpy2DAsync(kv_full_ + (long)q * Tl_ * 2 * D, (size_t)T_ * row,
                                     sp_kv_recv_ + (long)q * M_ * 2 * D, (size_t)Tl_ * row, (size_t)valid * row, B_,
                                     hipMemcpyDeviceToDevice, s));
  }
  return 0;
}

// Self-attention of this rank's query rows with the K/V exchange overlapped (the ring
// idea with one all-gather). The K/V rows go to the send buffer, the exchange runs on xstream_ while the
// attention over the rank's OWN keys runs on s, leaving the partial (O, l) in fp32; then the other ranks' rows
// are packed per sequence (rank order, own block skipped) and a second launch over them adds the partial and
// normalises. The bounded softmax has a fixed shift, so the two partial sums add exactly as one pass would
// (up to fp32 summation order). `a` is the whole-sequence parameter set of run_block.
int DitEngine::sp_self_attention(hipStream_t s, AttnParams a) {
  const size_t row = 2 * (size_t)D * 2;
  FLITE_HIP_CHECK(hipMemcpy2DAsync(sp_kv_send_, row, qkv_ + D, 3 * (size_t)D * 2, row, M_, hipMemcpyDeviceToDevice, s));
  FLITE_HIP_CHECK(hipEventRecord(ev_kv_, s));
  // (1) own keys, straight from the qkv rows (the last rank's padding rows excluded by k_end)
  AttnParams l = a;
  l.k = qkv_ + D;
  l.v = qkv_ + 2L * D;
  l.k_row_stride = l.v_row_stride = 3L * D;
  l.cu_k = cu_self_;
  l.k_end = kend_loc_;
  l.max_k = Tl_;
  l.part_mode = 1;
  l.part_o = part_o_;
  l.part_l = part_l_;
  if (attn_fwd(l, s)) return 1;
  // (2) the exchange, on the side stream (an RCCL all-gather returns at once; a host-staged one blocks here
  // while (1) runs)
  FLITE_HIP_CHECK(hipStreamWaitEvent(xstream_, ev_kv_, 0));
  FLITE_REQUIRE(sp_fn_(sp_user_, 0, (void*)xstream_) == 0, "sequence parallel: K/V exchange failed");
  FLITE_HIP_CHECK(hipEventRecord(ev_x_, xstream_));
  FLITE_HIP_CHECK(hipStreamWaitEvent(s, ev_x_, 0));
  // (3) the other ranks' rows, packed per sequence: [B][T - v][2D]
  const int v = std::max(0, std::min(T_, (sp_rank_ + 1) * Tl_) - sp_rank_ * Tl_);
  const long rem = T_ - v;
  for (int q = 0; q < sp_n_; ++q) {
    if (q == sp_rank_) continue;
    const int valid = std::min(T_, (q + 1) * Tl_) - q * Tl_;
    if (valid <= 0) continue;
    const long off = (long)q * Tl_ - (q > sp_rank_ ? v : 0);
    FLITE_HIP_CHECK(hipMemcpy2DAsync(kv_full_ + off * 2 * D, (size_t)rem * row, sp_kv_recv_ + (long)q * M_ * 2 * D,
                                     (size_t)Tl_ * row, (size_t)valid * row, B_, hipMemcpyDeviceToDevice, s));
  }
  // (4) remote keys, adding the partial of (1)
  AttnParams r = a;
  r.k = kv_full_;
  r.v = kv_full_ + D;
  r.k_row_stride = r.v_row_stride = 2L * D;
  r.cu_k = cu_rem_;
  r.max_k = (int)rem;
  r.part_mode = 2;
  r.part_o = part_o_;
  r.part_l = part_l_;
  return attn_fwd(r, s);
}

// Self-attention of this rank's query rows over a ring of K/V blocks (ring attention over T):
// step 0 attends to the rank's own keys while the first shift (own block -> rank + 1, rank - 1's block -> ring
// slot 0) runs on xstream_; step j attends to the block of rank (r - j) mod N in slot (j - 1) & 1 while shift j + 1
// forwards that block and receives the next into the other slot. Every step but the last leaves the unnormalised
// partial (O, l) (attention part_mode 1 / 3); the last adds it and normalises (part_mode 2). The bounded softmax's
// fixed shift makes the partials add exactly, so no (m, l) rescale is needed. A slot is overwritten only after the
// attention that read it (ev_used_). Per step each rank sends and receives one block (2 x Tl x D bf16 per
// sequence): N - 1 neighbour transfers over one xGMI link each, instead of an all-gather.
int DitEngine::sp_ring_attention(hipStream_t s, AttnParams a) {
  const size_t row = 2 * (size_t)D * 2;
  const int N = sp_n_;
  bf16_t* slot[2] = {sp_kv_recv_, sp_kv_recv_ + M_ * 2 * D};  // kv_recv holds N >= 2 blocks: two ring slots
  FLITE_HIP_CHECK(hipMemcpy2DAsync(sp_kv_send_, row, qkv_ + D, 3 * (size_t)D * 2, row, M_, hipMemcpyDeviceToDevice, s));
  FLITE_HIP_CHECK(hipEventRecord(ev_kv_, s));
  // shift 1 on the side stream: own block -> rank + 1, rank - 1's block -> slot 0
  FLITE_HIP_CHECK(hipStreamWaitEvent(xstream_, ev_kv_, 0));
  FLITE_REQUIRE(sp_fn_(sp_user_, 2, (void*)xstream_) == 0, "sequence parallel: ring shift failed");
  FLITE_HIP_CHECK(hipEventRecord(ev_ring_[0], xstream_));
  // step 0: own keys, straight from the qkv rows
  AttnParams l = a;
  l.k = qkv_ + D;
  l.v = qkv_ + 2L * D;
  l.k_row_stride = l.v_row_stride = 3L * D;
  l.cu_k = cu_self_;
  l.k_end = kend_loc_;
  l.max_k = Tl_;
  l.part_mode = 1;
  l.part_o = part_o_;
  l.part_l = part_l_;
  if (attn_fwd(l, s)) return 1;
  for (int j = 1; j < N; ++j) {
    const int cur = (j - 1) & 1;
    FLITE_HIP_CHECK(hipStreamWaitEvent(s, ev_ring_[cur], 0));  // block of rank (r - j) mod N has landed
    if (j + 1 < N) {
      // shift j + 1: forward the block in `cur`, receive into the other slot once step j - 1 has read it
      if (j >= 2) FLITE_HIP_CHECK(hipStreamWaitEvent(xstream_, ev_used_[j & 1], 0));
      FLITE_REQUIRE(sp_fn_(sp_user_, 2 + j, (void*)xstream_) == 0, "sequence parallel: ring shift failed");
      FLITE_HIP_CHECK(hipEventRecord(ev_ring_[j & 1], xstream_));
    }
    const int q = ((sp_rank_ - j) % N + N) % N;
    AttnParams r = a;
    r.k = slot[cur];
    r.v = slot[cur] + D;
    r.k_row_stride = r.v_row_stride = 2L * D;
    r.cu_k = cu_self_;
    r.k_end = kend_all_ + (long)q * B_;
    r.max_k = Tl_;
    r.part_mode = j + 1 < N ? 3 : 2;
    r.part_o = part_o_;
    r.part_l = part_l_;
    if (attn_fwd(r, s)) return 1;
    FLITE_HIP_CHECK(hipEventRecord(ev_used_[cur], s));
  }
  return 0;
}

int DitEngine::set_sp_ring(int on) {
  sp_ring_ = on != 0;
  return 0;
}

// final-projection rows of every rank -> the model output [B][HW][C p p] (fout_), registers and padding dropped
int DitEngine::sp_gather_out(hipStream_t s) {
  const size_t row = (size_t)C * P * P * 4;
  FLITE_REQUIRE(sp_fn_(sp_user_, 1, (void*)s) == 0, "sequence parallel: output exchange failed");
  for (int q = 0; q < sp_n_; ++q) {
    const int t_lo = std::max(q * Tl_, R), t_hi = std::min(T_, (q + 1) * Tl_);
    if (t_hi <= t_lo) continue;
    FLITE_HIP_CHECK(hipMemcpy2DAsync((char*)fout_ + (size_t)(t_lo - R) * row, (size_t)HW_ * row,
                                     (const char*)sp_out_recv_ + ((size_t)q * M_ + (t_lo - q * Tl_)) * row,
                                     (size_t)Tl_ * row, (size_t)(t_hi - t_lo) * row, B_, hipMemcpyDeviceToDevice, s));
  }
  return 0;
}

int DitEngine::set_sequence_parallel(int rank, int nranks, flite_sp_allgather_fn fn, void* user) {
  FLITE_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "sequence parallel: bad rank / nranks");
  FLITE_REQUIRE(nranks == 1 || fn != nullptr, "sequence parallel: exchange callback missing");
  sp_rank_ = rank;
  sp_n_ = nranks;
  sp_fn_ = fn;
  sp_user_ = user;
  drop_graph();
  free_ws();
  B_ = Hl_ = Wl_ = 0;  // the next prepare lays out the rows of this rank
  return 0;
}

int DitEngine::sp_buffer_bytes(long* kv_send, long* out_send) const {
  FLITE_REQUIRE(x_ != nullptr, "sp_buffer_bytes: call prepare first");
  *kv_send = M_ * 2 * D * 2;
  *out_send = M_ * (long)C * P * P * 4;
  return 0;
}

int DitEngine::sp_bind_buffers(void* kv_send, void* kv_recv, void* out_send, void* out_recv) {
  FLITE_REQUIRE(kv_send && kv_recv && out_send && out_recv, "sp_bind_buffers: null buffer");
  sp_kv_send_ = (bf16_t*)kv_send;
  sp_kv_recv_ = (bf16_t*)kv_recv;
  sp_out_send_ = (float*)out_send;
  sp_out_recv_ = (float*)out_recv;
  return 0;
}

int DitEngine::unpatchify_out(hipStream_t s, void* y, bool out_bf16) {
  FLITE_REQUIRE(fout_ != nullptr && y != nullptr, "unpatchify: call prepare first (and pass an output)");
  return unpatchify(fout_, y, out_bf16, B_, C, Hl_, Wl_, P, s);
}

int DitEngine::sample(hipStream_t s, float* acc, int Bi, int n_steps, const float* t_host, const float* dt_host,
                      float guidance, int use_cfg, int apg, float apg_thr, int use_graph) {
  FLITE_REQUIRE(n_steps >= 1 && n_steps <= ntmax_, "sample: too many steps for the prepared workspace");
  const int dup = use_cfg ? 2 : 1;
  FLITE_REQUIRE(Bi * dup == B_, "sample: batch does not match the prepared workspace");
  FLITE_REQUIRE(!apg || use_cfg, "sample: APG requires classifier-free guidance");
  FLITE_REQUIRE(!ctx_stale_, "sample: context K/V cache is stale (weights changed since set_context, or it "
                "failed): set the context again");
  if (fp8_ && w8_stale_ && quantise_fp8(s)) return 1;  // before any capture: quantise_fp8 synchronises
  if (fp8_ && collapse_fp8(s)) return 1;
  // timesteps: one row per step, shared by every sample of the batch (pipeline.py:260,268)
  FLITE_HIP_CHECK(hipMemcpyAsync(tdev_, t_host, n_steps * 4, hipMemcpyHostToDevice, s));
  if (set_timesteps(s, tdev_, n_steps, cfg.bf16_timestep_quant)) return 1;

  auto body = [&](hipStream_t st, float* acc) -> int {
    probe_n_ = 0;
    for (int i = 0; i < n_steps; ++i) {
      char name[32];
      snprintf(name, sizeof(name), "flite.step.%d", i);
      RoctxRange range(name);
      if (probe_begin(st, FLITE_PROBE_STEP)) return 1;
      if (forward(st, acc, false, Bi, dup, i, 0)) return 1;
      if (probe_end(st, FLITE_PROBE_STEP)) return 1;
      if (apg) {
        if (apg_euler(fout_, acc, Bi, C, Hl_, Wl_, P, guidance, apg_thr, dt_host[i], st)) return 1;
      } else {
        if (cfg_euler(fout_, acc, Bi, C, Hl_, Wl_, P, dup, guidance, dt_host[i], st)) return 1;
      }
    }
    return 0;
  };
  if (!use_graph || sp_n_ > 1) return body(s, acc);  // the host exchange callback cannot be captured

  // hipGraph: capture the whole n_steps loop once per (shape, schedule, guidance), replay after. The graph
  // integrates into the engine-owned accumulator acc_, so the caller's buffer address does not key the graph.
  std::vector<float> key = {(float)n_steps, guidance, (float)use_cfg, (float)apg, apg_thr};
  for (int i = 0; i < n_steps; ++i) key.push_back(dt_host[i]);
  if (!gstream_) {
    FLITE_HIP_CHECK(hipStreamCreateWithFlags(&gstream_, hipStreamNonBlocking));
    FLITE_HIP_CHECK(hipEventCreateWithFlags(&ev_in_, hipEventDisableTiming));
    FLITE_HIP_CHECK(hipEventCreateWithFlags(&ev_out_, hipEventDisableTiming));
  }
  const size_t acc_bytes = (size_t)Bi * HW_ * C * P * P * 4;
  FLITE_HIP_CHECK(hipMemcpyAsync(acc_, acc, acc_bytes, hipMemcpyDeviceToDevice, s));
  FLITE_HIP_CHECK(hipEventRecord(ev_in_, s));
  FLITE_HIP_CHECK(hipStreamWaitEvent(gstream_, ev_in_, 0));
  if (!gexec_ || key != gkey_) {
    drop_graph();
    hipGraph_t graph;
    FLITE_HIP_CHECK(hipStreamBeginCapture(gstream_, hipStreamCaptureModeThreadLocal));
    const int rc = body(gstream_, acc_);
    const hipError_t e = hipStreamEndCapture(gstream_, &graph);
    if (rc) return rc;
    FLITE_HIP_CHECK(e);
    FLITE_HIP_CHECK(hipGraphInstantiate(&gexec_, graph, nullptr, nullptr, 0));
    hipGraphDestroy(graph);
    gkey_ = key;
  }
  FLITE_HIP_CHECK(hipGraphLaunch(gexec_, gstream_));
  FLITE_HIP_CHECK(hipEventRecord(ev_out_, gstream_));
  FLITE_HIP_CHECK(hipStreamWaitEvent(s, ev_out_, 0));
  FLITE_HIP_CHECK(hipMemcpyAsync(acc, acc_, acc_bytes, hipMemcpyDeviceToDevice, s));
  return 0;
}

}  // namespace flite
