// C-ABI surface of libflite_hip.so (declared in include/flite.h). Plain pointers and sizes only; every
// entry point returns an int status (0 = ok) and never throws; the last error message is thread-local.
#include <string>

#include "../../include/flite.h"
#include "common.h"
#include "kernels.h"
#include "dit.h"
#include "fp8.h"
#include "t5.h"
#include <math.h>

namespace flite {
static thread_local std::string g_last_error;
void set_last_error(const std::string& msg) { g_last_error = msg; }
const char* get_last_error() { return g_last_error.c_str(); }
}  // namespace flite

using namespace flite;

extern "C" {

const char* flite_last_error(void) { return get_last_error(); }

int flite_version(void) { return FLITE_ABI_VERSION; }

int flite_gemm_bf16(void* stream, int M, int N, int K, const void* A, long lda, const void* W, long ldw,
                    const void* W2, const void* bias, int epilogue, void* out, long ldo, const float* gate,
                    long gate_seg_stride, int rows_per_seg) {
  GemmParams p;
  p.A = (const bf16_t*)A;
  p.lda = lda;
  p.W = (const bf16_t*)W;
  p.ldw = ldw;
  p.W2 = (const bf16_t*)W2;
  p.bias = (const bf16_t*)bias;
  p.out = out;
  p.ldo = ldo;
  p.gate = gate;
  p.gate_seg_stride = gate_seg_stride;
  p.rows_per_seg = rows_per_seg;
  p.M = M;
  p.N = N;
  p.K = K;
  return gemm_bf16(p, epilogue, (hipStream_t)stream);
}

long flite_gemm_workspace_bytes(void) { return (long)gemm_sk_workspace_bytes(); }

int flite_gemm_bf16_ws(void* stream, int M, int N, int K, const void* A, long lda, const void* W, long ldw,
                       const void* W2, const void* bias, int epilogue, void* out, long ldo, const float* gate,
                       long gate_seg_stride, int rows_per_seg, void* workspace) {
  GemmParams p;
  p.A = (const bf16_t*)A;
  p.lda = lda;
  p.W = (const bf16_t*)W;
  p.ldw = ldw;
  p.W2 = (const bf16_t*)W2;
  p.bias = (const bf16_t*)bias;
  p.out = out;
  p.ldo = ldo;
  p.gate = gate;
  p.gate_seg_stride = gate_seg_stride;
  p.rows_per_seg = rows_per_seg;
  p.M = M;
  p.N = N;
  p.K = K;
  const int G = gemm_sk_workspace_cus();
  if (workspace != nullptr && G > 0) {
    p.sk_ws = (float*)workspace;
    p.sk_flags = (int*)((char*)workspace + (size_t)G * 256 * 256 * 4);
  }
  return gemm_bf16(p, epilogue, (hipStream_t)stream);
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------------
extern "C" {

int flite_attn_varlen_fwd(void* stream, const void* q, const void* k, const void* v, void* o, long q_row_stride,
                          long k_row_stride, long v_row_stride, long o_row_stride, long head_stride,
                          const int* cu_seqlens_q, const int* cu_seqlens_k, int batch, int num_heads, int head_dim,
                          int max_seqlen_q, float softmax_scale, float max_score) {
  AttnParams a;
  a.q = (const bf16_t*)q;
  a.k = (const bf16_t*)k;
  a.v = (const bf16_t*)v;
  a.o = (bf16_t*)o;
  a.q_row_stride = q_row_stride;
  a.k_row_stride = k_row_stride;
  a.v_row_stride = v_row_stride;
  a.o_row_stride = o_row_stride;
  a.q_head_stride = a.k_head_stride = a.v_head_stride = a.o_head_stride = head_stride;
  a.cu_q = cu_seqlens_q;
  a.cu_k = cu_seqlens_k;
  a.B = batch;
  a.H = num_heads;
  a.head_dim = head_dim;
  a.max_q = max_seqlen_q;
  a.scale = softmax_scale;
  a.max_score = max_score;
  return attn_fwd(a, (hipStream_t)stream);
}

long flite_attn_workspace_bytes(int batch, int num_heads) { return attn_split_workspace_bytes(batch, num_heads); }

int flite_attn_set_q256(int mode) { return attn_q256_set(mode); }

long flite_attn_workspace_bytes_for(int batch, int num_heads, int max_seqlen_q, int max_seqlen_k) {
  if (batch <= 0 || num_heads <= 0 || max_seqlen_q < 0 || max_seqlen_k < 0) return 0;
  return attn_workspace_bytes(batch, num_heads, max_seqlen_q, max_seqlen_k);
}

int flite_attn_varlen_fwd_ws(void* stream, const void* q, const void* k, const void* v, void* o, long q_row_stride,
                             long k_row_stride, long v_row_stride, long o_row_stride, long head_stride,
                             const int* cu_seqlens_q, const int* cu_seqlens_k, int batch, int num_heads, int head_dim,
                             int max_seqlen_q, int max_seqlen_k, float softmax_scale, float max_score,
                             void* workspace, long workspace_bytes) {
  AttnParams a;
  a.q = (const bf16_t*)q;
  a.k = (const bf16_t*)k;
  a.v = (const bf16_t*)v;
  a.o = (bf16_t*)o;
  a.q_row_stride = q_row_stride;
  a.k_row_stride = k_row_stride;
  a.v_row_stride = v_row_stride;
  a.o_row_stride = o_row_stride;
  a.q_head_stride = a.k_head_stride = a.v_head_stride = a.o_head_stride = head_stride;
  a.cu_q = cu_seqlens_q;
  a.cu_k = cu_seqlens_k;
  a.B = batch;
  a.H = num_heads;
  a.head_dim = head_dim;
  a.max_q = max_seqlen_q;
  a.scale = softmax_scale;
  a.max_score = max_score;
  a.max_k = max_seqlen_k;
  a.split_ws = workspace;
  a.split_ws_bytes = workspace != nullptr ? workspace_bytes : 0;
  return attn_fwd(a, (hipStream_t)stream);
}

int flite_rmsnorm_modulate(void* stream, const void* x, int x_is_bf16, long ldx, void* y, long ldy, const void* w,
                           const float* shift, const float* scale, long mod_seg_stride, long seg_rows, long rows,
                           int dim, float eps) {
  NormModParams p;
  p.x = x;
  p.ldx = ldx;
  p.y = (bf16_t*)y;
  p.ldy = ldy;
  p.w = (const bf16_t*)w;
  p.shift = shift;
  p.scale = scale;
  p.mod_seg_stride = mod_seg_stride;
  p.rows = rows;
  p.D = dim;
  p.eps = eps;
  p.in_seg = seg_rows;
  p.in_stride = seg_rows;
  p.in_off = 0;
  return rmsnorm_mod(p, x_is_bf16 != 0, (hipStream_t)stream);
}

int flite_rope_qknorm(void* stream, void* x, long ldx, long rows, int heads, int rope_heads, const float* cos_t,
                      const float* sin_t, long tokens_per_seq, float eps) {
  RopeNormParams p;
  p.x = (bf16_t*)x;
  p.ldx = ldx;
  p.rows = rows;
  p.heads = heads;
  p.rope_heads = rope_heads;
  p.cos = cos_t;
  p.sin = sin_t;
  p.tokens_per_seq = tokens_per_seq;
  p.eps = eps;
  return rope_qknorm(p, (hipStream_t)stream);
}

int flite_rope_tables(void* stream, float* cos_t, float* sin_t, int h, int w, int n_reg, float base,
                      int round_bf16) {
  float inv[64];
  for (int i = 0; i < 64; ++i) inv[i] = (float)(1.0 / pow((double)base, (double)(2 * i) / 128.0));
  float* dinv = nullptr;
  FLITE_HIP_CHECK(hipMalloc(&dinv, sizeof(inv)));
  FLITE_HIP_CHECK(hipMemcpy(dinv, inv, sizeof(inv), hipMemcpyHostToDevice));
  const int rc = rope_table(dinv, cos_t, sin_t, h, w, n_reg, round_bf16, (hipStream_t)stream);
  FLITE_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
  hipFree(dinv);
  return rc;
}

int flite_timestep_embedding(void* stream, const float* t, void* emb, int n, int dim, int quantize) {
  return timestep_embed(t, (bf16_t*)emb, n, dim, quantize, (hipStream_t)stream);
}

struct flite_dit {
  flite::DitEngine* eng;
};

int flite_dit_create(const flite_dit_config* cfg, flite_dit** out) {
  FLITE_REQUIRE(cfg != nullptr && out != nullptr, "flite_dit_create: null argument");
  FLITE_REQUIRE(cfg->depth > 0 && cfg->hidden_size > 0 && cfg->num_heads > 0, "flite_dit_create: bad config");
  if (gemm_init()) return 1;
  if (attn_init()) return 1;
  flite_dit* d = new flite_dit;
  d->eng = new DitEngine(*cfg);
  *out = d;
  return 0;
}

int flite_dit_set_sequence_parallel(flite_dit* dit, int rank, int nranks, flite_sp_allgather_fn fn, void* user) {
  FLITE_REQUIRE(dit != nullptr, "flite_dit_set_sequence_parallel: null engine");
  return dit->eng->set_sequence_parallel(rank, nranks, fn, user);
}

int flite_dit_sp_buffer_bytes(flite_dit* dit, long* kv_send_bytes, long* out_send_bytes) {
  FLITE_REQUIRE(dit && kv_send_bytes && out_send_bytes, "flite_dit_sp_buffer_bytes: null argument");
  return dit->eng->sp_buffer_bytes(kv_send_bytes, out_send_bytes);
}

int flite_dit_sp_bind_buffers(flite_dit* dit, void* kv_send, void* kv_recv, void* out_send, void* out_recv) {
  FLITE_REQUIRE(dit != nullptr, "flite_dit_sp_bind_buffers: null engine");
  return dit->eng->sp_bind_buffers(kv_send, kv_recv, out_send, out_recv);
}

int flite_dit_sp_set_ring(flite_dit* dit, int ring) {
  FLITE_REQUIRE(dit != nullptr, "flite_dit_sp_set_ring: null engine");
  return dit->eng->set_sp_ring(ring);
}

int flite_dit_destroy(flite_dit* dit) {
  if (dit) {
    delete dit->eng;
    delete dit;
  }
  return 0;
}

int flite_dit_bind(flite_dit* dit, const char* name, const void* ptr, long numel) {
  FLITE_REQUIRE(dit && name, "flite_dit_bind: null argument");
  return dit->eng->bind(name, ptr, numel);
}

int flite_dit_prepare(flite_dit* dit, int batch, int latent_h, int latent_w, int n_ctx, int n_t) {
  FLITE_REQUIRE(dit, "flite_dit_prepare: null engine");
  return dit->eng->prepare(batch, latent_h, latent_w, n_ctx, n_t);
}

int flite_dit_set_context(flite_dit* dit, void* stream, const void* ctx, const int* cu_seqlens_host, int batch) {
  FLITE_REQUIRE(dit && cu_seqlens_host, "flite_dit_set_context: null argument");
  return dit->eng->set_context((hipStream_t)stream, ctx, cu_seqlens_host, batch);
}

int flite_dit_set_timesteps(flite_dit* dit, void* stream, const float* t, int n, int quantize) {
  FLITE_REQUIRE(dit && t, "flite_dit_set_timesteps: null argument");
  return dit->eng->set_timesteps((hipStream_t)stream, t, n, quantize);
}

int flite_gather_rows(void* stream, const void* src, void* dst, const int* idx, long n, int cols) {
  return gather_rows((const bf16_t*)src, (bf16_t*)dst, idx, n, cols, (hipStream_t)stream);
}

int flite_t5_attention(void* stream, const void* q, long ldq, const void* k, long ldk, const void* v, long ldv,
                       void* o, long ldo, const int* bucket, const void* rel_weight, const float* mask, int B,
                       int L, int H) {
  T5AttnParams p;
  p.q = (const bf16_t*)q;
  p.k = (const bf16_t*)k;
  p.v = (const bf16_t*)v;
  p.o = (bf16_t*)o;
  p.ldq = ldq;
  p.ldk = ldk;
  p.ldv = ldv;
  p.ldo = ldo;
  p.bucket = bucket;
  p.rel_weight = (const bf16_t*)rel_weight;
  p.mask = mask;
  p.B = B;
  p.L = L;
  p.H = H;
  return t5_attention(p, (hipStream_t)stream);
}

int flite_embed_rows_f32(void* stream, const void* table, const int* ids, float* out, long n, int cols, long vocab) {
  FLITE_REQUIRE(table && ids && out, "flite_embed_rows_f32: null argument");
  return embed_rows_f32((const bf16_t*)table, ids, out, n, cols, vocab, (hipStream_t)stream);
}

int flite_cfg_euler(void* stream, const float* uncond, const float* cond, float* acc, long n, float guidance,
                    float dt, int use_cfg) {
  FLITE_REQUIRE(acc && cond && (uncond || !use_cfg), "flite_cfg_euler: null argument");
  FLITE_REQUIRE(n >= 0, "flite_cfg_euler: negative element count");
  return cfg_euler_nchw(uncond, cond, acc, n, guidance, dt, use_cfg, (hipStream_t)stream);
}

int flite_apg_sums(void* stream, const float* uncond, const float* cond, long n, float k, int phase, float* out2) {
  FLITE_REQUIRE(uncond && cond && out2, "flite_apg_sums: null argument");
  FLITE_REQUIRE(n >= 0, "flite_apg_sums: negative element count");
  return apg_sums(uncond, cond, n, k, phase, out2, (hipStream_t)stream);
}

int flite_apg_euler(void* stream, const float* uncond, const float* cond, float* acc, long n, float guidance,
                    float k, float orth_scale, float dt) {
  FLITE_REQUIRE(uncond && cond && acc, "flite_apg_euler: null argument");
  FLITE_REQUIRE(n >= 0, "flite_apg_euler: negative element count");
  return apg_update_nchw(uncond, cond, acc, n, guidance, k, orth_scale, dt, (hipStream_t)stream);
}

int flite_apg_sums_dev(void* stream, const float* uncond, const float* cond, long n, int phase, float* ws4) {
  FLITE_REQUIRE(uncond && cond && ws4, "flite_apg_sums_dev: null argument");
  FLITE_REQUIRE(n >= 0, "flite_apg_sums_dev: negative element count");
  return apg_sums_dev(uncond, cond, n, phase, ws4, (hipStream_t)stream);
}

int flite_apg_euler_dev(void* stream, const float* uncond, const float* cond, float* acc, long n, float guidance,
                        float threshold, long n_total, const float* ws4, float dt) {
  FLITE_REQUIRE(uncond && cond && acc && ws4, "flite_apg_euler_dev: null argument");
  FLITE_REQUIRE(n >= 0 && n_total >= n, "flite_apg_euler_dev: bad element counts");
  return apg_update_nchw_dev(uncond, cond, acc, n, guidance, threshold, n_total, ws4, dt, (hipStream_t)stream);
}

int flite_dit_forward(flite_dit* dit, void* stream, const void* x, int x_is_bf16, int batch, int t_row0,
                      int t_row_step, void* out, int out_is_bf16) {
  FLITE_REQUIRE(dit && x && out, "flite_dit_forward: null argument");
  if (dit->eng->forward((hipStream_t)stream, x, x_is_bf16 != 0, batch, 1, t_row0, t_row_step)) return 1;
  return dit->eng->unpatchify_out((hipStream_t)stream, out, out_is_bf16 != 0);
}

int flite_dit_sample(flite_dit* dit, void* stream, float* acc, int n_img, int n_steps, const float* t_host,
                     const float* dt_host, float guidance, int use_cfg, int apg, float apg_threshold,
                     int use_graph) {
  FLITE_REQUIRE(dit && acc && t_host && dt_host, "flite_dit_sample: null argument");
  return dit->eng->sample((hipStream_t)stream, acc, n_img, n_steps, t_host, dt_host, guidance, use_cfg, apg,
                          apg_threshold, use_graph);
}

}  // extern "C"

extern "C" {
int flite_init_param(void* stream, void* out, int out_is_bf16, long numel, const char* name, unsigned long long seed,
                     double std, int ones) {
  FLITE_REQUIRE(out && name, "flite_init_param: null argument");
  if (ones) {
    FLITE_REQUIRE(out_is_bf16, "flite_init_param: ones only for bf16");
    return fill_bf16((bf16_t*)out, numel, 1.0f, (hipStream_t)stream);
  }
  return hash_init(out, out_is_bf16, numel, name, seed, std, (hipStream_t)stream);
}
}  // extern "C"

extern "C" {
int flite_dit_set_probe(flite_dit* dit, int kind, int max_pairs) {
  FLITE_REQUIRE(dit, "flite_dit_set_probe: null engine");
  return dit->eng->set_probe(kind, max_pairs);
}
int flite_dit_read_probe(flite_dit* dit, float* ms, int cap, int* n) {
  FLITE_REQUIRE(dit && ms && n, "flite_dit_read_probe: null argument");
  return dit->eng->read_probe(ms, cap, n);
}
}  // extern "C"

extern "C" {
int flite_conv3x3_pack_weight(void* stream, const void* w, void* packed, int cout, int cin, int cin_pad) {
  FLITE_REQUIRE(w && packed && cin_pad % 64 == 0 && cin_pad >= cin, "flite_conv3x3_pack_weight: bad arguments");
  return pack_conv_weight((const bf16_t*)w, (bf16_t*)packed, cout, cin, cin_pad, (hipStream_t)stream);
}

int flite_conv3x3_bf16(void* stream, const void* x, int batch, int h, int w, int cin, int upsample,
                       const void* w_packed, const void* bias, int cout, void* out, const void* resid,
                       int out_is_f32) {
  FLITE_REQUIRE(batch == 1, "flite_conv3x3_bf16: one image per call");
  GemmParams g;
  g.conv_in = (const bf16_t*)x;
  g.conv_c = cin;
  g.conv_ih = h;
  g.conv_iw = w;
  g.conv_up = upsample ? 1 : 0;
  g.conv_oh = upsample ? 2 * h : h;
  g.conv_ow = upsample ? 2 * w : w;
  g.conv_in_bytes = (long)h * w * cin * 2;
  g.W = (const bf16_t*)w_packed;
  g.ldw = 9L * cin;
  g.bias = (const bf16_t*)bias;
  g.out = out;
  g.ldo = cout;
  g.resid = (const bf16_t*)resid;
  g.M = g.conv_oh * g.conv_ow;
  g.N = cout;
  g.K = 9 * cin;
  return gemm_bf16(g, out_is_f32 ? EPI_STORE_F32 : EPI_STORE_BF16, (hipStream_t)stream);
}

int flite_group_norm(void* stream, const void* x, void* y, long rows, int channels, int groups, const void* gamma,
                     const void* beta, float eps, int silu, double* stats_workspace) {
  return group_norm((const bf16_t*)x, (bf16_t*)y, rows, channels, groups, (const bf16_t*)gamma,
                    (const bf16_t*)beta, eps, silu != 0, stats_workspace, (hipStream_t)stream);
}
}  // extern "C"

// ---------------------------------------------------------------------------------------------------------------
// MXFP8 (fp8.hip, gemm_fp8.hip)
// ---------------------------------------------------------------------------------------------------------------
extern "C" {
int flite_quant_fp8_rows(void* stream, const void* src, long ld_src, long rows, int K, void* dst, long ld_dst,
                         void* scales, long rows_pad) {
  FLITE_REQUIRE(src && dst && scales, "flite_quant_fp8_rows: null argument");
  return quant_rows_fp8((const bf16_t*)src, ld_src, rows, K, (uint8_t*)dst, ld_dst, (uint8_t*)scales, rows_pad,
                        (hipStream_t)stream);
}

int flite_quant_fp8_gateup(void* stream, const void* gate, const void* up, long ld_src, int F, int K, void* dst,
                           void* scales) {
  FLITE_REQUIRE(gate && up && dst && scales, "flite_quant_fp8_gateup: null argument");
  return quant_gateup_fp8((const bf16_t*)gate, (const bf16_t*)up, ld_src, F, K, (uint8_t*)dst, (uint8_t*)scales,
                          (hipStream_t)stream);
}

int flite_gemm_fp8(void* stream, int M, int N, int K, const void* A8, long lda, const void* a_scales,
                   long a_rows_pad, const void* W8, long ldw, const void* w_scales, long w_rows_pad,
                   const void* bias, int epilogue, void* out, long ldo, void* out_scales, long out_rows_pad,
                   const float* gate, long gate_seg_stride, int rows_per_seg) {
  return flite_gemm_fp8_ws(stream, M, N, K, A8, lda, a_scales, a_rows_pad, W8, ldw, w_scales, w_rows_pad, bias,
                           epilogue, out, ldo, out_scales, out_rows_pad, gate, gate_seg_stride, rows_per_seg, nullptr);
}

int flite_gemm_fp8_ws(void* stream, int M, int N, int K, const void* A8, long lda, const void* a_scales,
                      long a_rows_pad, const void* W8, long ldw, const void* w_scales, long w_rows_pad,
                      const void* bias, int epilogue, void* out, long ldo, void* out_scales, long out_rows_pad,
                      const float* gate, long gate_seg_stride, int rows_per_seg, void* workspace) {
  FLITE_REQUIRE(A8 && a_scales && W8 && w_scales && out, "flite_gemm_fp8: null argument");
  GemmFp8Params p;
  p.A = (const uint8_t*)A8;
  p.lda = lda;
  p.As = (const uint8_t*)a_scales;
  p.a_rows_pad = a_rows_pad;
  p.W = (const uint8_t*)W8;
  p.ldw = ldw;
  p.Ws = (const uint8_t*)w_scales;
  p.w_rows_pad = w_rows_pad;
  p.bias = (const bf16_t*)bias;
  p.out = out;
  p.ldo = ldo;
  p.out_sc = (uint8_t*)out_scales;
  p.out_rows_pad = out_rows_pad;
  p.gate = gate;
  p.gate_seg_stride = gate_seg_stride;
  p.rows_per_seg = rows_per_seg;
  p.M = M;
  p.N = N;
  p.K = K;
  const int G = gemm_sk_workspace_cus();
  if (workspace != nullptr && G > 0) {  // the bf16 workspace layout: partial tiles, then one flag per CU
    p.sk_ws = (float*)workspace;
    p.sk_flags = (int*)((char*)workspace + (size_t)G * 256 * 256 * sizeof(float));
  }
  return gemm_fp8(p, epilogue, (hipStream_t)stream);
}

int flite_rmsnorm_modulate_fp8(void* stream, const float* x, long ldx, void* y8, long ldy, void* y_scales,
                               long rows_pad, const void* w, const float* shift, const float* scale,
                               long mod_seg_stride, long seg_rows, long rows, int dim, float eps) {
  FLITE_REQUIRE(x && y8 && y_scales, "flite_rmsnorm_modulate_fp8: null argument");
  NormModParams p;
  p.x = x;
  p.ldx = ldx;
  p.y8 = (uint8_t*)y8;
  p.ldy = ldy;
  p.ysc = (uint8_t*)y_scales;
  p.ysc_rows_pad = rows_pad;
  p.w = (const bf16_t*)w;
  p.shift = shift;
  p.scale = scale;
  p.mod_seg_stride = mod_seg_stride;
  p.rows = rows;
  p.D = dim;
  p.eps = eps;
  p.in_seg = seg_rows;
  p.in_stride = seg_rows;
  p.in_off = 0;
  return rmsnorm_mod(p, false, (hipStream_t)stream);
}

int flite_dit_enable_fp8(flite_dit* dit, void* stream, int enable) {
  FLITE_REQUIRE(dit, "flite_dit_enable_fp8: null engine");
  return dit->eng->enable_fp8((hipStream_t)stream, enable != 0);
}

int flite_dit_set_fp8_bf16_blocks(flite_dit* dit, const int* blocks, int n) {
  FLITE_REQUIRE(dit, "flite_dit_set_fp8_bf16_blocks: null engine");
  return dit->eng->set_fp8_bf16_blocks(blocks, n);
}

int flite_dit_set_fp8_gemm_classes(flite_dit* dit, int mask) {
  FLITE_REQUIRE(dit, "flite_dit_set_fp8_gemm_classes: null engine");
  return dit->eng->set_fp8_classes(mask);
}

int flite_dit_set_fp8_block_classes(flite_dit* dit, const int* masks, int n_blocks) {
  FLITE_REQUIRE(dit, "flite_dit_set_fp8_block_classes: null engine");
  return dit->eng->set_fp8_block_classes(masks, n_blocks);
}

int flite_dit_set_residual_bf16(flite_dit* dit, int enable) {
  FLITE_REQUIRE(dit, "flite_dit_set_residual_bf16: null engine");
  return dit->eng->set_residual_bf16(enable != 0);
}

int flite_dit_residual_bf16(flite_dit* dit) {
  if (!dit) {
    set_last_error("flite: flite_dit_residual_bf16: null engine");
    return -1;
  }
  return dit->eng->residual_bf16() ? 1 : 0;
}

int flite_dit_weights_updated(flite_dit* dit, void* stream) {
  FLITE_REQUIRE(dit, "flite_dit_weights_updated: null engine");
  return dit->eng->weights_updated((hipStream_t)stream);
}
}  // extern "C"
