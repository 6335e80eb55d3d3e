// Internal launcher declarations for the gfx950 kernels (host side). Not part of the C ABI.
#pragma once
#include "common.h"

namespace flite {

enum GemmEpilogue {
  EPI_STORE_BF16 = 0,   // out_bf16[m][n] = acc + bias[n]
  EPI_STORE_F32 = 1,    // out_f32[m][n]  = acc + bias[n]
  EPI_RESID_F32 = 2,    // out_f32[m][n] += gate[seg(m)][n] * (acc + bias[n])   (gated residual, model.py:289,297,301)
  EPI_SWIGLU_BF16 = 3,  // out_bf16[m][f] = silu(A.Wg[f]) * (A.Wu[f])            (LigerSwiGLUMLP gate/up)
  EPI_GEGLU_BF16 = 6,   // out_bf16[m][f] = gelu_tanh(A.Wg[f]) * (A.Wu[f])     (T5 DenseGatedActDense wi_0 / wi_1)
  EPI_QKV_NORM_BF16 = 5,  // out_bf16 = acc + bias; columns [0, norm_cols) (heads of 256) first get 2-D RoPE
                          // (columns [0, rope_cols)) and QKNorm's per-head RMSNorm (model.py:166-180,197)
  EPI_RESID_BF16 = 7,   // out_bf16[m][n] = bf16(out[m][n] + gate * (acc + bias))   (EPI_RESID_F32 on a bf16 residual
                        // stream: fp32 math, one rounding -- the reference rounds twice, model.py:289)
};

struct GemmParams {
  const bf16_t* A = nullptr;  // [M, K], row stride lda (elements)
  long lda = 0;
  const bf16_t* W = nullptr;  // [N, K], row stride ldw (nn.Linear weight)
  long ldw = 0;
  const bf16_t* W2 = nullptr;    // SwiGLU only: up_proj weight [F, K]; W = gate_proj, N = 2F
  const bf16_t* bias = nullptr;  // [N] bf16 (model parameter dtype) or null
  void* out = nullptr;           // output, row stride ldo (elements)
  long ldo = 0;
  const float* gate = nullptr;   // RESID: gate rows, one per segment of rows_per_seg rows
  long gate_seg_stride = 0;      // elements between consecutive segments' gate rows (0 = shared)
  int rows_per_seg = 1;
  int M = 0, N = 0, K = 0;
  int act = 0;                   // 1: SiLU after bias (time_embed / adaLN inputs, model.py:448-456)
  // output row mapping: out_row = (m / out_seg) * out_seg_stride + out_seg_off + m % out_seg (0 = identity)
  long out_seg = 0, out_seg_stride = 0, out_seg_off = 0;
  const bf16_t* resid = nullptr;  // STORE_BF16: residual added before the store (same layout as out)
  // implicit-GEMM 3x3 conv (pad 1): A is read from the NHWC input instead of p.A; M = B*oh*ow, K = 9*C,
  // W = packed weight [Cout][ky][kx][C]; conv_up = nearest-2x upsample folded in (oh = 2*ih)
  const bf16_t* conv_in = nullptr;
  long conv_in_bytes = 0;
  int conv_ih = 0, conv_iw = 0, conv_c = 0, conv_oh = 0, conv_ow = 0, conv_up = 0;
  // stream-K workspace (optional): fp32 partial tiles [CUs][256*256] + int flags [CUs], zero-initialised.
  // When present the launcher may cut a partial last wave of tiles into equal k-ranges (gemm.hip).
  float* sk_ws = nullptr;
  int* sk_flags = nullptr;
  int sk_tiles = 0;  // set by the launcher
  int sk_wgs = 0;    // set by the launcher: workgroups sharing the stream-K iterations
  // EPI_QKV_NORM_BF16: factorised RoPE table (common.h RopeAxes) for columns [0, rope_cols)
  RopeAxes rope;
  int rope_cols = 0, norm_cols = 0;
  float norm_eps = 1e-6f;
  // optional read-ahead (data-parallel tiles): a byte range a later kernel reads (its weights), touched by the
  // workgroups after their mainloops so that it comes from the Infinity Cache instead of HBM
  const void* pf = nullptr;
  long pf_bytes = 0;
  int resid_narrow = 0;  // set by the launcher: EPI_RESID_BF16 with 8-B lanes (FLITE_GEMM_RESID_NARROW, A/B switch)
};

// bytes of the stream-K workspace (partials + flags) for the current device
size_t gemm_sk_workspace_bytes();
int gemm_sk_workspace_cus();

int gemm_bf16(const GemmParams& p, int epi, hipStream_t stream);

// Varlen flash attention (flash_attn_varlen_func semantics, non-causal). Token t of sequence b lives at
// row cu[b] + t; head h of a row starts at h * head_stride elements.
struct AttnParams {
  const bf16_t* q = nullptr;
  const bf16_t* k = nullptr;
  const bf16_t* v = nullptr;
  bf16_t* o = nullptr;
  long q_row_stride = 0, k_row_stride = 0, v_row_stride = 0, o_row_stride = 0;
  long q_head_stride = 0, k_head_stride = 0, v_head_stride = 0, o_head_stride = 0;
  const int* cu_q = nullptr;  // device int32 [B+1]
  const int* cu_k = nullptr;  // device int32 [B+1]
  int B = 0, H = 0, head_dim = 0;
  int max_q = 0;              // max query length (grid size)
  int max_k = 0;              // max key length (0 = unknown): a hint for the schedule only
  float scale = 1.f;
  // > 0: every score*scale is bounded by +-max_score (QK-normed inputs) -> fixed-shift softmax, no rescale
  float max_score = 0.f;
  // optional split workspace (attention.hip "Schedule"; bounded softmax only): zero-filled once by its owner,
  // left zeroed by every launch; launches sharing it must be stream-ordered
  void* split_ws = nullptr;
  long split_ws_bytes = 0;
  // optional key-range ends (device int32 [B]); null: cu_k[b + 1]
  const int* k_end = nullptr;
  // Partial (O, l) hand-over between two launches over disjoint key sets of the same queries (bounded softmax
  // only: with the fixed shift the two partial sums add without rescaling; the sequence-parallel overlap).
  // 1: write the unnormalised O (fp32, [query row][H * 256]) and the row sums l ([query row][H]) instead of o;
  // 2: add them to this launch's O and l, then normalise into o; 3: add them and write the sums back as the new
  // partial (a middle step of the ring, dit.cpp sp_ring_attention). No tail split in any partial mode.
  int part_mode = 0;
  float* part_o = nullptr;
  float* part_l = nullptr;
  // Optional MXFP8 output (the fp8 DiT's proj A operand, bound for fp8.hip's layout): o8 e4m3 bytes at the
  // element offsets of o, scales [cols/128][o8_rows_pad][4] by query row. The values are the bf16 outputs
  // quantised (bit-identical to quant_rows_fp8 of o). The tail-split rows still pass through o (bf16).
  uint8_t* o8 = nullptr;
  uint8_t* o8_scale = nullptr;
  long o8_rows_pad = 0;
  int n_main = 0, n_split = 0;  // set by the launcher
  int split_first = 0;          // set by the launcher: tail chunks dispatched before the full q-tiles
};

int attn_fwd(const AttnParams& p, hipStream_t stream);
// bytes of a split workspace that lets a (B sequences, H heads) launch cut its tails over the chip (0: no split)
long attn_split_workspace_bytes(int B, int H);
// the same for launches of up to max_q queries over up to max_k keys: also holds the 256-row kernel's split plan
// (attention_q256.hip), which attn_fwd takes for long bounded launches when the workspace is this large
long attn_workspace_bytes(int B, int H, int max_q, int max_k);
// attention_q256.hip: the 256-row route (returns -1 when the launch does not qualify or the workspace is short)
int attn_q256_fwd(const AttnParams& p, hipStream_t stream);
long attn_q256_workspace_bytes(int B, int H, int max_q, int max_k);
int attn_q256_set(int mode);  // process-wide route policy: 0 never, 1 always, 2 by prediction (default)

}  // namespace flite

namespace flite {

struct NormModParams {
  const void* x = nullptr;  // fp32 or bf16 input rows
  long ldx = 0;
  bf16_t* y = nullptr;      // bf16 output rows
  long ldy = 0;
  const bf16_t* w = nullptr;  // norm weight [D] (bf16 param) or null
  const float* shift = nullptr;  // modulation rows (fp32), one per segment, or null
  const float* scale = nullptr;
  long mod_seg_stride = 0;
  long rows = 0;
  int D = 0;
  float eps = 1e-6f;
  // input row mapping: in_row = (m / in_seg) * in_stride + in_off + m % in_seg (in_seg = 0: identity);
  // the modulation segment of output row m is m / in_seg (0 when in_seg == 0)
  long in_seg = 0, in_stride = 0, in_off = 0;
  // MXFP8 output instead of y (fp8 DiT path): e4m3 rows (stride ldy bytes) + k-tile-major block scales
  // [D/128][ysc_rows_pad][4] (fp8.hip)
  uint8_t* y8 = nullptr;
  uint8_t* ysc = nullptr;
  long ysc_rows_pad = 0;
  // optional read-ahead (D = 3072 row kernel): up to two byte ranges the next GEMM reads (its weights), touched
  // once by the workgroups of this pass so that they come from the Infinity Cache instead of HBM
  const void* pf[2] = {nullptr, nullptr};
  long pf_bytes[2] = {0, 0};
  // optional deferred broadcast residual (D = 3072 row kernel, fp32 input, identity row mapping): rows m < bc_rows
  // first take x[m] += bc_gate[seg] * bc_c[seg], seg = m / bc_rows_per_seg, written back to x (the collapsed
  // sequences' cross-attention update, ctx_bcast_resid's expression), then normalise
  const float* bc_c = nullptr;
  const float* bc_gate = nullptr;
  long bc_gate_stride = 0;
  long bc_rows = 0;
  int bc_rows_per_seg = 1;
};
int rmsnorm_mod(const NormModParams& p, bool in_bf16, hipStream_t s);

struct RopeNormParams {
  bf16_t* x = nullptr;  // rows of heads (256 wide each), in place
  long ldx = 0;
  long rows = 0;
  int heads = 0;         // heads per row processed (starting at column 0)
  int rope_heads = 0;    // heads [0, rope_heads) get RoPE (q and k of self-attention), the rest norm only
  const float* cos = nullptr;  // [tokens_per_seq, 128] or null (no RoPE)
  const float* sin = nullptr;
  long tokens_per_seq = 0;
  float eps = 1e-6f;
};
int rope_qknorm(const RopeNormParams& p, hipStream_t s);

int patchify(const void* lat, bool in_bf16, bf16_t* out, int Bi, int C, int H, int W, int P, int dup, hipStream_t s);
int fill_registers(void* x, bool x16, const bf16_t* reg, int B, int T, int R, int D, hipStream_t s);
int add_pos_embed(void* x, bool x16, const bf16_t* pos, int B, int T, int D, hipStream_t s);
int cfg_euler(const float* out, float* acc, int Bi, int C, int H, int W, int P, int dup, float g, float dt,
              hipStream_t s);
int cfg_euler_nchw(const float* u, const float* c, float* acc, long n, float g, float dt, int use_cfg,
                   hipStream_t s);
int unpatchify(const float* out, void* y, bool out_bf16, int B, int C, int H, int W, int P, hipStream_t s);
int apg_sums(const float* u, const float* c, long n, float k, int phase, float* out2, hipStream_t s);
int apg_update_nchw(const float* u, const float* c, float* acc, long n, float g, float k, float sc, float dt,
                    hipStream_t s);
int apg_sums_dev(const float* u, const float* c, long n, int phase, float* ws4, hipStream_t s);
int rows_uniform(const void* x, int cols, const int* cu, int nseq, int* bad, hipStream_t s);
int ctx_bcast_resid(void* x, bool x16, const float* c, const float* gate, long gate_seg_stride, int rows_per_seg,
                    long rows, int D, hipStream_t s);
int apg_update_nchw_dev(const float* u, const float* c, float* acc, long n, float g, float thr, long n_total,
                        const float* ws4, float dt, hipStream_t s);
int apg_euler(const float* out, float* acc, int Bi, int C, int H, int W, int P, float g, float thr, float dt,
              hipStream_t s);
int timestep_embed(const float* t, bf16_t* emb, int n, int D, int quantize, hipStream_t s);
int rope_table(const float* inv_freq, float* cos_t, float* sin_t, int hh, int ww, int R, int round_bf16,
               hipStream_t s);
// the same angles as rope_table, factorised per axis (common.h RopeAxes): cs [1 + hh + ww][64][2]
int rope_axes_table(const float* inv_freq, float* cs, int hh, int ww, int round_bf16, hipStream_t s);
int gather_rows(const bf16_t* src, bf16_t* dst, const int* idx, long n, int cols, hipStream_t s);

}  // namespace flite

namespace flite {
int gemm_init();  // set kernel attributes once (outside any graph capture)
int attn_init();
}  // namespace flite

namespace flite {
uint64_t fnv1a64(const char* s);
int hash_init(void* out, int out_bf16, long n, const char* name, uint64_t seed, double std, hipStream_t s);
int fill_bf16(bf16_t* out, long n, float v, hipStream_t s);
}  // namespace flite

namespace flite {
// VAE decoder helpers (vae.hip)
int group_norm(const bf16_t* x, bf16_t* y, long rows, int C, int G, const bf16_t* gamma, const bf16_t* beta,
               float eps, bool silu, double* stats, hipStream_t s);
int softmax_rows(const float* S, bf16_t* P, int R, int L, int ld, float scale, hipStream_t s);
int transpose_bf16(const bf16_t* x, bf16_t* y, int R, int C, int ldy, hipStream_t s);
int latent_to_nhwc(const float* z, long plane, int ldz, int th, int tw, bf16_t* x, int C, int Cpad, float scaling,
                   float shift, hipStream_t s);
int tile_blend(const float* a, int a_h, int a_w, float* b, int b_h, int b_w, int e, bool vertical, hipStream_t s);
int tile_to_uint8(const float* t, int tw, unsigned char* img, int img_w, int y0, int x0, int rows, int cols,
                  hipStream_t s);
int to_uint8(const float* o, int ld, unsigned char* img, long hw, hipStream_t s);
int pack_conv_weight(const bf16_t* w, bf16_t* o, int Cout, int Cin, int Cpad, hipStream_t s);
// MXFP8 rows (e4m3 + one E8M0 scale per 32 K, scales row-major [rows][K/32]) <-> bf16 (the fp8 VAE weights)
int mx_quant_rows_rm(const bf16_t* x, long rows, int K, uint8_t* q, uint8_t* sc, hipStream_t s);
int mx_dequant_rows_rm(const uint8_t* q, const uint8_t* sc, long rows, int K, bf16_t* x, hipStream_t s);
}  // namespace flite
