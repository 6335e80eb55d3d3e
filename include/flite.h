/*
 * flite.h -- C ABI of libflite_hip.so, the MI355X (gfx950) native F-Lite sampling path.
 *
 * Conventions (all entry points):
 *   - Buffers are caller-owned DEVICE memory (e.g. torch .data_ptr()); sizes are element counts.
 *   - `stream` is a hipStream_t passed as void* (torch.cuda.current_stream().cuda_stream).
 *   - Return 0 on success, non-zero on error; the message is available from flite_last_error()
 *     (thread-local). Nothing throws across this boundary.
 *   - No allocation and no host synchronisation inside the launch entry points (hipGraph-capturable).
 *   - bf16 tensors are passed as their 16-bit storage; fp32 as float.
 *
 * Each entry point cites the reference interface it replaces (sippycoder/f-lite @ /root/reference).
 */
#ifndef FLITE_H_
#define FLITE_H_

#ifdef __cplusplus
extern "C" {
#endif

#define FLITE_ABI_VERSION 1

/* Thread-local message of the last failing call. */
const char* flite_last_error(void);
int flite_version(void);

/* ---------------------------------------------------------------------------------------------
 * Kernel-level operators (what the native library replaces under f_lite/model.py)
 * ------------------------------------------------------------------------------------------- */

/* Epilogue selectors for flite_gemm_bf16. */
#define FLITE_EPI_STORE_BF16 0  /* out_bf16[m][n]  = A.W^T + bias                                  */
#define FLITE_EPI_STORE_F32 1   /* out_f32[m][n]   = A.W^T + bias                                  */
#define FLITE_EPI_RESID_F32 2   /* out_f32[m][n]  += gate[m/rows_per_seg][n] * (A.W^T + bias)      */
#define FLITE_EPI_SWIGLU_BF16 3 /* out_bf16[m][f]  = silu(A.Wg^T)[f] * (A.Wu^T)[f], N = 2F          */
#define FLITE_EPI_GEGLU_BF16 6  /* out_bf16[m][f]  = gelu_tanh(A.Wg^T)[f] * (A.Wu^T)[f], N = 2F (T5)  */
#define FLITE_EPI_RESID_BF16 7  /* out_bf16[m][n]  = bf16(out + gate * (A.W^T + bias)), fp32 math      */

/*
 * bf16 GEMM with fused epilogue: C[M,N] = A[M,K] . W[N,K]^T  (W in nn.Linear [out,in] layout).
 * Replaces nn.Linear (f_lite/model.py:151,153-156,436,448-456,472-475) and LigerSwiGLUMLP
 * (model.py:261-267, SWIGLU: W = gate_proj.weight, W2 = up_proj.weight); the gated-residual
 * epilogue fuses `x + f(n) * gate` (model.py:289,297,301). K % 64 == 0; lda, ldw % 8 == 0.
 */
int flite_gemm_bf16(void* stream, int M, int N, int K, const void* A, long lda, const void* W, long ldw,
                    const void* W2, const void* bias, int epilogue, void* out, long ldo, const float* gate,
                    long gate_seg_stride, int rows_per_seg);

/*
 * Bytes of the optional stream-K workspace of flite_gemm_bf16_ws on the current device (fp32 partial tiles
 * + flags, one slot per CU).
 */
long flite_gemm_workspace_bytes(void);

/*
 * flite_gemm_bf16 with a caller-owned stream-K workspace (device memory of flite_gemm_workspace_bytes(),
 * zero-filled once before first use; every launch leaves it zeroed). When the last wave of 256x256 output
 * tiles is partial, the launch runs one workgroup per CU and splits that wave's k-iterations evenly over
 * them (partials reduced in a fixed order: deterministic). Launches sharing a workspace must be
 * stream-ordered.
 */
int flite_gemm_bf16_ws(void* stream, int M, int N, int K, const void* A, long lda, const void* W, long ldw,
                       const void* W2, const void* bias, int epilogue, void* out, long ldo, const float* gate,
                       long gate_seg_stride, int rows_per_seg, void* workspace);

/*
 * Varlen flash-attention forward, head_dim 256, non-causal.
 * Replaces flash_attn_interface.flash_attn_varlen_func(q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q,
 * max_seqlen_k, softmax_scale) (f_lite/model.py:203-210). Token t of sequence b is row cu[b]+t; head h of
 * a row starts at h*head_stride. cu_seqlens_* are device int32 [B+1]. Output o has the q layout.
 * max_score > 0 asserts |score*scale| <= max_score (QK-normed q, k): unshifted softmax p = exp2(score*scale*log2 e),
 * no running max, no online rescale (max_score <= 40, so every sum stays in fp32 range); max_score = 0 runs the
 * general online softmax.
 */
int flite_attn_varlen_fwd(void* stream, const void* q, const void* k, const void* v, void* o, long q_row_stride,
                          long k_row_stride, long v_row_stride, long o_row_stride, long head_stride,
                          const int* cu_seqlens_q, const int* cu_seqlens_k, int batch, int num_heads,
                          int head_dim, int max_seqlen_q, float softmax_scale, float max_score);

/*
 * Bytes of the optional split workspace of flite_attn_varlen_fwd_ws for `batch` sequences x `num_heads` heads on
 * the current device (0: that launch shape gains nothing from it).
 */
long flite_attn_workspace_bytes(int batch, int num_heads);

/*
 * The same for launches of up to max_seqlen_q queries over up to max_seqlen_k keys per sequence: also large enough
 * for the 256-query-row kernel's split plan, which flite_attn_varlen_fwd_ws takes for bounded launches over long
 * key ranges (max_seqlen_k >= 1024 given; the DiT's self-attention, reference f_lite/model.py:203-210). Always
 * >= flite_attn_workspace_bytes(batch, num_heads).
 */
long flite_attn_workspace_bytes_for(int batch, int num_heads, int max_seqlen_q, int max_seqlen_k);
/* Process-wide policy of that 256-query-row route: 0 never, 1 always (where eligible), 2 (the default) where its split
 * plan is predicted >= 4.5 % faster than the 128-row schedule. FLITE_ATTN_Q256=0/1 in the environment sets 0/1. */
int flite_attn_set_q256(int mode);

/*
 * flite_attn_varlen_fwd with a caller-owned split workspace (device memory, zero-filled once, left zeroed by
 * every launch; launches sharing it must be stream-ordered). With max_score > 0 the partial last q-tile of each
 * (sequence, head) is cut over the chip by key ranges and reduced in a fixed order (deterministic).
 * max_seqlen_k (flash_attn_varlen_func's argument; 0 = unknown) only steers that schedule.
 */
int flite_attn_varlen_fwd_ws(void* stream, const void* q, const void* k, const void* v, void* o, long q_row_stride,
                             long k_row_stride, long v_row_stride, long o_row_stride, long head_stride,
                             const int* cu_seqlens_q, const int* cu_seqlens_k, int batch, int num_heads,
                             int head_dim, int max_seqlen_q, int max_seqlen_k, float softmax_scale, float max_score,
                             void* workspace, long workspace_bytes);

/*
 * RMSNorm (+weight) (+adaLN modulate) to bf16: y = x*rsqrt(mean(x^2)+eps) * w * (1+scale) + shift.
 * Replaces LigerRMSNorm (model.py:238,248,260,437), RMSNorm (model.py:92-108) and the modulate
 * `norm_x * (1 + scale) + shift` (model.py:284,293,300,580). x is fp32 (x_is_bf16 = 0) or bf16.
 * shift/scale are fp32 rows, one per segment of seg_rows rows (seg_rows = 0: single segment), may be NULL.
 */
int flite_rmsnorm_modulate(void* stream, const void* x, int x_is_bf16, long ldx, void* y, long ldy, const void* w,
                           const float* shift, const float* scale, long mod_seg_stride, long seg_rows, long rows,
                           int dim, float eps);

/*
 * In-place 2-D RoPE (rotate-half, model.py:403-414) on heads [0, rope_heads) followed by the per-head
 * RMSNorm of QKNorm (model.py:115-126) on heads [0, heads) of bf16 rows (head size 256).
 * cos/sin: fp32 [tokens_per_seq, 128] tables (NULL = no RoPE); row r uses table row r % tokens_per_seq.
 */
int flite_rope_qknorm(void* stream, void* x, long ldx, long rows, int heads, int rope_heads, const float* cos_t,
                      const float* sin_t, long tokens_per_seq, float eps);

/* ---------------------------------------------------------------------------------------------
 * MXFP8 (BASELINE.json configs[4]: fp8 weights + activations). Elements OCP e4m3fn, one E8M0 scale per 32
 * consecutive K elements: e = ceil(log2(amax/448)), q = RNE(clamp(x * 2^-e, +-448)). Scale arrays are
 * "k-tile major": scales[K/128][rows_pad][4] bytes (rows_pad a multiple of 256, >= rows; pad rows are never
 * read back). The reference has no fp8 path: these replace the nn.Linear calls of model.py:151-156 and
 * LigerSwiGLUMLP (model.py:261-267) in the fp8 configuration.
 * ------------------------------------------------------------------------------------------- */
#define FLITE_EPI8_STORE_BF16 0  /* out_bf16[m][n]  = A.W^T + bias                                   */
#define FLITE_EPI8_RESID_F32 2   /* out_f32[m][n]  += gate[m/rows_per_seg][n] * (A.W^T + bias)       */
#define FLITE_EPI8_RESID_BF16 7  /* out_bf16[m][n]  = bf16(out + gate * (A.W^T + bias)), fp32 math     */
#define FLITE_EPI8_SWIGLU_FP8 4  /* out_fp8[m][f]   = MX(silu(A.Wg^T) * (A.Wu^T)), W = gate|up interleaved in
                                    16-row sub-tiles (flite_quant_fp8_gateup), N = 2F; scales to out_scales */
#define FLITE_EPI8_SWIGLU_BF16 6 /* out_bf16[m][f]  = silu(A.Wg^T) * (A.Wu^T), same W layout (an fp8 gate/up
                                    feeding a bf16 down projection)                                  */

/* bf16 rows [rows, K] (row stride ld_src elements) -> fp8 [rows, K] (row stride ld_dst bytes) + scales. */
int flite_quant_fp8_rows(void* stream, const void* src, long ld_src, long rows, int K, void* dst, long ld_dst,
                         void* scales, long rows_pad);
/* SwiGLU weights gate_proj/up_proj [F, K] -> one fp8 [2F, K] matrix with gate and up rows interleaved in 16-row
 * sub-tiles (the pairing of the fused SwiGLU epilogue) + scales [K/128][2F][4]. */
int flite_quant_fp8_gateup(void* stream, const void* gate, const void* up, long ld_src, int F, int K, void* dst,
                           void* scales);
/* MXFP8 GEMM C = A8 . W8^T on the block-scaled MFMA (fp32 accumulate). K % 128 == 0; lda, ldw % 16 == 0. */
int flite_gemm_fp8(void* stream, int M, int N, int K, const void* A8, long lda, const void* a_scales,
                   long a_rows_pad, const void* W8, long ldw, const void* w_scales, long w_rows_pad,
                   const void* bias, int epilogue, void* out, long ldo, void* out_scales, long out_rows_pad,
                   const float* gate, long gate_seg_stride, int rows_per_seg);
/* flite_gemm_fp8 with the stream-K workspace of flite_gemm_bf16_ws (flite_gemm_workspace_bytes, zero-filled
 * once, left zeroed; launches sharing it must be stream-ordered): the launcher may cut a partial last wave of
 * 256x256 tiles into equal k-ranges over the CUs. */
int flite_gemm_fp8_ws(void* stream, int M, int N, int K, const void* A8, long lda, const void* a_scales,
                      long a_rows_pad, const void* W8, long ldw, const void* w_scales, long w_rows_pad,
                      const void* bias, int epilogue, void* out, long ldo, void* out_scales, long out_rows_pad,
                      const float* gate, long gate_seg_stride, int rows_per_seg, void* workspace);
/* flite_rmsnorm_modulate with MXFP8 output (fp32 x): y8 [rows, dim] bytes (row stride ldy) + scales. */
int flite_rmsnorm_modulate_fp8(void* stream, const float* x, long ldx, void* y8, long ldy, void* y_scales,
                               long rows_pad, const void* w, const float* shift, const float* scale,
                               long mod_seg_stride, long seg_rows, long rows, int dim, float eps);

/* Row gather dst[i] = src[idx[i]] (bf16 rows of `cols`, cols % 8 == 0): the context compaction of
 * prepare_flash_attention_inputs (model.py:61-62) for a ragged context_attn_mask. idx: device int32 [n]. */
int flite_gather_rows(void* stream, const void* src, void* dst, const int* idx, long n, int cols);

/* ---- text encoder (T5 v1.1 encoder; reference pipeline.py:126-175 encode_prompt) ----
 * Replaces the transformers T5EncoderModel forward the reference calls for prompt embeddings (pt.py:150-155:
 * the 4096-wide context of cross_attn_input_size = 4096). GEMMs go through flite_gemm_bf16 (GEGLU epilogue
 * for DenseGatedActDense), norms through flite_rmsnorm_modulate (no modulation).
 *
 * Self-attention of one layer (T5Attention, no 1/sqrt(d) scaling): o = softmax(q k^T + bias + mask) v per head
 * of 64, for L <= 512 tokens per sequence, B sequences of L rows each. bucket: device int32 [2L-1], the
 * relative-position bucket of (key - query), indexed (key - query + L - 1); rel_weight: layer 0's
 * relative_attention_bias.weight [num_buckets, H] (bf16); mask: additive fp32 [B, L] over keys (0 keep,
 * -inf drop) or NULL. q/k/v/o: bf16 rows, head h at column 64 h, row strides in elements. */
int flite_t5_attention(void* stream, const void* q, long ldq, const void* k, long ldk, const void* v, long ldv,
                       void* o, long ldo, const int* bucket, const void* rel_weight, const float* mask, int B,
                       int L, int H);

/* Token-embedding gather into an fp32 residual stream: out[i][:] = float(table[ids[i]][:]) (bf16 table
 * [vocab, cols], ids clamped to [0, vocab), cols % 4 == 0). */
int flite_embed_rows_f32(void* stream, const void* table, const int* ids, float* out, long n, int cols, long vocab);

/* TwoDimRotary tables (model.py:334-386) for an (h, w) patch grid with n_reg leading register rows. */
int flite_rope_tables(void* stream, float* cos_t, float* sin_t, int h, int w, int n_reg, float base, int round_bf16);

/* timestep_embedding (model.py:20-28) of t*1000 to bf16 [n, dim]; quantize=1 reproduces the bf16 pipeline
 * (t -> bf16, t*1000 -> bf16; pipeline.py:260, model.py:551). */
int flite_timestep_embedding(void* stream, const float* t, void* emb, int n, int dim, int quantize);

/*
 * Deterministic synthetic parameters (no weights are shipped): fills `out` ([numel], bf16 or
 * fp32) with the splitmix64 counter-hash generator of oracle/weights.py keyed by (seed, name), uniform with
 * standard deviation `std`; ones=1 fills 1.0 (norm weights). Bit-identical to the CPU generator.
 */
int flite_init_param(void* stream, void* out, int out_is_bf16, long numel, const char* name, unsigned long long seed,
                     double std, int ones);

/* ---------------------------------------------------------------------------------------------
 * Model-level engine: the DiT forward (model.py:525-591 / model_v2.py:528-594) and the denoise loop
 * (pipeline.py:250-297) as native launch sequences; weights are caller-owned device tensors bound by
 * their state-dict names (model.py:417-479); the engine owns only its workspace.
 * ------------------------------------------------------------------------------------------- */
typedef struct flite_dit_config {
  int in_channels;            /* DiT(in_channels=...)                         */
  int patch_size;             /* patch_size                                   */
  int hidden_size;            /* hidden_size (num_heads * 256)                */
  int depth;                  /* depth                                        */
  int num_heads;              /* num_heads                                    */
  int mlp_hidden;             /* int(hidden_size * mlp_ratio)                 */
  int cross_attn_input_size;  /* cross_attn_input_size                        */
  int train_bias_and_rms;     /* qkv/q/kv biases + final_norm weight          */
  int per_block_adaln;        /* 1 = model_v2.py layout (adaLN per block, cross-attn in every block) */
  int n_register_tokens;      /* 16 (model.py:446)                            */
  float rope_base;            /* rope_base                                    */
  int bf16_timestep_quant;    /* 1 = bf16 model semantics for t  */
  int bf16_rope_tables;       /* 1 = RoPE tables rounded to bf16 (bf16 model) */
  int use_rope;               /* 1 = 2-D RoPE (model.py:537-544); 0 = learned positional_embedding
                                 [1, 2048, D] added to the register+patch rows (model.py:444,546), no RoPE */
} flite_dit_config;

typedef struct flite_dit flite_dit;

int flite_dit_create(const flite_dit_config* cfg, flite_dit** out);
int flite_dit_destroy(flite_dit* dit);
/* Bind one parameter by its state-dict key (e.g. "blocks.3.self_attn.qkv.weight"); bf16 device memory. */
int flite_dit_bind(flite_dit* dit, const char* name, const void* ptr, long numel);
/* Allocate the workspace for batch B (CFG included) of latents [C, h, w]; up to n_ctx context rows and
 * n_t timestep rows. Re-entrant: a call with an equal/smaller shape is a no-op. */
int flite_dit_prepare(flite_dit* dit, int batch, int latent_h, int latent_w, int n_ctx, int n_t);
/* Context embeddings [cu[batch], cross_attn_input_size] bf16, packed by host cu_seqlens [batch+1]:
 * context_proj + context_norm + per-block cross-attention K/V (step-invariant cache). Also finds the leading
 * sequences whose context rows are all bit-identical (the pipeline's zero negative prompt, pipeline.py:160-161) and
 * makes their step-invariant cross-attention output per block (the uniform-context collapse; env
 * FLITE_NO_CTX_COLLAPSE=1 disables it). That test reads one int per sequence back to the host, so this call
 * synchronises `stream` and is not graph-capturable (forward / sample are). */
int flite_dit_set_context(flite_dit* dit, void* stream, const void* ctx, const int* cu_seqlens_host, int batch);
/* Timesteps (device fp32 [n]): time embedding + adaLN/final modulation rows. quantize=1: the timesteps
 * tensor is bf16 in the reference call, so t and t*1000 are rounded to bf16 (pipeline.py:260, model.py:551). */
int flite_dit_set_timesteps(flite_dit* dit, void* stream, const float* t, int n, int quantize);
/* DiT forward of latents [batch, C, h, w] (fp32 or bf16); sample b uses timestep row t_row0 + b*t_row_step.
 * Output [batch, C, h, w] in out (bf16 if out_is_bf16 else fp32). */
int flite_dit_forward(flite_dit* dit, void* stream, const void* x, int x_is_bf16, int batch, int t_row0,
                      int t_row_step, void* out, int out_is_bf16);
/*
 * The rectified-flow denoise loop of FLitePipeline.__call__ (pipeline.py:250-297) for n_img images:
 * per step the CFG batch [latents; latents] (uncond context first) runs through the DiT, then
 * CFG (u + g(c-u)) or APG combine and the Euler update acc += dt*v, with acc fp32 [n_img, C, h, w]
 * updated in place. t/dt are host arrays [n_steps]. use_graph=1 captures the loop in one hipGraph.
 */
int flite_dit_sample(flite_dit* dit, void* stream, float* acc, int n_img, int n_steps, const float* t_host,
                     const float* dt_host, float guidance, int use_cfg, int apg, float apg_threshold,
                     int use_graph);
/*
 * CFG combine + Euler update of pipeline.py:290,296-297 on NCHW fp32 branch outputs [n elements]:
 * acc += dt * (use_cfg ? u + g (c - u) : c). Used by the CFG-parallel latency mode, where
 * the uncond and cond branches of one image run on two ranks and are exchanged before the update; the fp32
 * arithmetic is that of flite_dit_sample's fused update.
 */
int flite_cfg_euler(void* stream, const float* uncond, const float* cond, float* acc, long n, float guidance,
                    float dt, int use_cfg);
/*
 * APG (pipeline.py:276-287) on NCHW fp32 branch outputs, split at its two batch-global reductions so that
 * ranks holding different images of one reference batch can all-reduce the partial sums in between (SURVEY §8e;
 * the CFG-parallel mode calls them without a collective). out2 (device, 2 floats):
 *   phase 0: [sum c (c - u), sum c^2]             -> k = sum0 / sum1 (0 if sum1 == 0)
 *   phase 1: [sum o, sum o^2], o = (c - u) - k c  -> unbiased std s of o, orth_scale = min(1, threshold / s)
 * flite_apg_euler: acc += dt * (c + (guidance - 1) * orth_scale * o). The sums use flite_dit_sample's APG
 * kernel's expressions and summation order (bit-identical when one rank holds the whole batch).
 */
int flite_apg_sums(void* stream, const float* uncond, const float* cond, long n, float k, int phase, float* out2);
int flite_apg_euler(void* stream, const float* uncond, const float* cond, float* acc, long n, float guidance,
                    float k, float orth_scale, float dt);
/*
 * The same APG split with the scalars kept on the device (no host round trip per step; replaces the host algebra
 * between pipeline.py:281 and :285). ws4 = 4 device floats: flite_apg_sums_dev(phase 0) writes ws4[0..1] = [sum
 * c (c - u), sum c^2]; phase 1 derives k = ws4[0] / ws4[1] and writes ws4[2..3] = [sum o, sum o^2]. Between the
 * phases the caller may all-reduce ws4[0..1] (resp. ws4[2..3]) in place on the same stream order.
 * flite_apg_euler_dev derives k and orth_scale = min(1, threshold / std) (unbiased std over n_total elements, the
 * whole reference batch) from ws4 with the fp32 expressions of flite_dit_sample's APG kernel, then updates acc.
 */
int flite_apg_sums_dev(void* stream, const float* uncond, const float* cond, long n, int phase, float* ws4);
int flite_apg_euler_dev(void* stream, const float* uncond, const float* cond, float* acc, long n, float guidance,
                        float threshold, long n_total, const float* ws4, float dt);
/*
 * fp8 mode (BASELINE.json configs[4]): enable=1 quantises every bound block GEMM weight (qkv, proj, cross q /
 * proj, SwiGLU gate|up, down) once into engine-owned MXFP8 copies and runs those GEMMs on the block-scaled fp8
 * MFMA with MXFP8 activations (RMSNorm+modulate, attention output and SwiGLU output quantised where they are
 * produced). Attention, norms, RoPE, the residual stream and the small GEMMs stay bf16/fp32. enable=0 returns to
 * the bf16 path. enable=1 always requantises from the weights bound now. Re-binding a weight to new storage
 * keeps fp8 mode on: the next flite_dit_forward / flite_dit_sample requantises before it runs.
 */
int flite_dit_enable_fp8(flite_dit* dit, void* stream, int enable);
/*
 * fp8 precision policy: the `n` listed blocks keep the bf16 GEMMs (run as in bf16 mode) while fp8 mode is on; the
 * others run MXFP8. n = 0 (the default) puts every block on fp8. Blocks are self-contained between residual-stream
 * reads and writes (fp32), so any mix is valid. No reference counterpart (the reference is bf16 only).
 */
int flite_dit_set_fp8_bf16_blocks(flite_dit* dit, const int* blocks, int n);
/*
 * fp8 precision policy by GEMM class (round 5): in the fp8 blocks only the classes in `mask` run MXFP8, the others
 * run their bf16 GEMMs on bf16 operands (each activation is produced in the format its consumer takes: the norm,
 * the attention epilogue and the SwiGLU epilogue write bf16 or MXFP8 accordingly). Default FLITE_FP8_ALL. Classes:
 * qkv (model.py:151), self-attention proj (:212), cross q (:196), cross proj (:212 of the cross block), SwiGLU
 * gate|up (:261-267) and down (:267).
 */
#define FLITE_FP8_QKV 1
#define FLITE_FP8_PROJ 2
#define FLITE_FP8_CROSS_Q 4
#define FLITE_FP8_CROSS_PROJ 8
#define FLITE_FP8_GATE_UP 16
#define FLITE_FP8_DOWN 32
#define FLITE_FP8_ALL 63
int flite_dit_set_fp8_gemm_classes(flite_dit* dit, int mask);
/*
 * fp8 precision policy per block (round 6): masks[i] = the FLITE_FP8_* classes block i runs on MXFP8 (0 = the
 * whole block bf16), one mask per block (n_blocks = depth); n_blocks = 0 returns to the single mask of
 * flite_dit_set_fp8_gemm_classes. flite_dit_set_fp8_bf16_blocks still forces its blocks to bf16. The classes are
 * those of model.py:151-156,212 (attention) and :261-267 (SwiGLU MLP) per DiTBlock.
 */
int flite_dit_set_fp8_block_classes(flite_dit* dit, const int* masks, int n_blocks);
/*
 * Residual-stream storage (round 6): enable=1 (the default) keeps the DiTBlock residual x (model.py:289,297,301) in
 * bf16, the reference's own storage type; enable=0 keeps it in fp32. Every update stays one fp32 fma rounded once
 * (the reference rounds gate*f and x + (.) separately, model.py:289); in bf16 the norms read 2 B per element
 * instead of 4 and the gated-residual GEMM epilogues move 4 B instead of 8 (+1.55 % images/s at the metric
 * workload). Drops a cached graph; takes effect at the next forward / sample.
 */
int flite_dit_set_residual_bf16(flite_dit* dit, int enable);
/* 1: the residual stream is bf16 (the default unless FLITE_RESID_BF16=0 at engine creation), 0: fp32, -1: error */
int flite_dit_residual_bf16(flite_dit* dit);
/*
 * The CONTENTS of bound weights changed in place (a load_state_dict copy, a LoRA merge, re-initialisation):
 * every engine-owned copy derived from them is remade -- in fp8 mode the MXFP8 weights are requantised on
 * `stream` now. The bf16 path reads the bound storage directly. The cross-attention K/V cached by
 * flite_dit_set_context were projected with the old weights: after this call (or a re-bind to new storage)
 * flite_dit_forward / flite_dit_sample fail until flite_dit_set_context runs again. No reference counterpart
 * (nn.Linear reads its parameters on every call).
 */
int flite_dit_weights_updated(flite_dit* dit, void* stream);

/* ---- sequence parallelism: one image's rows over `nranks` GPUs ("ring attention over T")
 * Rank r holds rows [r*Tl, (r+1)*Tl) of every sequence, Tl = ceil(T / nranks) (T = 16 registers + patches;
 * the last rank's rows past T are padding). Every GEMM, norm and the cross-attention are row-local; the
 * self-attention of a block needs every key, so after the qkv GEMM each rank's K/V rows are all-gathered and
 * reordered into whole sequences; after the final projection the output rows are all-gathered, so every rank
 * ends each forward with the full model output and runs the same CFG/Euler update (flite_dit_sample with
 * use_graph = 0, or flite_dit_forward + flite_cfg_euler). The exchange is the host's: `fn(user, which,
 * stream)` must all-gather the caller-bound send buffer of `which` (0 = K/V rows, 1 = output rows) into its
 * receive buffer (nranks x send bytes, rank order) on `stream` (RCCL all_gather over xGMI; gloo in tests).
 * Call before flite_dit_prepare; then size (flite_dit_sp_buffer_bytes) and bind the four buffers. bf16 path
 * only (not with flite_dit_enable_fp8), learned-positional-embedding models excluded. */
typedef int (*flite_sp_allgather_fn)(void* user, int which, void* stream);
int flite_dit_set_sequence_parallel(flite_dit* dit, int rank, int nranks, flite_sp_allgather_fn fn, void* user);
int flite_dit_sp_buffer_bytes(flite_dit* dit, long* kv_send_bytes, long* out_send_bytes);
int flite_dit_sp_bind_buffers(flite_dit* dit, void* kv_send, void* kv_recv, void* out_send, void* out_recv);
/* Ring exchange for the self-attention's keys (ring != 0; default 0 = one all-gather overlapped with the own-key
 * attention). The K/V rows then travel as N - 1 neighbour shifts, each overlapped with the attention over the
 * previous block: `fn(user, which >= 2, stream)` is shift k = which - 1 (k = 1 .. N-1) and must send a block of
 * kv_send bytes to rank (r + 1) mod N and receive one from rank (r - 1) mod N, on `stream`. Source: kv_send for
 * k = 1, else kv_recv slot (k - 2) & 1; destination: kv_recv slot (k - 1) & 1 (slot i = bytes
 * [i * kv_send_bytes, (i + 1) * kv_send_bytes) of kv_recv). RCCL send/recv over one xGMI link; gloo in tests.
 * Falls back to the all-gather when some rank holds no key ((N - 1) * Tl >= T). */
int flite_dit_sp_set_ring(flite_dit* dit, int ring);

/*
 * 3x3 convolution, padding 1, stride 1 (nn.Conv2d of the diffusers VAE decoder), optionally preceded by a
 * nearest-2x upsample (Upsample2D), as an implicit-GEMM on MFMA. x: NHWC bf16 [h, w, cin] (one image,
 * cin % 64 == 0); w_packed from flite_conv3x3_pack_weight ([cout][3][3][cin_pad], cin zero-padded to a
 * multiple of 64); out NHWC [H, W, cout] bf16 (or fp32); resid (optional, bf16, out layout) is added.
 */
int flite_conv3x3_pack_weight(void* stream, const void* w, void* packed, int cout, int cin, int cin_pad);
int flite_conv3x3_bf16(void* stream, const void* x, int batch, int h, int w, int cin, int upsample,
                       const void* w_packed, const void* bias, int cout, void* out, const void* resid,
                       int out_is_f32);
/* GroupNorm (+SiLU) over NHWC bf16 rows (torch.nn.GroupNorm semantics), groups <= 64; stats_workspace: device
 * double[FLITE_GROUP_NORM_WS_DOUBLES] (group sums and the per-workgroup partials of a fixed-order, atomic-free
 * reduction: bit-reproducible). */
#define FLITE_GROUP_NORM_WS_DOUBLES (2 * 64 + 1024 * 64)
int flite_group_norm(void* stream, const void* x, void* y, long rows, int channels, int groups, const void* gamma,
                     const void* beta, float eps, int silu, double* stats_workspace);

/* ---------------------------------------------------------------------------------------------
 * VAE decoder engine: diffusers AutoencoderKL.decode (FLUX.1 VAE config) as called at pipeline.py:301-307,
 * plus the uint8 post-processing of pipeline.py:324-326. Parameters bound by their diffusers state-dict keys
 * ("decoder.conv_in.weight", "decoder.up_blocks.2.resnets.0.conv_shortcut.weight", ...).
 * ------------------------------------------------------------------------------------------- */
typedef struct flite_vae_config {
  int latent_channels;        /* 16 */
  int n_blocks;               /* len(block_out_channels) = 4 */
  int block_out_channels[4];  /* (128, 256, 512, 512) */
  int layers_per_block;       /* 2 (decoder uses layers_per_block + 1 resnets per up block) */
  int norm_groups;            /* 32 */
  int mid_attention;          /* 1 */
} flite_vae_config;

typedef struct flite_vae flite_vae;

int flite_vae_create(const flite_vae_config* cfg, flite_vae** out);
int flite_vae_destroy(flite_vae* vae);
int flite_vae_bind(flite_vae* vae, const char* name, const void* ptr, long numel);
/* Workspace + packed conv weights for latents of [latent_channels, latent_h, latent_w]. */
/* fp8 weight storage (diffusers' layerwise casting with an fp8 storage dtype, compute bf16; no reference
 * counterpart: SURVEY 8f rank 4): the packed 3x3 conv weights are kept as MXFP8 (e4m3 + one E8M0 scale per 32
 * input-channel values of a tap) and expanded to bf16 right before each conv. Takes effect at the next prepare. */
int flite_vae_enable_fp8_weights(flite_vae* vae, int on);
/* The CONTENTS of bound weights changed in place: re-pack (and, with fp8 storage, requantise) the engine's conv
 * weights for the prepared shape now. */
int flite_vae_weights_updated(flite_vae* vae);
int flite_vae_prepare(flite_vae* vae, int latent_h, int latent_w);
/* latents fp32 [n_img, C, h, w] -> images uint8 [n_img, 8h, 8w, 3] (device), decoding z/scaling + shift. */
int flite_vae_decode_uint8(flite_vae* vae, void* stream, const float* latents, int n_img, void* images,
                           float scaling_factor, float shift_factor);
/*
 * Tiled decode, diffusers AutoencoderKL.tiled_decode / blend_v / blend_h (the reference turns it on with
 * pipe.vae.enable_tiling(), generate.py:77-78 / pipeline.py:90-93; AutoencoderKL.decode takes it when a latent
 * side exceeds tile_latent = sample_size / 8, e.g. the 1344x896 default). Latent tiles of tile_latent every
 * int(tile_latent * (1 - overlap_factor)); decoded tiles blended with their upper then left neighbour over
 * int(tile_sample * overlap_factor) pixels (linear ramp), cropped to tile_sample minus that, concatenated, then
 * post-processed to uint8. The FLUX VAE: tile_latent 128, tile_sample 1024, overlap_factor 0.25. Blending is
 * in fp32 (diffusers blends in the VAE dtype).
 */
int flite_vae_prepare_tiled(flite_vae* vae, int latent_h, int latent_w, int tile_latent, int tile_sample,
                            float overlap_factor);
/* latents fp32 [n_img, C, latent_h, latent_w] -> images uint8 [n_img, 8 latent_h, 8 latent_w, 3], tiled. */
int flite_vae_decode_tiled_uint8(flite_vae* vae, void* stream, const float* latents, int n_img, void* images,
                                 float scaling_factor, float shift_factor);

/*
 * Launch probe (measurement): bracket every launch of one kernel class with a pair of HIP events on the
 * stream it is launched on (inside the captured loop too). read returns the per-launch milliseconds of the
 * latest run (pairs in launch order). kind < 0 disables.
 */
#define FLITE_PROBE_GEMM_GATEUP 0 /* SwiGLU gate/up GEMM (largest kernel, ~38% of FLOPs) */
#define FLITE_PROBE_ATTN_SELF 1   /* self-attention flash kernel */
#define FLITE_PROBE_GEMM_DOWN 2   /* MLP down-projection GEMM + gated residual */
#define FLITE_PROBE_GEMM_QKV 3    /* qkv projection GEMM */
#define FLITE_PROBE_STEP 4        /* one whole denoise step (DiT forward + CFG/Euler) */
int flite_dit_set_probe(flite_dit* dit, int kind, int max_pairs);
int flite_dit_read_probe(flite_dit* dit, float* ms, int cap, int* n);

#ifdef __cplusplus
}
#endif

#endif /* FLITE_H_ */
