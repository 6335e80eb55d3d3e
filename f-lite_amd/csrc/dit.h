// Native DiT engine: owns the workspace and drives the per-step forward of f_lite/model.py
// (DiT.forward, model.py:525-591 / model_v2.py:528-594) and the denoise loop of FLitePipeline.__call__
// (pipeline.py:250-297) as a sequence of gfx950 kernel launches, optionally captured into one hipGraph.
#pragma once
#include <map>
#include <string>
#include <vector>

#include "../../include/flite.h"
#include "common.h"
#include "fp8.h"
#include "kernels.h"

namespace flite {

struct BlockW {
  bool cross = false;
  const bf16_t *norm1 = nullptr, *qkv_w = nullptr, *qkv_b = nullptr, *proj_w = nullptr;
  const bf16_t *norm2 = nullptr, *cq_w = nullptr, *cq_b = nullptr, *ckv_w = nullptr, *ckv_b = nullptr,
               *cproj_w = nullptr;
  const bf16_t *norm3 = nullptr, *gate_w = nullptr, *up_w = nullptr, *down_w = nullptr;
  const bf16_t *ada_w = nullptr, *ada_b = nullptr;  // per-block adaLN (model_v2 layout)
};

struct DitW {
  const bf16_t *ctx_proj_w = nullptr, *ctx_proj_b = nullptr, *ctx_norm = nullptr;
  const bf16_t *patch_w = nullptr, *patch_b = nullptr, *registers = nullptr;
  const bf16_t* pos_emb = nullptr;  // positional_embedding [1, 2048, D] (use_rope = 0)
  const bf16_t *te0_w = nullptr, *te0_b = nullptr, *te2_w = nullptr, *te2_b = nullptr;
  const bf16_t *ada_w = nullptr, *ada_b = nullptr;  // shared adaLN (model.py layout)
  const bf16_t *fmod_w = nullptr, *fmod_b = nullptr, *fnorm = nullptr, *fproj_w = nullptr, *fproj_b = nullptr;
  std::vector<BlockW> blocks;
};

class DitEngine {
 public:
  explicit DitEngine(const flite_dit_config& cfg);
  ~DitEngine();

  int bind(const std::string& name, const void* ptr, long numel);
  int check_bound();
  int prepare(int B, int Hl, int Wl, int n_ctx_max, int n_t_max);
  int set_context(hipStream_t s, const void* ctx, const int* cu_host, int nseq);
  int set_timesteps(hipStream_t s, const float* t_dev, int n, int quantize);
  // forward of the B = dup*Bi batch; segment b uses timestep row t_row0 + b*t_row_step
  int forward(hipStream_t s, const void* lat, bool lat_bf16, int Bi, int dup, int t_row0, int t_row_step);
  int unpatchify_out(hipStream_t s, void* y, bool out_bf16);
  int sample(hipStream_t s, float* acc, int Bi, int n_steps, const float* t_host, const float* dt_host,
             float guidance, int use_cfg, int apg, float apg_thr, int use_graph);

  // fp8 mode (flite_dit_enable_fp8): MXFP8 copies of the block GEMM weights + fp8 activations
  int enable_fp8(hipStream_t s, bool on);
  int set_fp8_bf16_blocks(const int* blocks, int n);
  int set_fp8_classes(int mask);
  // per-block class masks (flite_dit_set_fp8_block_classes): n = depth masks, or n = 0 to use set_fp8_classes' one
  int set_fp8_block_classes(const int* masks, int n);
  // residual stream storage: fp32 (default) or bf16 (drops the cached graph)
  int set_residual_bf16(bool on);
  bool residual_bf16() const { return x16_; }
  // the bound weights' CONTENTS changed in place (flite_dit_weights_updated): requantise the fp8 copies
  int weights_updated(hipStream_t s);

  // sequence parallelism (flite_dit_set_sequence_parallel)
  int set_sequence_parallel(int rank, int nranks, flite_sp_allgather_fn fn, void* user);
  int sp_buffer_bytes(long* kv_send, long* out_send) const;
  int sp_bind_buffers(void* kv_send, void* kv_recv, void* out_send, void* out_recv);
  int set_sp_ring(int on);

  const flite_dit_config cfg;
  int D, H, F, R, P, C;

  // launch probe: HIP event pairs around every launch of one kernel class (FLITE_PROBE_*), on the stream
  // the kernel is launched on (also inside a captured graph, as event-record nodes)
  int set_probe(int kind, int max_pairs);
  int read_probe(float* ms, int cap, int* n);

 private:
  int probe_begin(hipStream_t s, int kind);
  int probe_end(hipStream_t s, int kind);
  int probe_kind_ = -1;
  std::vector<hipEvent_t> probe_ev_;
  int probe_n_ = 0;

  int run_block(hipStream_t s, int blk, const float* mod, long mseg);
  int sp_gather_kv(hipStream_t s);
  int sp_self_attention(hipStream_t s, AttnParams a);
  int sp_ring_attention(hipStream_t s, AttnParams a);
  int sp_gather_out(hipStream_t s);
  int run_block_fp8(hipStream_t s, int blk, const float* mod, long mseg, int classes);
  int alloc_fp8_act();
  int quantise_fp8(hipStream_t s);
  void free_fp8_weights();
  int alloc(void** p, size_t bytes);
  void free_ws();
  void drop_graph();
  int gemm(GemmParams& g, int epi, hipStream_t s);

  DitW w_;
  std::map<std::string, std::pair<const void*, long>> bound_;
  std::vector<void*> allocs_;
  // shape
  int B_ = 0, Hl_ = 0, Wl_ = 0, T_ = 0, HW_ = 0, ntmax_ = 0, nctx_max_ = 0;
  int Tl_ = 0;  // rows of each sequence held here (T_ without sequence parallelism)
  // sequence parallelism
  int sp_rank_ = 0, sp_n_ = 1;
  flite_sp_allgather_fn sp_fn_ = nullptr;
  void* sp_user_ = nullptr;
  bf16_t *sp_kv_send_ = nullptr, *sp_kv_recv_ = nullptr, *kv_full_ = nullptr;
  float *sp_out_send_ = nullptr, *sp_out_recv_ = nullptr;
  int *cu_full_ = nullptr;
  // overlapped exchange (sp_self_attention): partial (O, l) of the local keys, the local key-range ends, the
  // remote keys' cu_seqlens, and the side stream the K/V all-gather runs on
  float *part_o_ = nullptr, *part_l_ = nullptr;
  int *kend_loc_ = nullptr, *cu_rem_ = nullptr;
  hipStream_t xstream_ = nullptr;
  hipEvent_t ev_kv_ = nullptr, ev_x_ = nullptr;
  bool sp_overlap_ = true;
  // ring exchange (sp_ring_attention): N - 1 neighbour shifts of one rank's K/V block, each overlapped with the
  // attention over the block before it; kend_all_[q][b] = key-range end of rank q's block in sequence b
  bool sp_ring_ = false;
  int* kend_all_ = nullptr;
  hipEvent_t ev_ring_[2] = {nullptr, nullptr}, ev_used_[2] = {nullptr, nullptr};
  bool attn_mx_ = true;  // fp8 path: the attention writes the proj GEMM's MXFP8 operand itself
  long M_ = 0;
  int sa_seqs_ = 0;  // > 0: block 0's self-attention on the first sa_seqs_ sequences only (forward, CFG batch)
  int nctx_ = 0, nseq_ctx_ = 0, ctx_max_len_ = 0;
  // uniform-context collapse (set_context, run_block): the first ctx_uni_ sequences have context rows that are all
  // equal (the pipeline's zero negative prompt, pipeline.py:160-161); ctx_c_[blk][seq] = V row . Wproj^T (fp32)
  int ctx_uni_ = 0;
  float* ctx_c_ = nullptr;
  bf16_t* ctx_vrow_ = nullptr;
  int* ctx_bad_ = nullptr;
  std::vector<int> ctx_row0_;  // first context row of each collapsed sequence (its V row in ctx_kv_)
  // fp8 blocks: the same c from the MXFP8 V row and cross-proj weights (collapse_fp8, before the first fp8 use after
  // set_context or a requantisation); only where the collapsed rows end on a 4-row boundary (uni_fp8)
  float* ctx_c8_ = nullptr;
  uint8_t *ctx_vrow8_ = nullptr, *ctx_vrow8_s_ = nullptr;
  long vrow8_rows_pad_ = 256;  // scale rows of ctx_vrow8_s_ (mx_rows_pad(B))
  bool ctx_c8_stale_ = true;
  int collapse_fp8(hipStream_t s);
  int uni_fp8() const;
  // workspace
  // residual stream [M, D]: bf16 (x16_, the default since round 6: the reference's own storage type, model.py:289) or
  // fp32 (flite_dit_set_residual_bf16(dit, 0)). Every writer is an fp32 fma with one rounding; the buffer is sized
  // for fp32 either way.
  void* x_ = nullptr;
  bool x16_ = true;
  size_t xbytes() const { return x16_ ? 2 : 4; }
  void* xrow(long r) const { return (char*)x_ + r * (long)D * (long)xbytes(); }
  int epi_resid() const { return x16_ ? EPI_RESID_BF16 : EPI_RESID_F32; }
  int epi8_resid() const { return x16_ ? EPI8_RESID_BF16 : EPI8_RESID_F32; }
  bf16_t *nbuf_ = nullptr, *qkv_ = nullptr, *obuf_ = nullptr, *hbuf_ = nullptr, *patches_ = nullptr;
  float* fout_ = nullptr;
  float* acc_ = nullptr;  // graph-owned Euler accumulator (sample)
  float* sk_ws_ = nullptr;  // stream-K GEMM partial tiles
  int* sk_flags_ = nullptr;
  void* attn_ws_ = nullptr;  // attention tail-split slabs + counters (attention.hip "Schedule")
  long attn_ws_bytes_ = 0;
  int *cu_self_ = nullptr, *cu_ctx_ = nullptr;
  float *cos_ = nullptr, *sin_ = nullptr, *inv_freq_ = nullptr;
  float* rope_axes_ = nullptr;  // factorised table of the fused qkv epilogues (common.h RopeAxes)
  RopeAxes rope_axes() const;
  bf16_t* ctx_p_ = nullptr;
  std::vector<bf16_t*> ctx_kv_;  // per block (cross blocks only)
  float* tdev_ = nullptr;
  bf16_t *temb_ = nullptr, *th_ = nullptr;  // sinusoid / hidden
  bf16_t* tsilu_ = nullptr;                 // silu(t_emb)
  float* mod_ = nullptr;                    // [n_t][depth or 1][9D]
  float* fmod_ = nullptr;                   // [n_t][2D]
  float* apg_scratch_ = nullptr;
  long mod_t_stride_ = 0;
  int nt_ = 0;
  // fp8 mode
  struct Fp8W {
    uint8_t *qkv = nullptr, *qkv_s = nullptr, *proj = nullptr, *proj_s = nullptr, *cq = nullptr, *cq_s = nullptr;
    uint8_t *cproj = nullptr, *cproj_s = nullptr, *gu = nullptr, *gu_s = nullptr, *down = nullptr, *down_s = nullptr;
  };
  bool fp8_ = false;
  std::vector<char> fp8_bf16_blk_;  // blocks that stay bf16 in fp8 mode (flite_dit_set_fp8_bf16_blocks)
  int fp8_classes_ = 63;            // GEMM classes on MXFP8 in the fp8 blocks (flite_dit_set_fp8_gemm_classes)
  std::vector<int> fp8_blk_mask_;   // per-block classes (flite_dit_set_fp8_block_classes); empty = fp8_classes_
  bool w8_stale_ = true;  // the fp8 copies do not reflect the bound bf16 weights (requantised before the next use)
  bool ctx_stale_ = false;  // a weight changed after set_context: the cached context K/V are stale
  std::vector<Fp8W> w8_;
  std::vector<void*> w8_allocs_;
  uint8_t *nbuf8_ = nullptr, *nbuf8_s_ = nullptr, *obuf8_ = nullptr, *obuf8_s_ = nullptr;
  uint8_t *hbuf8_ = nullptr, *hbuf8_s_ = nullptr;
  long mpad_ = 0;
  // graph cache
  hipStream_t gstream_ = nullptr;
  hipGraphExec_t gexec_ = nullptr;
  std::vector<float> gkey_;
  hipEvent_t ev_in_ = nullptr, ev_out_ = nullptr;
};

}  // namespace flite
