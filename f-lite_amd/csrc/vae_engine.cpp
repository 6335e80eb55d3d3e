// Native Flux VAE decoder (diffusers AutoencoderKL.decode with the FLUX.1 VAE config: latent_channels 16,
// block_out_channels (128, 256, 512, 512), layers_per_block 2, 32 groups, mid-block attention), called by the
// reference at pipeline.py:301-307 after `latents / scaling_factor + shift_factor`, followed by the uint8
// post-processing of pipeline.py:324-326. NHWC bf16 activations; convs = implicit-GEMM MFMA (gemm.hip).
#include <algorithm>
#include <map>
#include <string>
#include <vector>

#include "../../include/flite.h"
#include "common.h"
#include "kernels.h"

namespace flite {

class VaeEngine {
 public:
  explicit VaeEngine(const flite_vae_config& c) : cfg(c) {}
  ~VaeEngine() {
    free_ws();
    free_tiles();
  }

  // fp8 weight storage (diffusers' layerwise casting with an fp8 storage dtype, compute bf16): every packed 3x3
  // conv weight is kept as MXFP8 (e4m3 + one E8M0 scale per 32 of K) and expanded to bf16 right before its conv.
  // 1.03 instead of 2 bytes per weight; the convs themselves run in bf16 as before.
  int enable_fp8_weights(bool on) {
    if (on != fp8_w_) {
      fp8_w_ = on;
      packed_.clear();  // re-pack (and re-allocate) on the next prepare
    }
    return 0;
  }
  bool fp8_weights() const { return fp8_w_; }

  // the bound weights changed in place: re-pack (and requantise) now, for the prepared shape
  int weights_updated() {
    if (h_ == 0) return 0;  // nothing packed yet: the first prepare packs
    const int h = h_, w = w_;
    packed_.clear();
    return prepare(h, w);
  }

  int bind(const std::string& name, const void* p, long n) {
    FLITE_REQUIRE(p != nullptr && ((uintptr_t)p & 15) == 0, "vae bind: null or unaligned " + name);
    params_[name] = {(const bf16_t*)p, n};
    packed_.clear();  // re-pack on next prepare
    return 0;
  }

  int prepare(int h, int w) {
    FLITE_REQUIRE(cfg.n_blocks == 4, "vae: 4 decoder blocks expected");
    if (h == h_ && w == w_ && !packed_.empty()) return 0;
    free_ws();
    h_ = h;
    w_ = w;
    const long H = (long)h << (cfg.n_blocks - 1), W = (long)w << (cfg.n_blocks - 1);
    long maxe = (long)h * w * 64;
    // largest activation: any level's HW x max channels at that level (incl. the upsampled conv inputs)
    long hw = (long)h * w;
    int cprev = cfg.block_out_channels[cfg.n_blocks - 1];
    for (int i = 0; i < cfg.n_blocks; ++i) {
      const int cout = cfg.block_out_channels[cfg.n_blocks - 1 - i];
      maxe = std::max(maxe, hw * std::max(cprev, cout));
      if (i < cfg.n_blocks - 1) {
        hw *= 4;
        maxe = std::max(maxe, hw * cout);
      }
      cprev = cout;
    }
    maxe = std::max(maxe, H * W * 4);
    for (int i = 0; i < 5; ++i)
      if (alloc((void**)&buf_[i], maxe * 2)) return 1;
    const long L = (long)h * w;  // mid-block attention tokens; the P.V k dimension is padded to 64
    const long Lp = (L + 63) / 64 * 64;
    const int Cm = cfg.block_out_channels[cfg.n_blocks - 1];
    if (alloc((void**)&S_, L * Lp * 4)) return 1;
    if (alloc((void**)&P_, L * Lp * 2)) return 1;
    if (alloc((void**)&vt_, Lp * Cm * 2)) return 1;
    if (alloc((void**)&stats_, FLITE_GROUP_NORM_WS_DOUBLES * sizeof(double))) return 1;
    if (alloc((void**)&out32_, H * W * 4 * 4)) return 1;
    return pack_all();
  }

  // decode one image: z fp32 [C, h, w] -> img uint8 [H, W, 3]
  int decode(hipStream_t s, const float* z, unsigned char* img, float scaling, float shift) {
    FLITE_REQUIRE(h_ > 0, "vae decode: call prepare first");
    RoctxRange range("flite.vae.decode");
    if (decode_core(s, z, (long)h_ * w_, w_, h_, w_, out32_, scaling, shift)) return 1;
    const long H = (long)h_ << (cfg.n_blocks - 1), W = (long)w_ << (cfg.n_blocks - 1);
    return to_uint8(out32_, 4, img, H * W, s);
  }

  // Tiled decode (diffusers AutoencoderKL.tiled_decode; the reference enables it at generate.py:77-78, and
  // AutoencoderKL.decode takes it when a latent side exceeds tile_latent). Latent tiles of tile_latent start
  // every stride = int(tile_latent * (1 - overlap)) rows / columns (the last ones smaller); each decodes to an
  // fp32 tile that is blended in place with its already-blended upper, then left neighbour over
  // e = int(tile_sample * overlap) pixels, then cropped to tile_sample - e and post-processed into the image.
  int prepare_tiled(int H, int W, int tile_latent, int tile_sample, float overlap) {
    FLITE_REQUIRE(H > 0 && W > 0 && tile_latent > 0 && tile_sample == tile_latent << (cfg.n_blocks - 1),
                  "vae prepare_tiled: tile_sample must be tile_latent x 8");
    const int stride = (int)(tile_latent * (1.0 - overlap));
    const int blend = (int)(tile_sample * overlap);
    FLITE_REQUIRE(stride > 0 && blend > 0 && blend < tile_sample, "vae prepare_tiled: overlap out of range");
    if (prepare(std::min(H, tile_latent), std::min(W, tile_latent))) return 1;
    if (H == tH_ && W == tW_ && tile_latent == tl_ && tile_sample == ts_ && stride == tstride_ && !tiles_.empty())
      return 0;
    free_tiles();
    tH_ = H;
    tW_ = W;
    tl_ = tile_latent;
    ts_ = tile_sample;
    tstride_ = stride;
    tblend_ = blend;
    for (int i = 0; i < H; i += stride) ti_.push_back(i);
    for (int j = 0; j < W; j += stride) tj_.push_back(j);
    for (int i : ti_)
      for (int j : tj_) {
        const long th = std::min(tile_latent, H - i), tw = std::min(tile_latent, W - j);
        void* p = nullptr;
        FLITE_HIP_CHECK(hipMalloc(&p, (th << (cfg.n_blocks - 1)) * (tw << (cfg.n_blocks - 1)) * 4 * sizeof(float)));
        tiles_.push_back((float*)p);
      }
    return 0;
  }

  // one image: z fp32 [C, tH, tW] -> img uint8 [8 tH, 8 tW, 3]
  int decode_tiled(hipStream_t s, const float* z, unsigned char* img, float scaling, float shift) {
    FLITE_REQUIRE(!tiles_.empty(), "vae decode_tiled: call prepare_tiled first");
    const int up = cfg.n_blocks - 1;
    const int nj = (int)tj_.size();
    auto th = [&](int a) { return std::min(tl_, tH_ - ti_[a]) << up; };  // decoded tile height (pixels)
    auto tw = [&](int b) { return std::min(tl_, tW_ - tj_[b]) << up; };
    for (size_t a = 0; a < ti_.size(); ++a)
      for (int b = 0; b < nj; ++b)
        if (decode_core(s, z + (long)ti_[a] * tW_ + tj_[b], (long)tH_ * tW_, tW_, th(a) >> up, tw(b) >> up,
                        tiles_[a * nj + b], scaling, shift))
          return 1;
    const int row_limit = ts_ - tblend_;
    int y0 = 0;
    for (size_t a = 0; a < ti_.size(); ++a) {
      int x0 = 0;
      for (int b = 0; b < nj; ++b) {
        float* t = tiles_[a * nj + b];
        if (a > 0) {
          const float* u = tiles_[(a - 1) * nj + b];
          if (tile_blend(u, th(a - 1), tw(b), t, th(a), tw(b), std::min({th(a - 1), th(a), tblend_}), true, s))
            return 1;
        }
        if (b > 0) {
          const float* l = tiles_[a * nj + b - 1];
          if (tile_blend(l, th(a), tw(b - 1), t, th(a), tw(b), std::min({tw(b - 1), tw(b), tblend_}), false, s))
            return 1;
        }
        const int rows = std::min(row_limit, th(a)), cols = std::min(row_limit, tw(b));
        if (tile_to_uint8(t, tw(b), img, tW_ << up, y0, x0, rows, cols, s)) return 1;
        x0 += cols;
      }
      y0 += std::min(row_limit, th(a));
    }
    return 0;
  }

  // the decoder network on the th x tw latent window at z (channel planes of `plane`, rows of `ldz`) ->
  // conv_out fp32 [8th * 8tw, 4] in out
  int decode_core(hipStream_t s, const float* z, long plane, int ldz, int th, int tw, float* out, float scaling,
                  float shift) {
    FLITE_REQUIRE(th > 0 && tw > 0 && (long)th * tw <= (long)h_ * w_ && th <= std::max(h_, w_) &&
                      tw <= std::max(h_, w_),
                  "vae decode: window larger than the prepared size");
    const int C0 = cfg.latent_channels;
    const int G = cfg.norm_groups;
    long h = th, w = tw;
    const int Cm = cfg.block_out_channels[cfg.n_blocks - 1];
    bf16_t* x = buf_[0];
    if (latent_to_nhwc(z, plane, ldz, th, tw, buf_[4], C0, 64, scaling, shift, s)) return 1;
    if (conv3(s, buf_[4], 64, h, w, false, "decoder.conv_in", Cm, x, nullptr)) return 1;
    int cur = 0;
    int C = Cm;
    // mid block (UNetMidBlock2D): resnet, attention, resnet
    if (resnet(s, "decoder.mid_block.resnets.0", cur, C, C, h, w)) return 1;
    if (cfg.mid_attention && attention(s, "decoder.mid_block.attentions.0", cur, C, h, w)) return 1;
    if (resnet(s, "decoder.mid_block.resnets.1", cur, C, C, h, w)) return 1;
    // up blocks (UpDecoderBlock2D x n_blocks over reversed block_out_channels)
    for (int i = 0; i < cfg.n_blocks; ++i) {
      const int cout = cfg.block_out_channels[cfg.n_blocks - 1 - i];
      for (int j = 0; j < cfg.layers_per_block + 1; ++j) {
        const std::string pre = "decoder.up_blocks." + std::to_string(i) + ".resnets." + std::to_string(j);
        if (resnet(s, pre, cur, C, cout, h, w)) return 1;
        C = cout;
      }
      if (i < cfg.n_blocks - 1) {  // Upsample2D: nearest 2x + conv (folded into the conv addressing)
        const int nxt = (cur + 1) % 4;
        if (conv3(s, buf_[cur], C, h, w, true, "decoder.up_blocks." + std::to_string(i) + ".upsamplers.0.conv", C,
                  buf_[nxt], nullptr))
          return 1;
        cur = nxt;
        h *= 2;
        w *= 2;
      }
    }
    // conv_norm_out + SiLU + conv_out -> uint8
    const int t = (cur + 1) % 4;
    if (gn(s, buf_[cur], buf_[t], h * w, C, "decoder.conv_norm_out", true)) return 1;
    {
      GemmParams g;
      if (conv_params(s, g, buf_[t], C, h, w, false, "decoder.conv_out", 3)) return 1;
      g.out = out;
      g.ldo = 4;
      if (gemm_bf16(g, EPI_STORE_F32, s)) return 1;
    }
    (void)G;
    return 0;
  }

  const flite_vae_config cfg;
  long latent_elems() const { return (long)cfg.latent_channels * h_ * w_; }
  long image_bytes() const { return 3L * ((long)h_ << (cfg.n_blocks - 1)) * ((long)w_ << (cfg.n_blocks - 1)); }
  long tiled_latent_elems() const { return (long)cfg.latent_channels * tH_ * tW_; }
  long tiled_image_bytes() const { return 3L * ((long)tH_ << (cfg.n_blocks - 1)) * ((long)tW_ << (cfg.n_blocks - 1)); }

 private:
  struct Param {
    const bf16_t* p;
    long n;
  };

  const bf16_t* P(const std::string& n) const {
    auto it = params_.find(n);
    return it == params_.end() ? nullptr : it->second.p;
  }

  int alloc(void** p, size_t bytes) {
    FLITE_HIP_CHECK(hipMalloc(p, bytes));
    allocs_.push_back(*p);
    return 0;
  }
  void free_ws() {
    for (void* p : allocs_) hipFree(p);
    allocs_.clear();
    packed_.clear();
    h_ = w_ = 0;
  }
  void free_tiles() {
    for (float* p : tiles_) hipFree(p);
    tiles_.clear();
    ti_.clear();
    tj_.clear();
    tH_ = tW_ = 0;
  }

  // pack every 3x3 conv weight [Cout][Cin][3][3] -> [Cout][3][3][Cin_pad] (fp8 storage: packed into the bf16
  // scratch, then quantised)
  int pack_all() {
    struct Conv {
      std::string base;
      const bf16_t* p;
      int cout, cin, cpad;
    };
    std::vector<Conv> convs;
    long most = 0;
    for (auto& kv : params_) {
      const std::string& n = kv.first;
      if (n.size() < 12 || n.compare(n.size() - 7, 7, ".weight") != 0) continue;
      const std::string base = n.substr(0, n.size() - 7);
      const bool conv3x3 = base == "decoder.conv_in" || base == "decoder.conv_out" ||
                           base.find(".conv1") != std::string::npos || base.find(".conv2") != std::string::npos ||
                           base.find("upsamplers.0.conv") != std::string::npos;
      if (!conv3x3) continue;
      const auto b = params_.find(base + ".bias");
      FLITE_REQUIRE(b != params_.end(), "vae: missing bias for " + base);
      const int cout = (int)b->second.n;
      FLITE_REQUIRE(kv.second.n % (9L * cout) == 0, "vae: bad conv weight " + n);
      const int cin = (int)(kv.second.n / (9L * cout));
      const int cpad = (cin + 63) / 64 * 64;
      convs.push_back({base, kv.second.p, cout, cin, cpad});
      most = std::max(most, 9L * cout * cpad);
    }
    w8_.clear();
    wscratch_ = nullptr;
    if (fp8_w_ && alloc((void**)&wscratch_, (size_t)most * 2)) return 1;
    for (const Conv& c : convs) {
      bf16_t* o = nullptr;
      if (fp8_w_) {
        const int K = 9 * c.cpad;
        uint8_t *q = nullptr, *sc = nullptr;
        if (alloc((void**)&q, (size_t)c.cout * K)) return 1;
        if (alloc((void**)&sc, (size_t)c.cout * (K / 32))) return 1;
        if (pack_conv_weight(c.p, wscratch_, c.cout, c.cin, c.cpad, 0)) return 1;
        if (mx_quant_rows_rm(wscratch_, c.cout, K, q, sc, 0)) return 1;
        w8_[c.base] = {q, sc};
      } else {
        if (alloc((void**)&o, (size_t)c.cout * 9 * c.cpad * 2)) return 1;
        if (pack_conv_weight(c.p, o, c.cout, c.cin, c.cpad, 0)) return 1;
      }
      packed_[c.base] = {o, c.cpad};
    }
    FLITE_HIP_CHECK(hipDeviceSynchronize());
    return 0;
  }

  int conv_params(hipStream_t s, GemmParams& g, const bf16_t* in, int cin, long h, long w, bool up,
                  const std::string& name, int cout) {
    auto it = packed_.find(name);
    FLITE_REQUIRE(it != packed_.end(), "vae: unbound conv " + name);
    FLITE_REQUIRE(it->second.second == cin, "vae: channel mismatch for " + name);
    const bf16_t* wt = it->second.first;
    if (fp8_w_) {  // expand the stored MXFP8 weight into the scratch (stream-ordered before this conv)
      const auto q = w8_.find(name);
      FLITE_REQUIRE(q != w8_.end(), "vae: fp8 weight missing for " + name);
      if (mx_dequant_rows_rm(q->second.first, q->second.second, cout, 9 * cin, wscratch_, s)) return 1;
      wt = wscratch_;
    }
    g.conv_in = in;
    g.conv_c = cin;
    g.conv_ih = (int)h;
    g.conv_iw = (int)w;
    g.conv_oh = (int)(up ? 2 * h : h);
    g.conv_ow = (int)(up ? 2 * w : w);
    g.conv_up = up ? 1 : 0;
    g.conv_in_bytes = h * w * cin * 2;
    g.W = wt;
    g.ldw = 9L * cin;
    g.bias = P(name + ".bias");
    g.M = g.conv_oh * g.conv_ow;
    g.N = cout;
    g.K = 9 * cin;
    return 0;
  }

  int conv3(hipStream_t s, const bf16_t* in, int cin, long h, long w, bool up, const std::string& name, int cout,
            bf16_t* out, const bf16_t* resid) {
    GemmParams g;
    if (conv_params(s, g, in, cin, h, w, up, name, cout)) return 1;
    g.out = out;
    g.ldo = cout;
    g.resid = resid;
    return gemm_bf16(g, EPI_STORE_BF16, s);
  }

  int gn(hipStream_t s, const bf16_t* x, bf16_t* y, long rows, int C, const std::string& name, bool silu) {
    const bf16_t* gw = P(name + ".weight");
    const bf16_t* gb = P(name + ".bias");
    FLITE_REQUIRE(gw && gb, "vae: unbound " + name);
    return group_norm(x, y, rows, C, cfg.norm_groups, gw, gb, 1e-6f, silu, stats_, s);
  }

  // ResnetBlock2D (temb None, groups 32, eps 1e-6, SiLU, output_scale_factor 1): in buf_[cur], out -> buf_[cur']
  int resnet(hipStream_t s, const std::string& pre, int& cur, int cin, int cout, long h, long w) {
    const int a = (cur + 1) % 4, b = (cur + 2) % 4, c = (cur + 3) % 4;
    bf16_t* x = buf_[cur];
    if (gn(s, x, buf_[a], h * w, cin, pre + ".norm1", true)) return 1;
    if (conv3(s, buf_[a], cin, h, w, false, pre + ".conv1", cout, buf_[b], nullptr)) return 1;
    if (gn(s, buf_[b], buf_[a], h * w, cout, pre + ".norm2", true)) return 1;
    const bf16_t* sc = x;
    if (cin != cout) {  // conv_shortcut 1x1
      const bf16_t* wsc = P(pre + ".conv_shortcut.weight");
      FLITE_REQUIRE(wsc, "vae: unbound " + pre + ".conv_shortcut");
      GemmParams g;
      g.A = x;
      g.lda = cin;
      g.W = wsc;
      g.ldw = cin;
      g.bias = P(pre + ".conv_shortcut.bias");
      g.out = buf_[c];
      g.ldo = cout;
      g.M = (int)(h * w);
      g.N = cout;
      g.K = cin;
      if (gemm_bf16(g, EPI_STORE_BF16, s)) return 1;
      sc = buf_[c];
    }
    // conv2 + residual -> buf_[b] (x + h) / 1
    if (conv3(s, buf_[a], cout, h, w, false, pre + ".conv2", cout, buf_[b], sc)) return 1;
    cur = b;
    return 0;
  }

  // diffusers Attention (heads 1, dim_head C, residual_connection, group_norm): in place on buf_[cur]
  int attention(hipStream_t s, const std::string& pre, int& cur, int C, long h, long w) {
    const long L = h * w;
    const long Lp = (L + 63) / 64 * 64;
    const int a = (cur + 1) % 4, qb = (cur + 2) % 4, kb = (cur + 3) % 4;
    bf16_t* x = buf_[cur];
    if (gn(s, x, buf_[a], L, C, pre + ".group_norm", false)) return 1;
    auto lin = [&](const std::string& n, const bf16_t* in, bf16_t* out, const bf16_t* resid) -> int {
      GemmParams g;
      g.A = in;
      g.lda = C;
      g.W = P(n + ".weight");
      FLITE_REQUIRE(g.W, "vae: unbound " + n);
      g.ldw = C;
      g.bias = P(n + ".bias");
      g.out = out;
      g.ldo = C;
      g.M = (int)L;
      g.N = C;
      g.K = C;
      g.resid = resid;
      return gemm_bf16(g, EPI_STORE_BF16, s);
    };
    bf16_t* v = buf_[4];
    if (lin(pre + ".to_q", buf_[a], buf_[qb], nullptr)) return 1;
    if (lin(pre + ".to_k", buf_[a], buf_[kb], nullptr)) return 1;
    if (lin(pre + ".to_v", buf_[a], v, nullptr)) return 1;
    {  // S = Q K^T
      GemmParams g;
      g.A = buf_[qb];
      g.lda = C;
      g.W = buf_[kb];
      g.ldw = C;
      g.out = S_;
      g.ldo = Lp;
      g.M = (int)L;
      g.N = (int)L;
      g.K = C;
      if (gemm_bf16(g, EPI_STORE_F32, s)) return 1;
    }
    // P [L, Lp] and V^T [C, Lp] with zero columns L..Lp-1: the P.V GEMM runs over k = Lp (a multiple of 64)
    if (softmax_rows(S_, P_, (int)L, (int)L, (int)Lp, 1.0f / sqrtf((float)C), s)) return 1;
    if (Lp != L) FLITE_HIP_CHECK(hipMemsetAsync(vt_, 0, (size_t)C * Lp * 2, s));
    if (transpose_bf16(v, vt_, (int)L, C, (int)Lp, s)) return 1;
    {  // O = P V
      GemmParams g;
      g.A = P_;
      g.lda = Lp;
      g.W = vt_;
      g.ldw = Lp;
      g.out = buf_[qb];
      g.ldo = C;
      g.M = (int)L;
      g.N = C;
      g.K = (int)Lp;
      if (gemm_bf16(g, EPI_STORE_BF16, s)) return 1;
    }
    // to_out[0] + residual (rescale_output_factor 1)
    if (lin(pre + ".to_out.0", buf_[qb], buf_[kb], x)) return 1;
    cur = kb;
    return 0;
  }

  std::map<std::string, Param> params_;
  std::map<std::string, std::pair<bf16_t*, int>> packed_;
  std::vector<void*> allocs_;
  int h_ = 0, w_ = 0;
  bf16_t* buf_[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  float* S_ = nullptr;
  bf16_t* P_ = nullptr;
  bf16_t* vt_ = nullptr;
  bool fp8_w_ = false;
  std::map<std::string, std::pair<uint8_t*, uint8_t*>> w8_;  // fp8 storage: e4m3 bytes, scales [cout][K/32]
  bf16_t* wscratch_ = nullptr;                                // the expanded weight of the running conv
  double* stats_ = nullptr;
  float* out32_ = nullptr;
  // tiled decode: latent size, tile geometry, tile origins, decoded fp32 tiles (row-major over the grid)
  int tH_ = 0, tW_ = 0, tl_ = 0, ts_ = 0, tstride_ = 0, tblend_ = 0;
  std::vector<int> ti_, tj_;
  std::vector<float*> tiles_;
};

}  // namespace flite

using namespace flite;

struct flite_vae {
  VaeEngine* eng;
};

extern "C" {

int flite_vae_create(const flite_vae_config* cfg, flite_vae** out) {
  FLITE_REQUIRE(cfg && out, "flite_vae_create: null argument");
  FLITE_REQUIRE(cfg->n_blocks == 4 && cfg->layers_per_block >= 1 && cfg->norm_groups == 32,
                "flite_vae_create: unsupported config");
  if (gemm_init()) return 1;
  flite_vae* v = new flite_vae;
  v->eng = new VaeEngine(*cfg);
  *out = v;
  return 0;
}

int flite_vae_destroy(flite_vae* v) {
  if (v) {
    delete v->eng;
    delete v;
  }
  return 0;
}

int flite_vae_bind(flite_vae* v, const char* name, const void* ptr, long numel) {
  FLITE_REQUIRE(v && name, "flite_vae_bind: null argument");
  return v->eng->bind(name, ptr, numel);
}

int flite_vae_enable_fp8_weights(flite_vae* v, int on) {
  FLITE_REQUIRE(v, "flite_vae_enable_fp8_weights: null engine");
  return v->eng->enable_fp8_weights(on != 0);
}

int flite_vae_weights_updated(flite_vae* v) {
  FLITE_REQUIRE(v, "flite_vae_weights_updated: null engine");
  return v->eng->weights_updated();
}

int flite_vae_prepare(flite_vae* v, int latent_h, int latent_w) {
  FLITE_REQUIRE(v, "flite_vae_prepare: null engine");
  return v->eng->prepare(latent_h, latent_w);
}

int flite_vae_prepare_tiled(flite_vae* v, int latent_h, int latent_w, int tile_latent, int tile_sample,
                            float overlap_factor) {
  FLITE_REQUIRE(v, "flite_vae_prepare_tiled: null engine");
  return v->eng->prepare_tiled(latent_h, latent_w, tile_latent, tile_sample, overlap_factor);
}

int flite_vae_decode_tiled_uint8(flite_vae* v, void* stream, const float* latents, int n_img, void* images,
                                 float scaling_factor, float shift_factor) {
  FLITE_REQUIRE(v && latents && images, "flite_vae_decode_tiled_uint8: null argument");
  const long lat_elems = v->eng->tiled_latent_elems();
  const long img_bytes = v->eng->tiled_image_bytes();
  FLITE_REQUIRE(lat_elems > 0, "flite_vae_decode_tiled_uint8: call flite_vae_prepare_tiled first");
  for (int i = 0; i < n_img; ++i) {  // one image at a time (enable_slicing), each tiled
    if (v->eng->decode_tiled((hipStream_t)stream, latents + i * lat_elems, (unsigned char*)images + i * img_bytes,
                             scaling_factor, shift_factor))
      return 1;
  }
  return 0;
}

int flite_vae_decode_uint8(flite_vae* v, void* stream, const float* latents, int n_img, void* images,
                           float scaling_factor, float shift_factor) {
  FLITE_REQUIRE(v && latents && images, "flite_vae_decode_uint8: null argument");
  // one image at a time (the reference's enable_vae_slicing semantics, generate.py:77)
  const long lat_elems = v->eng->latent_elems();
  const long img_bytes = v->eng->image_bytes();
  FLITE_REQUIRE(lat_elems > 0, "flite_vae_decode_uint8: call flite_vae_prepare first");
  for (int i = 0; i < n_img; ++i) {
    if (v->eng->decode((hipStream_t)stream, latents + i * lat_elems, (unsigned char*)images + i * img_bytes,
                       scaling_factor, shift_factor))
      return 1;
  }
  return 0;
}

}  // extern "C"
