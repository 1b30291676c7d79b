// libsse.so host side: the C-ABI of include/sse.h, weight repacking and the forward
// orchestration of the WavLM / Whisper embedding path on one gfx950 device.
//
// Forward plan (WavLM, SURVEY.md §3.1, HF/models/wavlm/modeling_wavlm.py):
//   [a2] wave_stats (do_normalize)                 -> per-clip (mean, rstd)
//   [K1] conv0 + GroupNorm + GELU                  -> bufA [B][T0][C]      (channels-last)
//   [K2] conv1..6 implicit GEMM + GELU             -> ping-pong bufB/bufA  (rows overlap, no im2col)
//   [K3] LN(C) -> projection GEMM                  -> x (fp32 residual stream) + xt (GEMM operand)
//   [K4] grouped pos-conv GEMM + GELU + residual   -> x ; LN (post-LN base) -> hidden_states[0]
//   per layer [K5-K7]: QKV GEMM -> gated-bias attention -> out-proj(+x) -> LN -> FFN(GELU)(+x) -> LN
//   [K8] pool_mean of the selected hidden states   -> out [B][n_sel][H]
// Whisper: [K9] log-mel -> [K10] conv1/conv2 implicit GEMM (+positions) ->
//   32 pre-LN layers (q pre-scaled by 1/8 at load, k unbiased) -> final LN -> [K12] pooling.
// All activations that feed a GEMM are stored in the path's element type (bf16 or fp32);
// the residual stream, LayerNorm statistics and pooled sums stay fp32.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <algorithm>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/sse.h"
#include "common.h"
#include "kernels.h"
#include "kernels_logmel.h"

#define SSE_VERSION "sse 0.1.0 (gfx950)"

// A/B switches (common.h OPT_*), set only through sse_set_option
static int g_opt[OPT_COUNT] = {0};
static const char* const g_opt_name[OPT_COUNT] = {"gemm_cfg", "gemm_nonpersist", "gelu_exact", "conv0_valu",
                                                   "posconv_gemm", "no_lnfold", "gemm_mx_staged", "no_split",
                                                   "logmel_v1", "ln_x3_v1", "attn_x3_f32", "ln_rows_v1", "posconv_2cl",
                                                   "attn_short", "attn_long", "fp8_attn_bf16", "split_cumask",
                                                   "gemm_4phase", "f8_oproj"};
// the largest value each switch takes (0 .. max; anything else is SSE_ERR_INVALID, not a silent default)
static const int g_opt_max[OPT_COUNT] = {3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 1, 2, 1, 1};
int sse_opt(int id) { return __atomic_load_n(&g_opt[id], __ATOMIC_RELAXED); }

// CU-masked streams (split_forward, OPT_SPLIT_CUMASK) and their CU counts; registered once, never removed
// while the owning model lives (sse_model_destroy unregisters them)
static std::mutex g_mask_mu;
static std::vector<std::pair<hipStream_t, int>> g_mask_streams;
int sse_stream_cus(hipStream_t s, int dev_cus) {
  if (!s) return dev_cus;
  std::lock_guard<std::mutex> lk(g_mask_mu);
  for (const auto& e : g_mask_streams)
    if (e.first == s) return e.second;
  return dev_cus;
}
static void register_mask_stream(hipStream_t s, int cus) {
  std::lock_guard<std::mutex> lk(g_mask_mu);
  g_mask_streams.emplace_back(s, cus);
}
static void unregister_mask_stream(hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_mask_mu);
  for (size_t i = 0; i < g_mask_streams.size(); ++i)
    if (g_mask_streams[i].first == s) {
      g_mask_streams.erase(g_mask_streams.begin() + i);
      return;
    }
}

namespace {

// relative-position table covers |key - query| <= MAXD; the attention kernels clamp d to +-MAXD, which
// is exact for any clip length because the bucket saturates at max_distance (HF
// _relative_positions_bucket: every |d| >= max_distance maps to the last bucket of its sign)
constexpr int MAXD = 4095;

inline float bf_bits2f(uint16_t h) {
  const uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

inline uint16_t f2bf_bits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// OCP e4m3 (e4m3fn) of |y| <= 448 with round-to-nearest-even: what v_cvt_pk_fp8_f32 produces
// (checked exhaustively against nearest-even search, tools/probe_mx.hip).  Bit-level on the fp32.
uint8_t f32_to_e4m3(float y) {
  uint32_t u;
  std::memcpy(&u, &y, 4);
  const uint8_t sign = (uint8_t)((u >> 24) & 0x80);
  u &= 0x7FFFFFFFu;
  if (u >= 0x43E00000u) return sign | 0x7E;                  // >= 448: saturate (never reached by mx)
  if (u < 0x3C800000u) {                                      // < 2^-6: subnormal m * 2^-9, m in [0, 8]
    float a;
    std::memcpy(&a, &u, 4);
    const float m = std::nearbyint(a * 512.0f);               // exact scaling, ties to even
    return sign | (uint8_t)m;                                 // m == 8 is the first normal (0x08)
  }
  uint32_t keep = u >> 20;                                    // float exponent | top 3 mantissa bits
  const uint32_t rem = u & 0xFFFFFu;
  if (rem > 0x80000u || (rem == 0x80000u && (keep & 1))) ++keep;   // carry rolls into the exponent
  const int e = (int)(keep >> 3) - 127 + 7;
  return sign | (uint8_t)((e << 3) | (keep & 7));
}

// MX quantisation of row-major x [R][K] (K % 128 == 0): e4m3 bytes + E8M0 scales (role 0: A layout,
// 1: B layout), the same arithmetic as mx_quant4 (kernels_misc.hip)
void mx_quantize_rows(const float* x, int R, int K, int role, uint8_t* q, uint8_t* scale) {
  for (int r = 0; r < R; ++r)
    for (int b = 0; b < K / 32; ++b) {
      const float* v = x + (size_t)r * K + b * 32;
      float amax = 0.f;
      for (int i = 0; i < 32; ++i) amax = std::fmax(amax, std::fabs(v[i]));
      const int e = mx_scale_exp(amax);
      const float inv = mx_inv_scale(e);
      for (int i = 0; i < 32; ++i) q[(size_t)r * K + b * 32 + i] = f32_to_e4m3(v[i] * inv);
      scale[role ? mx_b_scale_off(r, b, K / 128) : mx_a_scale_off(r, b, K / 128)] = (uint8_t)e;
    }
}

int rel_bucket(int d, int num_buckets, int max_distance) {
  // HF WavLMAttention._relative_positions_bucket (modeling_wavlm.py:246-271), float32 path
  const int nb = num_buckets / 2;
  int bucket = d > 0 ? nb : 0;
  const int rel = d < 0 ? -d : d;
  const int max_exact = nb / 2;
  if (rel < max_exact) return bucket + rel;
  float v = logf((float)rel / (float)max_exact);
  v = v / (float)std::log((double)max_distance / (double)max_exact);
  v = v * (float)(nb - max_exact);
  int large = (int)((float)max_exact + v);
  if (large > nb - 1) large = nb - 1;
  return bucket + large;
}

// ---- canonical weight blob walker (mirrors config.param_specs) -------------------------
struct Blob {
  const float* p;
  size_t n, off = 0;
  bool ok = true;
  const float* take(size_t count) {
    if (off + count > n) { ok = false; return nullptr; }
    const float* r = p ? p + off : nullptr;
    off += count;
    return r;
  }
};

// ---- device arena for weights ----------------------------------------------------------
struct Arena {
  std::vector<std::pair<size_t, std::vector<char>>> pending;  // (offset, bytes)
  size_t size = 0;
  size_t put(const void* src, size_t bytes) {
    const size_t off = size;
    std::vector<char> v(bytes);
    if (src) std::memcpy(v.data(), src, bytes);
    pending.emplace_back(off, std::move(v));
    size = (size + bytes + 255) & ~(size_t)255;
    return off;
  }
  size_t put_f32(const float* src, size_t n) { return put(src, n * 4); }
  // split-fp16 GEMM weight (SSE_DTYPE_FP16X3, common.h x3_split4): rows of nblk blocks of blk values
  // (a conv tap is a block), scaled by 2^e so that max |w| 2^e <= 2^14, -> per block
  // [hi | hi * 2^-11 | lo], hi = f16(w 2^e), lo = f16(w 2^e - hi): matched to activation rows
  // [hi | lo' | hi] the K-sum is 2^e (hi*hi + lo*hi + hi*lo); alpha[offset] = 2^-e undoes the scale in
  // the GEMM epilogue (powers of two: exact)
  std::map<size_t, float> alpha;
  size_t put_x3(const std::vector<float>& v, size_t rows, int nblk, int blk) {
    float amax = 0.f;
    for (float w : v) amax = std::fmax(amax, std::fabs(w));
    int e = 0;
    if (amax > 0.f && std::isfinite(amax)) e = std::min(60, std::max(-60, (int)std::floor(std::log2(16384.0 / amax))));
    const float sc = std::ldexp(1.f, e);
    std::vector<f16> h(v.size() * 3);
    for (size_t r = 0; r < rows; ++r)
      for (int j = 0; j < nblk; ++j)
        for (int c = 0; c < blk; ++c) {
          const float w = v[(r * nblk + j) * blk + c] * sc;
          const f16 hi = (f16)w;
          f16* o = h.data() + (r * nblk + j) * 3 * (size_t)blk;
          o[c] = hi;
          o[blk + c] = (f16)((float)hi * (1.f / X3_LO_SCALE));
          o[2 * blk + c] = (f16)(w - (float)hi);
        }
    const size_t off = put(h.data(), h.size() * 2);
    alpha[off] = std::ldexp(1.f, -e);
    return off;
  }
  // split-fp16 positional-conv weight (posconv_x3_kernel): two planes [wh][wl] of w 2^e, wh = f16(w 2^e),
  // wl = f16(w 2^e - wh), e as put_x3; alpha[offset] = 2^-e
  size_t put_pos_x3(const std::vector<float>& v) {
    float amax = 0.f;
    for (float w : v) amax = std::fmax(amax, std::fabs(w));
    int e = 0;
    if (amax > 0.f && std::isfinite(amax)) e = std::min(60, std::max(-60, (int)std::floor(std::log2(16384.0 / amax))));
    const float sc = std::ldexp(1.f, e);
    std::vector<f16> h(v.size() * 2);
    for (size_t i = 0; i < v.size(); ++i) {
      const float w = v[i] * sc;
      const f16 hi = (f16)w;
      h[i] = hi;
      h[v.size() + i] = (f16)(w - (float)hi);
    }
    const size_t off = put(h.data(), h.size() * 2);
    alpha[off] = std::ldexp(1.f, -e);
    return off;
  }
  // kind 0: fp32, 1: bf16, 2: fp16 (SSE_DTYPE_FP16)
  size_t put_elem(const std::vector<float>& v, int kind) {
    if (!kind) return put(v.data(), v.size() * 4);
    std::vector<uint16_t> h(v.size());
    if (kind == 2) {
      for (size_t i = 0; i < v.size(); ++i) h[i] = __builtin_bit_cast(uint16_t, (f16)v[i]);
    } else {
      for (size_t i = 0; i < v.size(); ++i) h[i] = f2bf_bits(v[i]);
    }
    return put(h.data(), h.size() * 2);
  }
  // MX-fp8 weight [N][K] (B layout): e4m3 bytes at the returned offset, scales at *scale_off
  size_t put_mx(const std::vector<float>& v, int N, int K, size_t* scale_off) {
    std::vector<uint8_t> q((size_t)N * K), sc((size_t)mx_scale_bytes(N, K), 0x7F);
    mx_quantize_rows(v.data(), N, K, 1, q.data(), sc.data());
    const size_t o = put(q.data(), q.size());
    *scale_off = put(sc.data(), sc.size());
    return o;
  }
};

// LayerNorm folded into the GEMM that consumes its output: B' = W diag(lw) (bf16, or fp16 when h16),
// acol[n] = sum_k B'[n][k] of the rounded values (the operand values the MFMAs multiply),
// bias'[n] = bias[n] + sum_k W[n][k] lb[k]
void put_folded(Arena& ar, const float* W, const float* bias, int N, int K, const float* lw, const float* lb,
                size_t* w_off, size_t* c_off, size_t* b_off, bool h16) {
  std::vector<uint16_t> wf((size_t)N * K);
  std::vector<float> cs(N), bf(N);
  for (int n = 0; n < N; ++n) {
    double c = 0.0, d = bias ? (double)bias[n] : 0.0;
    for (int k = 0; k < K; ++k) {
      const float w = W[(size_t)n * K + k];
      const float wl = w * lw[k];
      const f16 hh = (f16)wl;
      const uint16_t h = h16 ? __builtin_bit_cast(uint16_t, hh) : f2bf_bits(wl);
      wf[(size_t)n * K + k] = h;
      c += h16 ? (double)(float)hh : (double)bf_bits2f(h);
      d += (double)w * (double)lb[k];
    }
    cs[n] = (float)c;
    bf[n] = (float)d;
  }
  *w_off = ar.put(wf.data(), wf.size() * 2);
  *c_off = ar.put_f32(cs.data(), N);
  *b_off = ar.put_f32(bf.data(), N);
}

struct LayerW {
  size_t qkv_w, qkv_b, o_w, o_b, ln1_w, ln1_b, f1_w, f1_b, f2_w, f2_b, ln2_w, ln2_b;
  size_t g_const, g_w, g_b;   // WavLM gate
  size_t qkv_q, qkv_s, f1_q, f1_s, f2_q, f2_s;   // SSE_DTYPE_FP8: MX-fp8 copies (e4m3 + scales)
  size_t o_q, o_s;                                // SSE_DTYPE_FP8: the out-projection's MX-fp8 copy (round 6)
  // folded LayerNorm (bf16 post-LN, common.h GemmArgs.apart): QKV folded with the previous layer's
  // final LayerNorm (layers >= 1), FFN1 with this layer's attention LayerNorm: weight W diag(ln_w)
  // (bf16), its column sums acol and bias b + W ln_b
  size_t qkv_wf, qkv_c, qkv_bf, f1_wf, f1_c, f1_bf;
};

// Whisper decoder layer for the 1-token pass (HF/models/whisper/modeling_whisper.py:448-506)
struct DecLayerW {
  size_t ln1_w, ln1_b, v_w, v_b, o_w, o_b;           // self-attention: one key -> softmax == 1
  size_t ln2_w, ln2_b, q_w, q_b, kv_w, kv_b, co_w, co_b;   // cross-attention (q pre-scaled)
  size_t ln3_w, ln3_b, f1_w, f1_b, f2_w, f2_b;
};

}  // namespace

struct sse_model {
  sse_cfg cfg;
  int device = 0, dtype = 0;
  char* dmem = nullptr;
  size_t dbytes = 0;
  // WavLM
  size_t conv_w[8], conv_b[8], conv_ln_w[8], conv_ln_b[8];
  bool has_conv_b = false;
  size_t fp_ln_w, fp_ln_b, fp_w, fp_b, pos_w, pos_b, enc_ln_w, enc_ln_b, relb, zero;
  size_t pos_w3 = 0;        // fp16x3: positional-conv weight planes [wh][wl] (Arena::put_pos_x3)
  size_t status = 0;   // device int: raised when an fp16-range call wrote a non-finite value (sse_check_range)
  // Whisper
  size_t c1_w, c1_b, c2_w, c2_b, positions;
  size_t dec_x0, dec_ln_w, dec_ln_b;   // decoder: embed_tokens[0] + embed_positions[0]; final LN
  std::vector<DecLayerW> dec;
  bool ln_fold = false;   // folded-LayerNorm weights present (bf16 post-LN WavLM, LayerW.qkv_wf / f1_wf)
  bool pre_fold = false;  // bf16 stable-LN WavLM (large): each layer's attention LayerNorm folded into its QKV (l > 0)
  int ldq = 0;   // QKV GEMM width: 3H (+ 8*heads gate columns for WavLM, then zero pad to 256 so the
                // 256x256 MFMA tile applies)
  std::vector<LayerW> layers;
  // live per-launch timing (sse_profile_*): events pre-created outside any capture
  struct Prof {
    bool on = false;
    int used = 0;
    std::vector<hipEvent_t> ev;
    std::vector<std::string> tag;
    std::vector<double> flops, bytes;
  } prof;

  // two-stream half-batch split of WavLM embedding calls (split_forward): the second half runs on
  // aux, forked from / joined to the caller's stream by events (created on first use, on the model's
  // device); the mutex serialises the host-side fork / join of concurrent callers
  static constexpr int MAX_PARTS = 4;
  hipStream_t aux[MAX_PARTS - 1] = {};
  hipEvent_t ev_fork = nullptr, ev_join[MAX_PARTS - 1] = {};
  // OPT_SPLIT_CUMASK: both halves on CU-masked streams (mask kind 1 / 2), joined back to the caller's stream
  hipStream_t mstream[2] = {};
  hipEvent_t mjoin[2] = {};
  int mkind = 0;
  std::mutex split_mu;

  template <typename X = void> const X* ptr(size_t off) const { return (const X*)(dmem + off); }
  bool bf() const { return dtype == SSE_DTYPE_BF16 || dtype == SSE_DTYPE_FP8; }   // bf16 activations
  bool h16() const { return dtype == SSE_DTYPE_FP16; }   // fp16 activations and GEMM operands (WavLM)
  bool half() const { return bf() || h16(); }          // 16-bit activations
  int ekind() const { return h16() ? 2 : (bf() ? 1 : 0); }   // Arena::put_elem kind of GEMM weights
  bool x3() const { return dtype == SSE_DTYPE_FP16X3; }   // split-fp16 GEMMs, fp32 activations
  std::map<size_t, float> x3_alpha;   // split-fp16 weight offset -> epilogue scale (Arena::put_x3)
  float alpha(size_t off) const {
    const auto it = x3_alpha.find(off);
    return it == x3_alpha.end() ? 0.f : it->second;   // 0: the GEMM launcher rejects the call
  }
  bool mx() const { return dtype == SSE_DTYPE_FP8; }   // MX-fp8 encoder-layer GEMMs (Whisper)
};

namespace {

bool cfg_valid(const sse_cfg* c) {
  if (!c || c->hidden <= 0 || c->layers <= 0 || c->heads <= 0 || c->ffn <= 0) return false;
  if (c->hidden % c->heads || c->hidden / c->heads != 64) return false;
  if (c->kind == SSE_KIND_WAVLM) {
    if (c->n_conv < 2 || c->n_conv > 8 || c->pos_groups <= 0 || c->hidden % c->pos_groups) return false;
    if (c->max_distance > MAXD) return false;   // the clamp to +-MAXD must lie in the saturated range
  } else if (c->kind == SSE_KIND_WHISPER) {
    if (c->n_mels <= 0 || c->max_positions <= 0) return false;
    if (c->decoder_layers < 0 || (c->decoder_layers > 0 && c->dec_ffn <= 0)) return false;
  } else {
    return false;
  }
  return true;
}

// Walk the canonical order; with a null blob only counts.
int build_wavlm(sse_model* m, Blob& bl, Arena& ar) {
  const sse_cfg& c = m->cfg;
  const int BF = m->ekind();   // weight element kind (fp32 / bf16 / fp16)
  const int H = c.hidden, F = c.ffn, nh = c.heads;
  int cin = 1;
  for (int i = 0; i < c.n_conv; ++i) {
    const int co = c.conv_dim[i], k = c.conv_kernel[i];
    const float* w = bl.take((size_t)co * cin * k);
    const float* b = c.conv_bias ? bl.take(co) : nullptr;
    const float* lw = nullptr;
    const float* lb = nullptr;
    if (c.feat_norm_layer || i == 0) { lw = bl.take(co); lb = bl.take(co); }
    if (!bl.ok) return SSE_ERR_WEIGHTS;
    if (!w) { cin = co; continue; }
    if (i == 0) {
      m->conv_w[0] = ar.put_f32(w, (size_t)co * k);      // [C][k] fp32 (VALU conv0)
    } else {
      std::vector<float> t((size_t)co * k * cin);        // [out][j*cin + c]
      for (int o = 0; o < co; ++o)
        for (int ci = 0; ci < cin; ++ci)
          for (int j = 0; j < k; ++j) t[((size_t)o * k + j) * cin + ci] = w[((size_t)o * cin + ci) * k + j];
      m->conv_w[i] = m->x3() ? ar.put_x3(t, co, k, cin) : ar.put_elem(t, BF);
    }
    m->conv_b[i] = b ? ar.put_f32(b, co) : 0;
    m->has_conv_b = b != nullptr;
    m->conv_ln_w[i] = lw ? ar.put_f32(lw, co) : 0;
    m->conv_ln_b[i] = lb ? ar.put_f32(lb, co) : 0;
    cin = co;
  }
  const int C = cin;
  const float* fplw = bl.take(C);
  const float* fplb = bl.take(C);
  const float* fpw = bl.take((size_t)H * C);
  const float* fpb = bl.take(H);
  const int K = c.pos_kernel, G = c.pos_groups, cg = H / G;
  const float* pg = bl.take(K);
  const float* pv = bl.take((size_t)H * cg * K);
  const float* pb = bl.take(H);
  const float* elw = bl.take(H);
  const float* elb = bl.take(H);
  const float* rel = bl.take((size_t)c.num_buckets * nh);
  if (!bl.ok) return SSE_ERR_WEIGHTS;
  if (fplw) {
    m->fp_ln_w = ar.put_f32(fplw, C);
    m->fp_ln_b = ar.put_f32(fplb, C);
    m->fp_w = m->x3() ? ar.put_x3(std::vector<float>(fpw, fpw + (size_t)H * C), H, 1, C)
                      : ar.put_elem(std::vector<float>(fpw, fpw + (size_t)H * C), BF);
    m->fp_b = ar.put_f32(fpb, H);
    // weight_norm(dim=2): w[o][c][j] = g[j] * v[o][c][j] / ||v[:, :, j]||  (fp64 norm), then
    // per group [cg_out][j*cg + c_in]
    std::vector<double> nrm(K, 0.0);
    for (size_t i = 0; i < (size_t)H * cg; ++i)
      for (int j = 0; j < K; ++j) nrm[j] += (double)pv[i * K + j] * pv[i * K + j];
    for (int j = 0; j < K; ++j) nrm[j] = std::sqrt(nrm[j]);
    std::vector<float> t((size_t)H * K * cg);
    for (int o = 0; o < H; ++o)
      for (int ci = 0; ci < cg; ++ci)
        for (int j = 0; j < K; ++j)
          t[((size_t)o * K + j) * cg + ci] = (float)((double)pg[j] * ((double)pv[((size_t)o * cg + ci) * K + j] / nrm[j]));
    m->pos_w = ar.put_elem(t, BF);
    if (m->x3()) m->pos_w3 = ar.put_pos_x3(t);
    m->pos_b = ar.put_f32(pb, H);
    m->enc_ln_w = ar.put_f32(elw, H);
    m->enc_ln_b = ar.put_f32(elb, H);
    std::vector<float> tab((size_t)nh * (2 * MAXD + 1));
    for (int d = -MAXD; d <= MAXD; ++d) {
      const int bk = rel_bucket(d, c.num_buckets, c.max_distance);
      for (int h = 0; h < nh; ++h) tab[(size_t)h * (2 * MAXD + 1) + d + MAXD] = rel[(size_t)bk * nh + h];
    }
    m->relb = ar.put_f32(tab.data(), tab.size());
  }
  const bool fold = m->half() && !c.stable_layer_norm && H == 768;   // the GEMM epilogues combine 3 column-tile partials
  // stable-LN (pre-LN, WavLM-large) in bf16: the QKV of layers l > 0 reads the bf16 residual stream itself with
  // W' = W diag(ln1_w), the previous layer's ffn2 writing the rows' per-256-column partials (round 6); the GEMM
  // epilogue's fold takes 3-5 partials per row on the plain bf16 kernel (H = 768..1280).  fc1 keeps its LayerNorm
  // kernel (its GELU epilogue with 4-5 partials spills, as for Whisper-large-v2)
  const bool prefold = m->dtype == SSE_DTYPE_BF16 && c.stable_layer_norm && H % 256 == 0 && H >= 768 && H <= 1280;
  const float *prev_l2w = nullptr, *prev_l2b = nullptr;
  for (int l = 0; l < c.layers; ++l) {
    const float *qw = bl.take((size_t)H * H), *qb = bl.take(H), *kw = bl.take((size_t)H * H), *kb = bl.take(H);
    const float *vw = bl.take((size_t)H * H), *vb = bl.take(H), *ow = bl.take((size_t)H * H), *ob = bl.take(H);
    const float *gc = bl.take(nh), *gw = bl.take((size_t)8 * 64), *gbb = bl.take(8);
    const float *l1w = bl.take(H), *l1b = bl.take(H);
    const float *f1w = bl.take((size_t)F * H), *f1b = bl.take(F), *f2w = bl.take((size_t)H * F), *f2b = bl.take(H);
    const float *l2w = bl.take(H), *l2b = bl.take(H);
    if (!bl.ok) return SSE_ERR_WEIGHTS;
    if (!qw) continue;
    LayerW L{};
    // rows [q | k | v | gate: head h, output o at 3H + 8h + o, block-diagonal over the
    // head's 64 input channels (gru_rel_pos_linear, HF :158-163) | zero pad to ldq]
    const int ldq = ((3 * H + 8 * nh + 255) / 256) * 256;
    m->ldq = ldq;
    std::vector<float> qkv((size_t)ldq * H, 0.f), qkvb((size_t)ldq, 0.f);
    std::memcpy(qkv.data(), qw, (size_t)H * H * 4);
    std::memcpy(qkv.data() + (size_t)H * H, kw, (size_t)H * H * 4);
    std::memcpy(qkv.data() + (size_t)2 * H * H, vw, (size_t)H * H * 4);
    std::memcpy(qkvb.data(), qb, H * 4);
    std::memcpy(qkvb.data() + H, kb, H * 4);
    std::memcpy(qkvb.data() + 2 * H, vb, H * 4);
    for (int hh = 0; hh < nh; ++hh)
      for (int o = 0; o < 8; ++o) {
        const size_t row = (size_t)3 * H + 8 * hh + o;
        for (int d = 0; d < 64; ++d) qkv[row * H + hh * 64 + d] = gw[o * 64 + d];
        qkvb[row] = gbb[o];
      }
    const bool X3 = m->x3();
    L.qkv_w = X3 ? ar.put_x3(qkv, ldq, 1, H) : ar.put_elem(qkv, BF);
    L.qkv_b = ar.put_f32(qkvb.data(), ldq);
    L.o_w = X3 ? ar.put_x3(std::vector<float>(ow, ow + (size_t)H * H), H, 1, H)
               : ar.put_elem(std::vector<float>(ow, ow + (size_t)H * H), BF);
    L.o_b = ar.put_f32(ob, H);
    L.g_const = ar.put_f32(gc, nh);
    L.g_w = ar.put_f32(gw, 8 * 64);
    L.g_b = ar.put_f32(gbb, 8);
    L.ln1_w = ar.put_f32(l1w, H);
    L.ln1_b = ar.put_f32(l1b, H);
    L.f1_w = X3 ? ar.put_x3(std::vector<float>(f1w, f1w + (size_t)F * H), F, 1, H)
                : ar.put_elem(std::vector<float>(f1w, f1w + (size_t)F * H), BF);
    L.f1_b = ar.put_f32(f1b, F);
    L.f2_w = X3 ? ar.put_x3(std::vector<float>(f2w, f2w + (size_t)H * F), H, 1, F)
                : ar.put_elem(std::vector<float>(f2w, f2w + (size_t)H * F), BF);
    L.f2_b = ar.put_f32(f2b, H);
    L.ln2_w = ar.put_f32(l2w, H);
    L.ln2_b = ar.put_f32(l2b, H);
    if (fold) {
      if (l > 0)
        put_folded(ar, qkv.data(), qkvb.data(), ldq, H, prev_l2w, prev_l2b, &L.qkv_wf, &L.qkv_c, &L.qkv_bf, m->h16());
      put_folded(ar, f1w, f1b, F, H, l1w, l1b, &L.f1_wf, &L.f1_c, &L.f1_bf, m->h16());
    }
    if (prefold && l > 0) put_folded(ar, qkv.data(), qkvb.data(), ldq, H, l1w, l1b, &L.qkv_wf, &L.qkv_c, &L.qkv_bf, false);
    prev_l2w = l2w;
    prev_l2b = l2b;
    m->layers.push_back(L);
  }
  m->ln_fold = fold;
  m->pre_fold = prefold;
  return bl.ok ? SSE_OK : SSE_ERR_WEIGHTS;
}

int build_whisper(sse_model* m, Blob& bl, Arena& ar) {
  const sse_cfg& c = m->cfg;
  const bool BF = m->bf();
  const int D = c.hidden, F = c.ffn, nm = c.n_mels;
  const float *c1w = bl.take((size_t)D * nm * 3), *c1b = bl.take(D);
  const float *c2w = bl.take((size_t)D * D * 3), *c2b = bl.take(D);
  const float* pos = bl.take((size_t)c.max_positions * D);
  if (!bl.ok) return SSE_ERR_WEIGHTS;
  auto conv_pack = [&](const float* w, int co, int ci) {   // [out][in][3] -> [out][j*in + c]
    std::vector<float> t((size_t)co * 3 * ci);
    for (int o = 0; o < co; ++o)
      for (int x = 0; x < ci; ++x)
        for (int j = 0; j < 3; ++j) t[((size_t)o * 3 + j) * ci + x] = w[((size_t)o * ci + x) * 3 + j];
    return t;
  };
  if (c1w) {
    m->c1_w = ar.put_elem(conv_pack(c1w, D, nm), BF);
    m->c1_b = ar.put_f32(c1b, D);
    m->c2_w = ar.put_elem(conv_pack(c2w, D, D), BF);
    m->c2_b = ar.put_f32(c2b, D);
    m->positions = ar.put_f32(pos, (size_t)c.max_positions * D);
  }
  const float scale = 0.125f;   // head_dim ** -0.5 for head_dim 64: exact power of two
  // bf16 / fp8 encoder: q also carries log2(e) (still one rounding of sWq to the operand type), so the
  // flash kernel's scores are log2-domain logits (AttnArgs::q_log2, scale ln 2 for any other consumer)
  const float qscale = m->bf() ? scale * 1.4426950408889634f : scale;
  // bf16 encoder at D = 768 (whisper-small) and 1280 (whisper-large: the folded-LN GEMM epilogue takes 3 / 5
  // 256-column partials per row; D = 1024 has no fixture, so it keeps the LayerNorm kernel): each pre-LN
  // folded into the GEMM that consumes it, as WavLM-base's post-LN (GemmArgs.apart).  The choice is made
  // here, at load (option no_lnfold read at sse_model_create): a folded model stores the plain QKV weights
  // for layer 0 only (its input has no partials) -- 305 MB less for large-v2 than keeping both forms.
  const bool wfold = m->dtype == SSE_DTYPE_BF16 && (D == 768 || D == 1280) && !sse_opt(OPT_NO_LNFOLD);
  for (int l = 0; l < c.layers; ++l) {
    const float *qw = bl.take((size_t)D * D), *qb = bl.take(D), *kw = bl.take((size_t)D * D);
    const float *vw = bl.take((size_t)D * D), *vb = bl.take(D), *ow = bl.take((size_t)D * D), *ob = bl.take(D);
    const float *l1w = bl.take(D), *l1b = bl.take(D);
    const float *f1w = bl.take((size_t)F * D), *f1b = bl.take(F), *f2w = bl.take((size_t)D * F), *f2b = bl.take(D);
    const float *l2w = bl.take(D), *l2b = bl.take(D);
    if (!bl.ok) return SSE_ERR_WEIGHTS;
    if (!qw) continue;
    LayerW L{};
    std::vector<float> qkv((size_t)3 * D * D), qkvb((size_t)3 * D, 0.f);
    for (size_t i = 0; i < (size_t)D * D; ++i) qkv[i] = qw[i] * qscale;   // (xWq + bq) * s == x(sWq) + s bq
    std::memcpy(qkv.data() + (size_t)D * D, kw, (size_t)D * D * 4);
    std::memcpy(qkv.data() + (size_t)2 * D * D, vw, (size_t)D * D * 4);
    for (int i = 0; i < D; ++i) qkvb[i] = qb[i] * qscale;
    std::memcpy(qkvb.data() + 2 * D, vb, D * 4);                           // k_proj has no bias
    const bool X3 = m->x3();   // split-fp16 encoder GEMMs (Arena::put_x3), the decoder and convs fp32
    if (!wfold || l == 0) L.qkv_w = X3 ? ar.put_x3(qkv, 3 * D, 1, D) : ar.put_elem(qkv, BF);
    L.qkv_b = ar.put_f32(qkvb.data(), 3 * D);
    m->ldq = 3 * D;
    if (wfold) {   // pre-LN folded into QKV (self_attn_layer_norm) and fc1 (final_layer_norm)
      put_folded(ar, qkv.data(), qkvb.data(), 3 * D, D, l1w, l1b, &L.qkv_wf, &L.qkv_c, &L.qkv_bf, false);
      if (D == 768) put_folded(ar, f1w, f1b, F, D, l2w, l2b, &L.f1_wf, &L.f1_c, &L.f1_bf, false);   // see f1fold
    }
    if (m->mx()) {
      L.qkv_q = ar.put_mx(qkv, 3 * D, D, &L.qkv_s);
      L.f1_q = ar.put_mx(std::vector<float>(f1w, f1w + (size_t)F * D), F, D, &L.f1_s);
      L.f2_q = ar.put_mx(std::vector<float>(f2w, f2w + (size_t)D * F), D, F, &L.f2_s);
      L.o_q = ar.put_mx(std::vector<float>(ow, ow + (size_t)D * D), D, D, &L.o_s);
    }
    L.o_w = X3 ? ar.put_x3(std::vector<float>(ow, ow + (size_t)D * D), D, 1, D)
               : ar.put_elem(std::vector<float>(ow, ow + (size_t)D * D), BF);
    L.o_b = ar.put_f32(ob, D);
    L.ln1_w = ar.put_f32(l1w, D);
    L.ln1_b = ar.put_f32(l1b, D);
    L.f1_w = X3 ? ar.put_x3(std::vector<float>(f1w, f1w + (size_t)F * D), F, 1, D)
                : ar.put_elem(std::vector<float>(f1w, f1w + (size_t)F * D), BF);
    L.f1_b = ar.put_f32(f1b, F);
    L.f2_w = X3 ? ar.put_x3(std::vector<float>(f2w, f2w + (size_t)D * F), D, 1, F)
                : ar.put_elem(std::vector<float>(f2w, f2w + (size_t)D * F), BF);
    L.f2_b = ar.put_f32(f2b, D);
    L.ln2_w = ar.put_f32(l2w, D);
    L.ln2_b = ar.put_f32(l2b, D);
    m->layers.push_back(L);
  }
  m->ln_fold = wfold;
  const float *elw = bl.take(D), *elb = bl.take(D);
  if (!bl.ok) return SSE_ERR_WEIGHTS;
  if (elw) {
    m->enc_ln_w = ar.put_f32(elw, D);
    m->enc_ln_b = ar.put_f32(elb, D);
  }
  if (c.decoder_layers <= 0) return SSE_OK;
  // ---- decoder (config.param_specs order) ----
  const int Fd = c.dec_ffn;
  const float *e0 = bl.take(D), *p0 = bl.take(D);
  if (!bl.ok) return SSE_ERR_WEIGHTS;
  if (e0) {
    std::vector<float> x0(D);
    for (int i = 0; i < D; ++i) x0[i] = e0[i] + p0[i];   // inputs_embeds + positions (fp32 add, as torch)
    m->dec_x0 = ar.put_f32(x0.data(), D);
  }
  auto mat = [&](const float* w, size_t n, float sc) {
    std::vector<float> v(w, w + n);
    if (sc != 1.f) for (auto& e : v) e *= sc;
    return v;
  };
  for (int l = 0; l < c.decoder_layers; ++l) {
    const float *l1w = bl.take(D), *l1b = bl.take(D);
    const float *vw = bl.take((size_t)D * D), *vb = bl.take(D), *ow = bl.take((size_t)D * D), *ob = bl.take(D);
    const float *l2w = bl.take(D), *l2b = bl.take(D);
    const float *qw = bl.take((size_t)D * D), *qb = bl.take(D), *kw = bl.take((size_t)D * D);
    const float *cvw = bl.take((size_t)D * D), *cvb = bl.take(D), *cow = bl.take((size_t)D * D), *cob = bl.take(D);
    const float *l3w = bl.take(D), *l3b = bl.take(D);
    const float *f1w = bl.take((size_t)Fd * D), *f1b = bl.take(Fd), *f2w = bl.take((size_t)D * Fd), *f2b = bl.take(D);
    if (!bl.ok) return SSE_ERR_WEIGHTS;
    if (!l1w) continue;
    DecLayerW W{};
    W.ln1_w = ar.put_f32(l1w, D); W.ln1_b = ar.put_f32(l1b, D);
    W.v_w = ar.put_elem(mat(vw, (size_t)D * D, 1.f), BF); W.v_b = ar.put_f32(vb, D);
    W.o_w = ar.put_elem(mat(ow, (size_t)D * D, 1.f), BF); W.o_b = ar.put_f32(ob, D);
    W.ln2_w = ar.put_f32(l2w, D); W.ln2_b = ar.put_f32(l2b, D);
    W.q_w = ar.put_elem(mat(qw, (size_t)D * D, scale), BF);
    std::vector<float> qbs(qb, qb + D);
    for (auto& e : qbs) e *= scale;
    W.q_b = ar.put_f32(qbs.data(), D);
    std::vector<float> kv((size_t)2 * D * D), kvb((size_t)2 * D, 0.f);   // [K rows | V rows]; k_proj has no bias
    std::memcpy(kv.data(), kw, (size_t)D * D * 4);
    std::memcpy(kv.data() + (size_t)D * D, cvw, (size_t)D * D * 4);
    std::memcpy(kvb.data() + D, cvb, D * 4);
    W.kv_w = ar.put_elem(kv, BF); W.kv_b = ar.put_f32(kvb.data(), 2 * D);
    W.co_w = ar.put_elem(mat(cow, (size_t)D * D, 1.f), BF); W.co_b = ar.put_f32(cob, D);
    W.ln3_w = ar.put_f32(l3w, D); W.ln3_b = ar.put_f32(l3b, D);
    W.f1_w = ar.put_elem(mat(f1w, (size_t)Fd * D, 1.f), BF); W.f1_b = ar.put_f32(f1b, Fd);
    W.f2_w = ar.put_elem(mat(f2w, (size_t)D * Fd, 1.f), BF); W.f2_b = ar.put_f32(f2b, D);
    m->dec.push_back(W);
  }
  const float *dlw = bl.take(D), *dlb = bl.take(D);
  if (!bl.ok) return SSE_ERR_WEIGHTS;
  if (dlw) {
    m->dec_ln_w = ar.put_f32(dlw, D);
    m->dec_ln_b = ar.put_f32(dlb, D);
  }
  return SSE_OK;
}

// ---- workspace planning ----------------------------------------------------------------
struct Plan {
  size_t total = 0;
  size_t add(size_t bytes) {
    const size_t o = total;
    total = (total + bytes + 255) & ~(size_t)255;
    return o;
  }
};

// Runs `launch` between two recorded events when profiling is on (tag, algorithmic FLOPs and
// bytes of that launch are kept for sse_profile_read).
template <typename F>
int prof(sse_model* m, hipStream_t s, const char* tag, double flops, double bytes, F&& launch) {
  auto& P = m->prof;
  const bool rec = P.on && P.used + 2 <= (int)P.ev.size();
  if (rec && hipEventRecord(P.ev[P.used], s) != hipSuccess) return SSE_ERR_HIP;
  const int rc = launch();
  if (rc) return rc;
  if (rec) {
    if (hipEventRecord(P.ev[P.used + 1], s) != hipSuccess) return SSE_ERR_HIP;
    P.used += 2;
    P.tag.emplace_back(tag);
    P.flops.push_back(flops);
    P.bytes.push_back(bytes);
  }
  return 0;
}

inline double gflops(const GemmArgs& g, int groups = 1) { return 2.0 * g.M * (double)g.N * g.K * groups; }

// Algorithmic HBM bytes of one GEMM launch: every operand element read once, every output written
// once.  A counts unique elements: strided-conv SEG rows overlap (a segment spans seg_stride),
// CONV-mode rows read a [T_in][ld_in] segment per clip.
template <typename T>
double gbytes(const GemmArgs& g, int amode = AMODE_SEG, int groups = 1) {
  const double e = sizeof(T);
  const double segs = g.rows_per_seg > 0 ? (double)((g.M + g.rows_per_seg - 1) / g.rows_per_seg) : 1.0;
  double a;
  if (amode == AMODE_CONV) a = segs * g.T_in * (double)g.ld_in * e;
  else if (g.lda != g.K) a = segs * (double)g.seg_stride * e;
  else a = (double)g.M * g.K * e;
  const double mn = (double)g.M * g.N * groups;
  const double b = (double)g.N * g.K * groups * e;
  const double c = mn * ((g.Cf ? 4.0 : 0.0) + (g.Ct ? e : 0.0));
  const double r = g.resid ? (g.resid_rows ? (double)g.resid_rows * g.N * groups * 4.0 : mn * 4.0)
                           : (g.resid_t ? mn * 2.0 : 0.0);
  return a + b + c + r;
}

int wavlm_frames(const sse_cfg& c, int L, int* Ts) {
  int t = L;
  for (int i = 0; i < c.n_conv; ++i) {
    if (t < c.conv_kernel[i]) return 0;       // shorter than the receptive field
    t = (t - c.conv_kernel[i]) / c.conv_stride[i] + 1;
    if (Ts) Ts[i] = t;
    if (t <= 0) return 0;
  }
  return t;
}

struct WavlmWs {
  size_t zero, norm, part, ss, bufA, bufB, x, xt, xb, qkv, ctx, ff, hf, p1, p2, fr;
};

WavlmWs wavlm_plan(const sse_model* m, int B, int L, Plan& p) {
  const sse_cfg& c = m->cfg;
  const size_t es = m->half() ? 2 : 4;
  int Ts[8];
  const int T = wavlm_frames(c, L, Ts);
  const size_t M = (size_t)B * T;
  const int C0 = c.conv_dim[0];
  size_t maxA = 0, maxB = 0;
  for (int i = 0; i < c.n_conv; ++i) {
    const size_t sz = (size_t)B * Ts[i] * c.conv_dim[i] * es;
    if (i % 2 == 0) maxA = sz > maxA ? sz : maxA; else maxB = sz > maxB ? sz : maxB;
  }
  WavlmWs w;
  w.zero = p.add(256);
  w.norm = p.add((size_t)B * 8);
  w.part = p.add(conv0_moments_bytes(B));
  w.ss = p.add((size_t)B * C0 * 8);
  w.bufA = p.add(maxA);
  w.bufB = p.add(maxB);
  const int H = c.hidden;
  w.x = p.add(M * H * 4);
  w.xt = p.add(M * H * es);
  w.xb = p.add(M * (H > c.conv_dim[c.n_conv - 1] ? H : c.conv_dim[c.n_conv - 1]) * es);
  w.qkv = p.add(M * (size_t)(((3 * H + 8 * c.heads + 255) / 256) * 256) * es);
  w.ctx = p.add(M * H * es);
  w.ff = p.add(M * (size_t)c.ffn * es);
  w.hf = c.stable_layer_norm ? p.add(M * H * 4) : 0;
  const size_t nt = H % 256 == 0 ? (size_t)H / 256 : 0;   // folded path: per-256-column partials
  w.p1 = p.add(M * nt * 8);
  w.p2 = p.add(M * nt * 8);
  w.fr = p.add((size_t)B * 8);   // ragged batches: per-clip conv0 frames | final frames
  return w;
}

struct WhisperWs {
  size_t zero, lm, mel, h1, x, xb, qkv, ctx, ff, xf;
  size_t vam;      // fp8 attention: per-(clip, column) max |V| (float bits), [B][D]
  size_t p1, p2;   // folded pre-LN: per-256-column (mean, M2) partials of the residual stream's rows
  size_t dx, dxb, dv, dq, dctx, dff, dxf;   // decoder rows [B][*]
};

WhisperWs whisper_plan(const sse_model* m, int B, Plan& p) {
  const sse_cfg& c = m->cfg;
  const size_t es = m->bf() ? 2 : 4;
  const int D = c.hidden, T = c.max_positions, T2 = 2 * T;
  const size_t M = (size_t)B * T;
  WhisperWs w;
  w.zero = p.add(256);
  w.lm = p.add(logmel_workspace_bytes(B, c.n_mels));
  w.mel = p.add((size_t)B * T2 * c.n_mels * es);
  w.h1 = p.add((size_t)B * T2 * D * es);
  const size_t ex = m->x3() ? 6 : es;   // GEMM operands: tripled f16 rows [hi | lo' | hi] on the fp16x3 path
  w.x = p.add(M * D * es);   // residual stream: bf16 on the bf16 / MX-fp8 paths, fp32 on the fp32 path
  w.xb = p.add(M * D * ex);
  w.qkv = p.add(M * 3 * D * es);
  w.ctx = p.add(M * D * ex);
  w.ff = p.add(M * (size_t)c.ffn * ex);
  w.xf = p.add(M * D * 4);
  w.vam = m->mx() ? p.add((size_t)B * D * 4) : 0;
  w.p1 = w.p2 = 0;
  if (m->ln_fold) {
    w.p1 = p.add(M * (D / 256) * 8);
    w.p2 = p.add(M * (D / 256) * 8);
  }
  if (c.decoder_layers > 0) {
    w.dx = p.add((size_t)B * D * 4);
    w.dxb = p.add((size_t)B * D * es);
    w.dv = p.add((size_t)B * D * es);
    w.dq = p.add((size_t)B * D * es);
    w.dctx = p.add((size_t)B * D * es);
    w.dff = p.add((size_t)B * c.dec_ffn * es);
    w.dxf = p.add((size_t)B * D * 4);
  }
  return w;
}

#define RC(expr)                \
  do {                          \
    const int _rc = (expr);     \
    if (_rc) return _rc;        \
  } while (0)

// Emits one hidden state: pooled into its output slots and/or copied into d_hs.
struct Sink {
  const int32_t* ids;
  int n_ids;
  float* pooled;         // [B][n_ids][H]
  float* hs;             // [n_hs][B][T][H]
  int B, T, H;
  hipStream_t s;
  const int* tlen = nullptr;   // ragged batch: frames of each clip (the time-means run over those)
  template <typename TI>
  int emit(int idx, const TI* x) const {   // fp32 or the bf16 residual stream
    for (int i = 0; i < n_ids; ++i)
      if (ids[i] == idx)
        RC(launch_pool_mean<TI>(x, B, T, H, pooled + (size_t)i * H, (long long)n_ids * H, s, nullptr, nullptr, nullptr,
                                nullptr, 0, 0.f, tlen));
    if (hs) {
      if constexpr (sizeof(TI) == 4) {
        const size_t bytes = (size_t)B * T * H * 4;
        if (hipMemcpyAsync(hs + (size_t)idx * B * T * H, x, bytes, hipMemcpyDeviceToDevice, s) != hipSuccess)
          return SSE_ERR_HIP;
      } else {
        RC((launch_cast<float, TI>(x, (long long)B * T * H, hs + (size_t)idx * B * T * H, s)));
      }
    }
    return 0;
  }
  // hidden state = LayerNorm(x) with per-row stats st, or per-256-column partials part [rows][nt],
  // already computed (x itself un-normalised)
  template <typename TI>
  int emit_ln(int idx, const TI* x, const float2* st, const float* w, const float* b, float eps,
              const float2* part = nullptr, int nt = 0) const {
    for (int i = 0; i < n_ids; ++i)
      if (ids[i] == idx)
        RC(launch_pool_mean<TI>(x, B, T, H, pooled + (size_t)i * H, (long long)n_ids * H, s, st, w, b, part, nt, eps,
                                tlen));
    if (hs)
      RC((launch_layernorm<TI, float>(x, w, b, B * T, H, eps, ACT_NONE, hs + (size_t)idx * B * T * H,
                                      (float*)nullptr, s)));
    return 0;
  }
};

// GELU of a GEMM epilogue whose output is rounded to the element type: the bf16 path uses the
// cheaper gelu_fast2 (clamped polynomial, error 7e-5 abs: 50x below the bf16 half-ulp, common.h); fp32 keeps
// the exact erf form.
template <typename T>
int gelu_rounded_act() {
  if constexpr (sizeof(T) == 2) {
    return gelu_exact_env() ? ACT_GELU : ACT_GELU_FAST;
  } else {
    return ACT_GELU;
  }
}

// Ragged batches (lens: samples of each clip, device): the per-clip conv0 frame counts t0 and
// final frame counts tf go to the workspace; the sink's means run over tf.
int ragged_frames(const sse_model* m, const int* lens, int B, int L, int* t0, int* tf, hipStream_t s) {
  ClipFrames cf{};
  cf.n_conv = m->cfg.n_conv;
  for (int i = 0; i < cf.n_conv; ++i) { cf.kernel[i] = m->cfg.conv_kernel[i]; cf.stride[i] = m->cfg.conv_stride[i]; }
  return launch_clip_frames(lens, B, L, cf, t0, tf, s);
}

template <typename T>
int wavlm_forward(sse_model* m, const float* wave, int B, int L, const Sink& sink_in, char* ws, hipStream_t s,
                  const int* lens = nullptr) {
  const sse_cfg& c = m->cfg;
  Plan p;
  const WavlmWs w = wavlm_plan(m, B, L, p);
  int* t0len = lens ? (int*)(ws + w.fr) : nullptr;
  int* tflen = lens ? t0len + B : nullptr;
  Sink sink = sink_in;
  sink.tlen = tflen;
  if (lens) RC(ragged_frames(m, lens, B, L, t0len, tflen, s));
  int Ts[8];
  const int Tf = wavlm_frames(c, L, Ts);
  const int H = c.hidden, nh = c.heads, F = c.ffn;
  const int M = B * Tf;
  const float eps = c.ln_eps;
  void* zero = ws + w.zero;
  if (hipMemsetAsync(zero, 0, 256, s) != hipSuccess) return SSE_ERR_HIP;
  const float* norm = nullptr;
  if (c.do_normalize) {
    RC(launch_wave_stats(wave, B, L, (float*)(ws + w.norm), s, lens));
    norm = (const float*)(ws + w.norm);
  }
  // ---- conv feature encoder ----
  const int C0 = c.conv_dim[0];
  T* bufs[2] = {(T*)(ws + w.bufA), (T*)(ws + w.bufB)};
  const float* b0 = m->conv_b[0] ? m->ptr<float>(m->conv_b[0]) : nullptr;
  if (c.feat_norm_layer) {
    // "layer" frontend (WavLM-large, HF modeling_wavlm.py:696-720): conv -> LN over channels -> GELU
    // conv0 + LN + GELU fused (one pass over the largest activation); other widths: two passes
    int frc = -3;
    RC(prof(m, s, "conv0_ln", 2.0 * B * (double)Ts[0] * C0 * c.conv_kernel[0], 0, [&] {
      frc = launch_conv0_ln<T>(wave, B, L, norm, m->ptr<float>(m->conv_w[0]), b0, C0, c.conv_kernel[0],
                               c.conv_stride[0], Ts[0], m->ptr<float>(m->conv_ln_w[0]), m->ptr<float>(m->conv_ln_b[0]),
                               1e-5f, bufs[0], s);
      if (frc != -3) return frc;
      return launch_conv0_raw<T>(wave, B, L, norm, m->ptr<float>(m->conv_w[0]), b0, C0, c.conv_kernel[0],
                                 c.conv_stride[0], Ts[0], bufs[0], s); }));
    if (frc == -3)
      RC((launch_layernorm<T, T>(bufs[0], m->ptr<float>(m->conv_ln_w[0]), m->ptr<float>(m->conv_ln_b[0]), B * Ts[0], C0,
                                 1e-5f, ACT_GELU, nullptr, bufs[0], s)));
  } else {
    RC(prof(m, s, "conv0_gn", 2.0 * B * (double)Ts[0] * C0 * c.conv_kernel[0], 0, [&] {
      return launch_conv0_gn<T>(wave, B, L, norm, m->ptr<float>(m->conv_w[0]), b0, C0, c.conv_kernel[0],
                                c.conv_stride[0], Ts[0], m->ptr<float>(m->conv_ln_w[0]), m->ptr<float>(m->conv_ln_b[0]),
                                1e-5f, (double*)(ws + w.part), (float2*)(ws + w.ss), bufs[0], s, t0len); }));
  }
  for (int i = 1; i < c.n_conv; ++i) {
    const int cin = c.conv_dim[i - 1], co = c.conv_dim[i], k = c.conv_kernel[i], st = c.conv_stride[i];
    GemmArgs g{};
    g.A = bufs[(i - 1) & 1]; g.B = m->ptr(m->conv_w[i]);
    g.M = B * Ts[i]; g.N = co; g.K = k * cin;
    g.rows_per_seg = Ts[i]; g.seg_stride = (long long)Ts[i - 1] * cin; g.lda = (long long)st * cin;
    g.bias = m->conv_b[i] ? m->ptr<float>(m->conv_b[i]) : nullptr;
    g.Ct = bufs[i & 1]; g.ldc = co; g.act = c.feat_norm_layer ? ACT_NONE : gelu_rounded_act<T>(); g.zero = zero;
    RC(prof(m, s, "gemm:conv", gflops(g), gbytes<T>(g), [&] { return launch_gemm<T>(g, AMODE_SEG, 1, s); }));
    if (c.feat_norm_layer)
      RC((launch_layernorm<T, T>(bufs[i & 1], m->ptr<float>(m->conv_ln_w[i]), m->ptr<float>(m->conv_ln_b[i]),
                                 B * Ts[i], co, 1e-5f, ACT_GELU, nullptr, bufs[i & 1], s)));
  }
  const T* feat = bufs[(c.n_conv - 1) & 1];
  const int C = c.conv_dim[c.n_conv - 1];
  // ---- feature projection ----
  float* x = (float*)(ws + w.x);
  T* xt = (T*)(ws + w.xt);
  T* xb = (T*)(ws + w.xb);
  RC((launch_layernorm<T, T>(feat, m->ptr<float>(m->fp_ln_w), m->ptr<float>(m->fp_ln_b), M, C, eps, ACT_NONE,
                             nullptr, xb, s)));
  {
    GemmArgs g{};
    g.A = xb; g.B = m->ptr(m->fp_w); g.M = M; g.N = H; g.K = C;
    g.rows_per_seg = M; g.seg_stride = 0; g.lda = C;
    g.bias = m->ptr<float>(m->fp_b); g.Cf = x; g.Ct = xt; g.ldc = H; g.act = ACT_NONE; g.zero = zero;
    RC(prof(m, s, "gemm:proj", gflops(g), gbytes<T>(g), [&] { return launch_gemm<T>(g, AMODE_SEG, 1, s); }));
  }
  // ---- positional conv embedding: x = x + gelu(conv(x) + b) ----
  if (lens) RC(launch_mask_rows<T>(xt, B, Tf, H, tflen, s));   // frames past a clip read as the conv's zero padding
  {
    const int G = c.pos_groups, cg = H / G, K = c.pos_kernel;
    GemmArgs g{};
    g.A = xt; g.B = m->ptr(m->pos_w); g.M = M; g.N = cg; g.K = K * cg;
    g.rows_per_seg = Tf; g.T_in = Tf; g.stride = 1; g.pad = K / 2; g.cin = cg; g.ld_in = H;
    g.bias = m->ptr<float>(m->pos_b); g.resid = x; g.Cf = x; g.ldc = H; g.act = ACT_GELU; g.zero = zero;
    // bf16: the dedicated kernel (input window staged once per block, kernels_posconv.hip);
    // OPT_POSCONV_GEMM keeps the grouped GEMM for bf16 A/B runs (the grouped GEMM has no fp16 form: ignored for fp16)
    const bool use_gemm = sizeof(T) != 2 || (!is_f16_v<T> && sse_opt(OPT_POSCONV_GEMM));
    RC(prof(m, s, "gemm_conv:posconv", gflops(g, G), gbytes<T>(g, AMODE_CONV, G), [&] {
      if (!use_gemm) {
        const int rc = launch_posconv_bf16((const bf16*)xt, m->ptr<bf16>(m->pos_w), m->ptr<float>(m->pos_b), x, B, Tf, H,
                                           G, K, K / 2, s, is_f16_v<T>);
        if (rc != -3) return rc;
      }
      return launch_gemm<T>(g, AMODE_CONV, G, s); }));
  }
  if (!c.stable_layer_norm)
    RC((launch_layernorm<float, T>(x, m->ptr<float>(m->enc_ln_w), m->ptr<float>(m->enc_ln_b), M, H, eps, ACT_NONE,
                                   x, xb, s)));
  // bf16 pre-LN (stable-LN, WavLM-large): the residual stream is kept in bf16 (xt, free after the
  // positional conv): the residual GEMMs read and write it in place, both LayerNorms read bf16, the
  // pooled hidden states are taken from it (half the residual traffic of an fp32 stream)
  const bool pre16 = sizeof(T) == 2 && c.stable_layer_norm;
  T* x16 = pre16 ? xt : nullptr;
  if (pre16) {
    RC((launch_cast<T, float>(x, (long long)M * H, x16, s)));
    RC(sink.emit(0, x16));
  } else {
    RC(sink.emit(0, x));
  }
  // ---- encoder layers ----
  T* qkv = (T*)(ws + w.qkv);
  T* ctx = (T*)(ws + w.ctx);
  T* ff = (T*)(ws + w.ff);
  float* hf = c.stable_layer_norm ? (float*)(ws + w.hf) : nullptr;
  // bf16 post-LN (WavLM-base): no LayerNorm kernel inside the layer loop, and the residual stream
  // in bf16.  The residual GEMMs (oproj, ffn2) write the un-normalised sum in bf16 -- xs after the
  // attention, xb after the FFN: at once the residual of the next residual GEMM and the A operand
  // of the next GEMM -- plus per-256-column partial statistics of the rounded values (p1 / p2);
  // the consumers apply the LayerNorm from those partials: QKV / FFN1 through folded weights
  // (GemmArgs.apart: rstd (acc - mean acol) + b'), the next residual GEMM on its residual load
  // (rpart), the pool on its loads.  OPT_NO_LNFOLD restores the materialised flow (LayerNorm
  // kernels, fp32 residual; A/B tests).
  const bool lnfold = sizeof(T) == 2 && m->ln_fold && !sse_opt(OPT_NO_LNFOLD);
  const int nt = H / 256;
  float2* p1 = (float2*)(ws + w.p1);
  float2* p2 = (float2*)(ws + w.p2);
  T* xs = xt;   // bf16 residual sum after the attention (xt, the projection output, is free by now)
  // bf16 stable-LN (WavLM-large, round 6): layer l > 0's attention LayerNorm folded into its QKV (the previous ffn2
  // writes the partials p2 of the bf16 stream); layer 0 and fc1 keep their LayerNorm kernels
  const bool prefold = pre16 && m->pre_fold && !sse_opt(OPT_NO_LNFOLD);
  for (int l = 0; l < c.layers; ++l) {
    const LayerW& Lw = m->layers[l];
    const LayerW* Lp = l > 0 ? &m->layers[l - 1] : nullptr;
    if (pre16) {
      if (!(prefold && l > 0))
        RC((launch_layernorm<T, T>(x16, m->ptr<float>(Lw.ln1_w), m->ptr<float>(Lw.ln1_b), M, H, eps, ACT_NONE,
                                   nullptr, xb, s)));
    } else if (c.stable_layer_norm)
      RC((launch_layernorm<float, T>(x, m->ptr<float>(Lw.ln1_w), m->ptr<float>(Lw.ln1_b), M, H, eps, ACT_NONE,
                                     nullptr, xb, s)));
    GemmArgs g{};
    g.A = xb; g.B = m->ptr(Lw.qkv_w); g.M = M; g.N = m->ldq; g.K = H;
    g.rows_per_seg = M; g.lda = H; g.bias = m->ptr<float>(Lw.qkv_b); g.Ct = qkv; g.ldc = m->ldq; g.zero = zero;
    if (lnfold && l > 0) {   // xb = bf16 of the previous layer's un-normalised sum: its final LN folded
      g.B = m->ptr(Lw.qkv_wf); g.bias = m->ptr<float>(Lw.qkv_bf); g.acol = m->ptr<float>(Lw.qkv_c);
      g.apart = p2; g.apart_nt = nt; g.ln_eps = eps;
    }
    if (prefold && l > 0) {   // the bf16 stream itself, this layer's attention LN folded (partials from ffn2)
      g.A = x16; g.B = m->ptr(Lw.qkv_wf); g.bias = m->ptr<float>(Lw.qkv_bf); g.acol = m->ptr<float>(Lw.qkv_c);
      g.apart = p2; g.apart_nt = nt; g.ln_eps = eps;
    }
    // algorithmic FLOPs count the 3H + 8*heads useful columns, not the zero pad to ldq
    RC(prof(m, s, "gemm:qkv", 2.0 * M * (3.0 * H + 8.0 * nh) * H, gbytes<T>(g),
            [&] { return launch_gemm<T>(g, AMODE_SEG, 1, s); }));
    AttnArgs a{};
    a.qkv = qkv; a.out = ctx; a.T = Tf; a.H = H; a.nh = nh; a.ldq = m->ldq; a.scale = 0.125f;
    a.gconst = m->ptr<float>(Lw.g_const); a.relb = m->ptr<float>(m->relb); a.maxd = MAXD; a.tlen = tflen;
    RC(prof(m, s, "attn", 4.0 * B * (double)Tf * Tf * H, (double)B * Tf * (4.0 * H + 8.0 * nh) * sizeof(T),
            [&] { return launch_attention<T>(a, B, s); }));
    g = GemmArgs{};
    g.A = ctx; g.B = m->ptr(Lw.o_w); g.M = M; g.N = H; g.K = H; g.rows_per_seg = M; g.lda = H;
    g.bias = m->ptr<float>(Lw.o_b); g.resid = x; g.Cf = x; g.ldc = H; g.zero = zero;
    if (lnfold) {   // residual = xb: layer 0 the encoder LN output, later the previous layer's bf16 sum
      g.resid = nullptr; g.Cf = nullptr; g.resid_t = (const bf16*)xb;
      if (l > 0) {   // the previous layer's final LN applied on the residual load
        g.rpart = p2; g.rpart_nt = nt; g.ln_eps = eps;
        g.rln_w = m->ptr<float>(Lp->ln2_w); g.rln_b = m->ptr<float>(Lp->ln2_b);
      }
      g.Ct = xs; g.opart = p1;
    }
    if (pre16) {
      g.resid = nullptr; g.Cf = nullptr; g.resid_t = (const bf16*)x16; g.Ct = x16;
    }
    RC(prof(m, s, "gemm:oproj", gflops(g), gbytes<T>(g), [&] { return launch_gemm<T>(g, AMODE_SEG, 1, s); }));
    if (pre16) {
      RC((launch_layernorm<T, T>(x16, m->ptr<float>(Lw.ln2_w), m->ptr<float>(Lw.ln2_b), M, H, eps, ACT_NONE,
                                 nullptr, xb, s)));
    } else if (!lnfold) {
      if (!c.stable_layer_norm)
        RC((launch_layernorm<float, T>(x, m->ptr<float>(Lw.ln1_w), m->ptr<float>(Lw.ln1_b), M, H, eps, ACT_NONE, x,
                                       xb, s)));
      else
        RC((launch_layernorm<float, T>(x, m->ptr<float>(Lw.ln2_w), m->ptr<float>(Lw.ln2_b), M, H, eps, ACT_NONE,
                                       nullptr, xb, s)));
    }
    g = GemmArgs{};
    g.A = xb; g.B = m->ptr(Lw.f1_w); g.M = M; g.N = F; g.K = H; g.rows_per_seg = M; g.lda = H;
    g.bias = m->ptr<float>(Lw.f1_b); g.Ct = ff; g.ldc = F; g.act = gelu_rounded_act<T>(); g.zero = zero;
    if (lnfold) {   // xs = bf16 of the un-normalised attention sum: the attention LN folded
      g.A = xs; g.B = m->ptr(Lw.f1_wf); g.bias = m->ptr<float>(Lw.f1_bf); g.acol = m->ptr<float>(Lw.f1_c);
      g.apart = p1; g.apart_nt = nt; g.ln_eps = eps;
    }
    RC(prof(m, s, "gemm:ffn1", gflops(g), gbytes<T>(g), [&] { return launch_gemm<T>(g, AMODE_SEG, 1, s); }));
    g = GemmArgs{};
    g.A = ff; g.B = m->ptr(Lw.f2_w); g.M = M; g.N = H; g.K = F; g.rows_per_seg = M; g.lda = F;
    g.bias = m->ptr<float>(Lw.f2_b); g.resid = x; g.Cf = x; g.ldc = H; g.zero = zero;
    if (lnfold) {
      g.resid = nullptr; g.Cf = nullptr; g.resid_t = (const bf16*)xs;
      g.rpart = p1; g.rpart_nt = nt; g.ln_eps = eps; g.rln_w = m->ptr<float>(Lw.ln1_w); g.rln_b = m->ptr<float>(Lw.ln1_b);
      g.Ct = xb; g.opart = p2;
    }
    if (pre16) {
      g.resid = nullptr; g.Cf = nullptr; g.resid_t = (const bf16*)x16; g.Ct = x16;
      if (prefold && l + 1 < c.layers) g.opart = p2;   // the next QKV's LayerNorm statistics
    }
    RC(prof(m, s, "gemm:ffn2", gflops(g), gbytes<T>(g), [&] { return launch_gemm<T>(g, AMODE_SEG, 1, s); }));
    if (pre16) {
      if (l + 1 < c.layers) RC(sink.emit(l + 1, x16));
      continue;
    }
    if (lnfold) {
      RC(sink.emit_ln<T>(l + 1, xb, nullptr, m->ptr<float>(Lw.ln2_w), m->ptr<float>(Lw.ln2_b), eps, p2, nt));
      continue;
    }
    if (!c.stable_layer_norm) {
      RC((launch_layernorm<float, T>(x, m->ptr<float>(Lw.ln2_w), m->ptr<float>(Lw.ln2_b), M, H, eps, ACT_NONE, x,
                                     xb, s)));
    }
    if (l + 1 < c.layers || !c.stable_layer_norm) RC(sink.emit(l + 1, x));
  }
  if (pre16) {
    RC((launch_layernorm<T, T>(x16, m->ptr<float>(m->enc_ln_w), m->ptr<float>(m->enc_ln_b), M, H, eps, ACT_NONE,
                               x, xb, s)));
    RC(sink.emit(c.layers, x));
  } else if (c.stable_layer_norm) {
    RC((launch_layernorm<float, T>(x, m->ptr<float>(m->enc_ln_w), m->ptr<float>(m->enc_ln_b), M, H, eps, ACT_NONE,
                                   x, xb, s)));
    RC(sink.emit(c.layers, x));
  }
  return 0;
}

// ---- SSE_DTYPE_FP16X3: the fp32 path with split-fp16 GEMMs ----------------------------------
// Every GEMM operand is stored tripled (common.h x3_split4): an activation row [hi | lo' | hi] of 3K
// fp16 (hi = f16(v), lo' = f16((v - hi) 2^11)), the weights 2^e-scaled [hi | hi 2^-11 | lo] per
// K-block (Arena::put_x3).  The 8-phase kernels run on K' = 3K with the f16 MFMA and accumulate
// hi*hi + lo*hi + hi*lo in fp32 (~22 significant bits per operand; the dropped lo*lo is ~2^-22
// relative); the epilogue scales by alpha = 2^-e.  Strided convs keep their overlapping-row
// addressing: a frame is 3C values, a window of k frames k*3C.  conv0 + GroupNorm + GELU, the
// positional conv and the attention core (scores, softmax, P.V) run in exact fp32 as in the fp32
// path; LayerNorms read / write fp32 and tripled rows.
struct X3Ws {
  size_t zero, norm, part, ss, bufA, bufB, x, xt, xb, qkv, ctx3, ff, fr;
};

X3Ws x3_plan(const sse_model* m, int B, int L, Plan& p) {
  const sse_cfg& c = m->cfg;
  int Ts[8];
  const int T = wavlm_frames(c, L, Ts);
  const size_t M = (size_t)B * T;
  const int H = c.hidden, C0 = c.conv_dim[0];
  size_t maxA = 0, maxB = 0;
  for (int i = 0; i < c.n_conv; ++i) {
    const size_t sz = (size_t)B * Ts[i] * c.conv_dim[i] * 6;
    if (i % 2 == 0) maxA = sz > maxA ? sz : maxA; else maxB = sz > maxB ? sz : maxB;
  }
  const int Cl = c.conv_dim[c.n_conv - 1];
  X3Ws w;
  w.zero = p.add(256);
  w.norm = p.add((size_t)B * 8);
  w.part = p.add(conv0_moments_bytes(B));
  w.ss = p.add((size_t)B * C0 * 8);
  w.bufA = p.add(maxA);
  w.bufB = p.add(maxB);
  w.x = p.add(M * H * 4);
  w.xt = p.add(M * H * 4);
  w.xb = p.add(M * (size_t)(H > Cl ? H : Cl) * 6);
  w.qkv = p.add(M * (size_t)(((3 * H + 8 * c.heads + 255) / 256) * 256) * 4);
  w.ctx3 = p.add(M * H * 6);
  w.ff = p.add(M * (size_t)c.ffn * 6);
  w.fr = p.add((size_t)B * 8);
  return w;
}

int wavlm_forward_x3(sse_model* m, const float* wave, int B, int L, const Sink& sink_in, char* ws, hipStream_t s,
                     const int* lens = nullptr) {
  const sse_cfg& c = m->cfg;
  Plan p;
  const X3Ws w = x3_plan(m, B, L, p);
  int* t0len = lens ? (int*)(ws + w.fr) : nullptr;
  int* tflen = lens ? t0len + B : nullptr;
  Sink sink = sink_in;
  sink.tlen = tflen;
  if (lens) RC(ragged_frames(m, lens, B, L, t0len, tflen, s));
  int Ts[8];
  const int Tf = wavlm_frames(c, L, Ts);
  const int H = c.hidden, nh = c.heads, F = c.ffn;
  const int M = B * Tf;
  const float eps = c.ln_eps;
  void* zero = ws + w.zero;
  if (hipMemsetAsync(zero, 0, 256, s) != hipSuccess) return SSE_ERR_HIP;
  const float* norm = nullptr;
  if (c.do_normalize) {
    RC(launch_wave_stats(wave, B, L, (float*)(ws + w.norm), s, lens));
    norm = (const float*)(ws + w.norm);
  }
  // split-fp16 GEMM: logical K (the FLOP count), physical operands K' = 3K
  auto gemm3 = [&](const char* tag, GemmArgs& g, int Klog) {
    g.zero = zero;
    g.f16 = 1;
    g.alpha = m->alpha((size_t)((const char*)g.B - m->dmem));
    return prof(m, s, tag, 2.0 * g.M * (double)g.N * Klog, gbytes<bf16>(g), [&] { return launch_gemm8_bf16(g, s); });
  };
  // ---- conv feature encoder: conv0 + GroupNorm + GELU in fp32, then tripled ----
  const int C0 = c.conv_dim[0];
  const float* b0 = m->conv_b[0] ? m->ptr<float>(m->conv_b[0]) : nullptr;
  f16* bufs[2] = {(f16*)(ws + w.bufA), (f16*)(ws + w.bufB)};
  const f16* feat = nullptr;
  if (c.feat_norm_layer) {
    // "layer" frontend (WavLM-large, HF modeling_wavlm.py:696-720): conv -> LayerNorm over channels ->
    // erf-GELU per layer.  conv0 + LN + GELU in one fp32 pass written tripled (bufA); each later conv is a
    // split GEMM with fp32 output (into bufB) whose LayerNorm + GELU writes the next tripled operand back
    // over its own (consumed) input in bufA
    RC(prof(m, s, "conv0_ln", 2.0 * B * (double)Ts[0] * C0 * c.conv_kernel[0], 0, [&] {
      return launch_conv0_ln_x3(wave, B, L, norm, m->ptr<float>(m->conv_w[0]), b0, C0, c.conv_kernel[0],
                                c.conv_stride[0], Ts[0], m->ptr<float>(m->conv_ln_w[0]), m->ptr<float>(m->conv_ln_b[0]),
                                1e-5f, bufs[0], s); }));
    float* yf = (float*)bufs[1];
    for (int i = 1; i < c.n_conv; ++i) {
      const int cin = c.conv_dim[i - 1], co = c.conv_dim[i], k = c.conv_kernel[i], st = c.conv_stride[i];
      GemmArgs g{};
      g.A = bufs[0]; g.B = m->ptr(m->conv_w[i]);
      g.M = B * Ts[i]; g.N = co; g.K = k * 3 * cin;
      g.rows_per_seg = Ts[i]; g.seg_stride = (long long)Ts[i - 1] * 3 * cin; g.lda = (long long)st * 3 * cin;
      g.bias = m->conv_b[i] ? m->ptr<float>(m->conv_b[i]) : nullptr;
      g.Cf = yf; g.ldc = co; g.act = ACT_NONE;
      RC(gemm3("gemm:conv", g, k * cin));
      RC(launch_layernorm_x3(yf, false, m->ptr<float>(m->conv_ln_w[i]), m->ptr<float>(m->conv_ln_b[i]), B * Ts[i], co,
                             1e-5f, nullptr, bufs[0], s, ACT_GELU));
    }
    feat = bufs[0];
  } else {
    RC(prof(m, s, "conv0_gn", 2.0 * B * (double)Ts[0] * C0 * c.conv_kernel[0], 0, [&] {
      return launch_conv0_gn_x3(wave, B, L, norm, m->ptr<float>(m->conv_w[0]), b0, C0, c.conv_kernel[0],
                                c.conv_stride[0], Ts[0], m->ptr<float>(m->conv_ln_w[0]), m->ptr<float>(m->conv_ln_b[0]),
                                1e-5f, (double*)(ws + w.part), (float2*)(ws + w.ss), bufs[0], s, t0len); }));
    for (int i = 1; i < c.n_conv; ++i) {
      const int cin = c.conv_dim[i - 1], co = c.conv_dim[i], k = c.conv_kernel[i], st = c.conv_stride[i];
      GemmArgs g{};
      g.A = bufs[(i - 1) & 1]; g.B = m->ptr(m->conv_w[i]);
      g.M = B * Ts[i]; g.N = co; g.K = k * 3 * cin;
      g.rows_per_seg = Ts[i]; g.seg_stride = (long long)Ts[i - 1] * 3 * cin; g.lda = (long long)st * 3 * cin;
      g.bias = m->conv_b[i] ? m->ptr<float>(m->conv_b[i]) : nullptr;
      g.Ct = bufs[i & 1]; g.ct3 = 1; g.ldc = 3 * co; g.act = ACT_GELU;
      RC(gemm3("gemm:conv", g, k * cin));
    }
    feat = bufs[(c.n_conv - 1) & 1];
  }
  const int C = c.conv_dim[c.n_conv - 1];
  float* x = (float*)(ws + w.x);
  float* xt = (float*)(ws + w.xt);
  f16* xb = (f16*)(ws + w.xb);
  // ---- feature projection ----
  RC(launch_layernorm_x3(feat, true, m->ptr<float>(m->fp_ln_w), m->ptr<float>(m->fp_ln_b), M, C, eps, nullptr, xb, s));
  {
    GemmArgs g{};
    g.A = xb; g.B = m->ptr(m->fp_w); g.M = M; g.N = H; g.K = 3 * C; g.rows_per_seg = M; g.lda = 3 * C;
    g.bias = m->ptr<float>(m->fp_b); g.Cf = x; g.ldc = H;
    RC(gemm3("gemm:proj", g, C));
  }
  if (hipMemcpyAsync(xt, x, (size_t)M * H * 4, hipMemcpyDeviceToDevice, s) != hipSuccess) return SSE_ERR_HIP;
  if (lens) RC(launch_mask_rows<float>(xt, B, Tf, H, tflen, s));
  // ---- positional conv embedding: x = x + gelu(conv(x) + b), split-fp16 matrix cores (the fp32
  // grouped GEMM for shapes outside posconv_x3_kernel or under OPT_POSCONV_GEMM) ----
  int prc = -3;
  if (!sse_opt(OPT_POSCONV_GEMM))
    RC(prof(m, s, "gemm_conv:posconv", 2.0 * B * (double)Tf * H * c.pos_kernel * (H / c.pos_groups),
            (double)B * Tf * H * 8 + (double)H * c.pos_kernel * (H / c.pos_groups) * 4, [&] {
      prc = launch_posconv_x3(xt, m->ptr<f16>(m->pos_w3), m->alpha(m->pos_w3), m->ptr<float>(m->pos_b), x, B, Tf, H,
                              c.pos_groups, c.pos_kernel, c.pos_kernel / 2, s);
      return prc == -3 ? 0 : prc; }));
  if (prc == -3) {
    const int G = c.pos_groups, cg = H / G, K = c.pos_kernel;
    GemmArgs g{};
    g.A = xt; g.B = m->ptr(m->pos_w); g.M = M; g.N = cg; g.K = K * cg;
    g.rows_per_seg = Tf; g.T_in = Tf; g.stride = 1; g.pad = K / 2; g.cin = cg; g.ld_in = H;
    g.bias = m->ptr<float>(m->pos_b); g.resid = x; g.Cf = x; g.ldc = H; g.act = ACT_GELU; g.zero = zero;
    RC(prof(m, s, "gemm_conv:posconv", gflops(g, G), gbytes<float>(g, AMODE_CONV, G),
            [&] { return launch_gemm<float>(g, AMODE_CONV, G, s); }));
  }
  // post-LN (WavLM-base): the encoder LayerNorm before the layers; stable-LN (WavLM-large, HF
  // modeling_wavlm.py:465-522): pre-LN layers and the encoder LayerNorm after the last one
  const bool pre = c.stable_layer_norm;
  if (!pre) RC(launch_layernorm_x3(x, false, m->ptr<float>(m->enc_ln_w), m->ptr<float>(m->enc_ln_b), M, H, eps, x, xb, s));
  RC(sink.emit(0, x));
  float* qkv = (float*)(ws + w.qkv);
  f16* ctx3 = (f16*)(ws + w.ctx3);
  f16* ff = (f16*)(ws + w.ff);
  for (int l = 0; l < c.layers; ++l) {
    const LayerW& Lw = m->layers[l];
    if (pre) RC(launch_layernorm_x3(x, false, m->ptr<float>(Lw.ln1_w), m->ptr<float>(Lw.ln1_b), M, H, eps, nullptr, xb, s));
    GemmArgs g{};
    g.A = xb; g.B = m->ptr(Lw.qkv_w); g.M = M; g.N = m->ldq; g.K = 3 * H;
    g.rows_per_seg = M; g.lda = 3 * H; g.bias = m->ptr<float>(Lw.qkv_b); g.Cf = qkv; g.ldc = m->ldq;
    g.zero = zero;
    g.f16 = 1;
    g.alpha = m->alpha(Lw.qkv_w);
    RC(prof(m, s, "gemm:qkv", 2.0 * M * (3.0 * H + 8.0 * nh) * H, gbytes<bf16>(g),
            [&] { return launch_gemm8_bf16(g, s); }));
    AttnArgs a{};
    a.qkv = qkv; a.out = ctx3; a.out3 = 1; a.T = Tf; a.H = H; a.nh = nh; a.ldq = m->ldq; a.scale = 0.125f;
    a.gconst = m->ptr<float>(Lw.g_const); a.relb = m->ptr<float>(m->relb); a.maxd = MAXD; a.tlen = tflen;
    // the attention writes the out-projection's tripled operand itself (no fp32 context round trip)
    RC(prof(m, s, "attn", 4.0 * B * (double)Tf * Tf * H, (double)B * Tf * ((3.0 * H + 8.0 * nh) * 4.0 + 6.0 * H),
            [&] { return launch_attention<float>(a, B, s); }));
    g = GemmArgs{};
    g.A = ctx3; g.B = m->ptr(Lw.o_w); g.M = M; g.N = H; g.K = 3 * H; g.rows_per_seg = M; g.lda = 3 * H;
    g.bias = m->ptr<float>(Lw.o_b); g.resid = x; g.Cf = x; g.ldc = H;
    RC(gemm3("gemm:oproj", g, H));
    if (pre)
      RC(launch_layernorm_x3(x, false, m->ptr<float>(Lw.ln2_w), m->ptr<float>(Lw.ln2_b), M, H, eps, nullptr, xb, s));
    else
      RC(launch_layernorm_x3(x, false, m->ptr<float>(Lw.ln1_w), m->ptr<float>(Lw.ln1_b), M, H, eps, x, xb, s));
    g = GemmArgs{};
    g.A = xb; g.B = m->ptr(Lw.f1_w); g.M = M; g.N = F; g.K = 3 * H; g.rows_per_seg = M; g.lda = 3 * H;
    g.bias = m->ptr<float>(Lw.f1_b); g.Ct = ff; g.ct3 = 1; g.ldc = 3 * F; g.act = ACT_GELU;
    RC(gemm3("gemm:ffn1", g, H));
    g = GemmArgs{};
    g.A = ff; g.B = m->ptr(Lw.f2_w); g.M = M; g.N = H; g.K = 3 * F; g.rows_per_seg = M; g.lda = 3 * F;
    g.bias = m->ptr<float>(Lw.f2_b); g.resid = x; g.Cf = x; g.ldc = H;
    RC(gemm3("gemm:ffn2", g, F));
    if (pre) {   // hidden_states[l + 1] = the residual stream (the last one: after the encoder LayerNorm)
      if (l + 1 < c.layers) RC(sink.emit(l + 1, x));
      continue;
    }
    RC(launch_layernorm_x3(x, false, m->ptr<float>(Lw.ln2_w), m->ptr<float>(Lw.ln2_b), M, H, eps, x, xb, s));
    RC(sink.emit(l + 1, x));
  }
  if (pre) {
    RC(launch_layernorm_x3(x, false, m->ptr<float>(m->enc_ln_w), m->ptr<float>(m->enc_ln_b), M, H, eps, x, xb, s));
    RC(sink.emit(c.layers, x));
  }
  return 0;
}

// The reference's 1-token decoder pass (REF/whisper_embeddings_large.py:257-262): input id 0 at
// position 0, cross-attending to the encoder's last_hidden_state enc [B*Tq][D] (type T).  Rows
// are clips (M = B); the K|V projection of the encoder output is the one large GEMM per layer.
// hidden_states[i] = input of layer i, hidden_states[L] = final-LN output
// (HF/models/whisper/modeling_whisper.py:739-790, HF/utils/output_capturing.py:268-279).
template <typename T>
int whisper_decoder(sse_model* m, const T* enc, int B, const Sink& sink, char* ws, const WhisperWs& w,
                    hipStream_t s) {
  const sse_cfg& c = m->cfg;
  const int D = c.hidden, Fd = c.dec_ffn, nh = c.heads, Tq = c.max_positions;
  const float eps = c.ln_eps;
  void* zero = ws + w.zero;
  float* x = (float*)(ws + w.dx);
  T* xb = (T*)(ws + w.dxb);
  T* v = (T*)(ws + w.dv);
  T* q = (T*)(ws + w.dq);
  T* ctx = (T*)(ws + w.dctx);
  T* ff = (T*)(ws + w.dff);
  T* kv = (T*)(ws + w.qkv);   // encoder QKV buffer [B*Tq][3D] >= [B*Tq][2D]
  RC(launch_bcast_rows(m->ptr<float>(m->dec_x0), D, B, x, s));
  RC(sink.emit(0, x));
  auto lin = [&](const char* tag, const T* A, size_t wo, size_t bo, int N, int K, const float* resid, float* Cf,
                 T* Ct, int act) {
    GemmArgs g{};
    g.A = A; g.B = m->ptr(wo); g.M = B; g.N = N; g.K = K; g.rows_per_seg = B; g.lda = K;
    g.bias = m->ptr<float>(bo); g.resid = resid; g.Cf = Cf; g.Ct = Ct; g.ldc = N; g.act = act; g.zero = zero;
    return prof(m, s, tag, gflops(g), gbytes<T>(g), [&] { return launch_gemm<T>(g, AMODE_SEG, 1, s); });
  };
  for (int l = 0; l < c.decoder_layers; ++l) {
    const DecLayerW& W = m->dec[l];
    // self-attention over the single (own) key: softmax == 1, so attn == v_proj(LN(x))
    RC((launch_layernorm<float, T>(x, m->ptr<float>(W.ln1_w), m->ptr<float>(W.ln1_b), B, D, eps, ACT_NONE, nullptr,
                                   xb, s)));
    RC(lin("dec_gemm:v", xb, W.v_w, W.v_b, D, D, nullptr, nullptr, v, ACT_NONE));
    RC(lin("dec_gemm:o", v, W.o_w, W.o_b, D, D, x, x, nullptr, ACT_NONE));
    // cross-attention
    RC((launch_layernorm<float, T>(x, m->ptr<float>(W.ln2_w), m->ptr<float>(W.ln2_b), B, D, eps, ACT_NONE, nullptr,
                                   xb, s)));
    RC(lin("dec_gemm:q", xb, W.q_w, W.q_b, D, D, nullptr, nullptr, q, ACT_NONE));
    {
      GemmArgs g{};
      g.A = enc; g.B = m->ptr(W.kv_w); g.M = B * Tq; g.N = 2 * D; g.K = D; g.rows_per_seg = B * Tq; g.lda = D;
      g.bias = m->ptr<float>(W.kv_b); g.Ct = kv; g.ldc = 2 * D; g.zero = zero;
      RC(prof(m, s, "gemm:dec_kv", gflops(g), gbytes<T>(g), [&] { return launch_gemm<T>(g, AMODE_SEG, 1, s); }));
    }
    RC(prof(m, s, "dec_xattn", 4.0 * B * (double)Tq * D, (double)B * Tq * 2 * D * sizeof(T),
            [&] { return launch_xattn1<T>(q, kv, B, Tq, D, nh, ctx, s); }));
    RC(lin("dec_gemm:co", ctx, W.co_w, W.co_b, D, D, x, x, nullptr, ACT_NONE));
    // feed-forward
    RC((launch_layernorm<float, T>(x, m->ptr<float>(W.ln3_w), m->ptr<float>(W.ln3_b), B, D, eps, ACT_NONE, nullptr,
                                   xb, s)));
    RC(lin("dec_gemm:fc1", xb, W.f1_w, W.f1_b, Fd, D, nullptr, nullptr, ff, gelu_rounded_act<T>()));
    RC(lin("dec_gemm:fc2", ff, W.f2_w, W.f2_b, D, Fd, x, x, nullptr, ACT_NONE));
    if (l + 1 < c.decoder_layers) RC(sink.emit(l + 1, x));
  }
  float* xf = (float*)(ws + w.dxf);
  RC((launch_layernorm<float, T>(x, m->ptr<float>(m->dec_ln_w), m->ptr<float>(m->dec_ln_b), B, D, eps, ACT_NONE, xf,
                                 (T*)nullptr, s)));
  return sink.emit(c.decoder_layers, xf);
}

template <typename T>
int whisper_forward(sse_model* m, const float* wave, int B, int L, const Sink& sink, char* ws, hipStream_t s,
                    const float* mel_hf = nullptr, const Sink* dsink = nullptr, const int* lens = nullptr) {
  const sse_cfg& c = m->cfg;
  Plan p;
  const WhisperWs w = whisper_plan(m, B, p);
  const int D = c.hidden, F = c.ffn, nh = c.heads, Tq = c.max_positions, T2 = 2 * Tq, nm = c.n_mels;
  const int M = B * Tq;
  const float eps = c.ln_eps;
  void* zero = ws + w.zero;
  if (hipMemsetAsync(zero, 0, 256, s) != hipSuccess) return SSE_ERR_HIP;
  T* mel = (T*)(ws + w.mel);
  if (mel_hf)
    RC(launch_mel_to_cl<T>(mel_hf, B, nm, mel, s));
  else
    RC(prof(m, s, "logmel", B * 3000.0 * 5.0 * 200 * 7.64, (double)B * (480000.0 * 4 + 3000.0 * nm * (8.0 + sizeof(T))),
            [&] { return launch_logmel<T>(wave, B, L, nm, nullptr, mel, ws + w.lm, logmel_workspace_bytes(B, nm), s,
                                          lens); }));
  T* h1 = (T*)(ws + w.h1);
  // residual stream in the path's element type: the bf16 / MX-fp8 paths keep it in bf16 (the residual
  // GEMMs read and write half the bytes, LayerNorm reads half; adds ~1e-3 rel-L2 against a ~6e-3 bf16
  // path error), the fp32 path in fp32
  using R = std::conditional_t<sizeof(T) == 2, bf16, float>;
  R* x = (R*)(ws + w.x);
  T* xb = (T*)(ws + w.xb);
  auto set_out = [&](GemmArgs& g) {   // C = x (+ residual x): bf16 stream or fp32
    if constexpr (sizeof(R) == 2) g.Ct = x; else g.Cf = x;
  };
  auto set_resid = [&](GemmArgs& g) {
    if constexpr (sizeof(R) == 2) g.resid_t = x; else g.resid = x;
    set_out(g);
  };
  {
    GemmArgs g{};   // conv1: k3 pad1, 80 -> D, GELU
    g.A = mel; g.B = m->ptr(m->c1_w); g.M = B * T2; g.N = D; g.K = 3 * nm;
    g.rows_per_seg = T2; g.T_in = T2; g.stride = 1; g.pad = 1; g.cin = nm; g.ld_in = nm;
    g.bias = m->ptr<float>(m->c1_b); g.Ct = h1; g.ldc = D; g.act = gelu_rounded_act<T>(); g.zero = zero;
    RC(prof(m, s, "gemm_conv:conv1", gflops(g), gbytes<T>(g, AMODE_CONV), [&] { return launch_gemm<T>(g, AMODE_CONV, 1, s); }));
    g = GemmArgs{};   // conv2: k3 s2 pad1, GELU, + embed_positions
    g.A = h1; g.B = m->ptr(m->c2_w); g.M = M; g.N = D; g.K = 3 * D;
    g.rows_per_seg = Tq; g.T_in = T2; g.stride = 2; g.pad = 1; g.cin = D; g.ld_in = D;
    g.bias = m->ptr<float>(m->c2_b); g.resid = m->ptr<float>(m->positions); g.resid_rows = Tq;
    set_out(g); g.ldc = D; g.act = ACT_GELU; g.zero = zero;
    RC(prof(m, s, "gemm_conv:conv2", gflops(g), gbytes<T>(g, AMODE_CONV), [&] { return launch_gemm<T>(g, AMODE_CONV, 1, s); }));
  }
  RC(sink.emit(0, x));
  T* qkv = (T*)(ws + w.qkv);
  T* ctx = (T*)(ws + w.ctx);
  T* ff = (T*)(ws + w.ff);
  // SSE_DTYPE_FP8: LayerNorm writes the MX-fp8 operand (e4m3 + scales) into xb's space, fc1 writes
  // MX-fp8 into ff's space; QKV / fc1 / fc2 run on the MX GEMM (kernels_gemm8.hip)
  const bool mx = m->mx();
  unsigned char* xq = (unsigned char*)(ws + w.xb);
  unsigned char* xq_s = xq + (size_t)M * D;
  unsigned char* fq = (unsigned char*)(ws + w.ff);
  unsigned char* fq_s = fq + (size_t)M * F;
  // fp8 attention (default on the MX path): Q | K e4m3 [M][2D] | V bf16 [M][D] | Q | K scales [M][2D / 32] in
  // the QKV space ([M][3D] bf16 = 6D bytes per row)
  const bool f8attn = mx && !sse_opt(OPT_FP8_ATTN_BF16);
  // MX-fp8 out-projection (round 6, opt-in f8_oproj = 1): the attention writes its output as MX-fp8 (e4m3 +
  // A-layout scales) into ctx's space and the out-projection runs on the MX GEMM with the residual.  Not the
  // default: one more e4m3 rounding per layer takes Whisper-large-v2 (B = 128, 32 layers) from 0.066 to 0.083
  // rel-L2 against the reference fixture, over the fp8 bar of 0.08 (tests/test_gpu_whisper.py)
  const bool f8oproj = f8attn && D % 128 == 0 && sse_opt(OPT_F8_OPROJ);
  unsigned char* cq = (unsigned char*)ctx;
  unsigned char* cq_s = cq + (size_t)M * D;
  unsigned char* qk8 = (unsigned char*)qkv;
  bf16* v16 = (bf16*)(qk8 + (size_t)M * 2 * D);
  unsigned char* qks = qk8 + (size_t)M * 4 * D;
  unsigned* vam = mx ? (unsigned*)(ws + w.vam) : nullptr;
  auto mx_gemm = [&](const char* tag, const unsigned char* A, const unsigned char* As, size_t wq, size_t wsc, size_t bo,
                     int N, int K, bool res, void* Ct, unsigned char* Cs, int act) {
    GemmArgs g{};
    g.A = A; g.a_scale = As; g.B = m->ptr(wq); g.b_scale = m->ptr<unsigned char>(wsc);
    g.M = M; g.N = N; g.K = K; g.rows_per_seg = M; g.lda = K;
    g.bias = m->ptr<float>(bo); g.Ct = Ct; g.c_scale = Cs; g.ldc = N; g.act = act;
    if (res) set_resid(g);   // C = x + A B^T + b (the residual stream, in place)
    g.zero = zero;
    const double bytes = (double)M * K + (double)N * K + (M + (double)N) * K / 32.0 +
                         (res ? 2.0 * M * N * sizeof(R) : 0.0) +
                         (!res && Ct ? (double)M * N * (Cs ? 1.0 + 1.0 / 32 : 2.0) : 0.0);
    return prof(m, s, tag, gflops(g), bytes, [&] { return launch_gemm8_mx(g, s); });
  };
  // folded pre-LN (bf16 whisper-small): the residual GEMMs (oproj, fc2) also write per-256-column partial
  // statistics of the rows they store (p1 after the attention, p2 after the FFN), and QKV / fc1 apply their
  // LayerNorm from those partials through folded weights (rstd (x W'^T - mean acol) + b') -- no LayerNorm
  // kernel and no normalised copy of the stream, except layer 0's QKV input (the conv stem has no partials)
  const bool lnfold = sizeof(T) == 2 && !mx && m->ln_fold;   // fixed at load (build_whisper: wfold)
  // fc1's fold only at D = 768: its GELU epilogue with 4-5 partials per row spills (the LayerNorm kernel
  // plus the plain fc1 are the faster pair there); QKV folds at every D
  const bool f1fold = lnfold && D == 768;
  const int nt = D / 256;
  float2* p1 = (float2*)(ws + w.p1);
  float2* p2 = (float2*)(ws + w.p2);
  for (int l = 0; l < c.layers; ++l) {
    const LayerW& Lw = m->layers[l];
    if (mx) {
      RC(launch_layernorm_mx<R>(x, m->ptr<float>(Lw.ln1_w), m->ptr<float>(Lw.ln1_b), M, D, eps, xq, xq_s, s));
      if (f8attn) {
        // one GEMM over the packed [3D][D] weights: Q | K columns as MX-fp8 with row-major scales (the attention
        // reads them per row), V columns bf16 plus their per-(clip, column) amax (gemm8_kernel<MXE = 6>)
        RC(hipMemsetAsync(vam, 0, (size_t)B * D * 4, s) == hipSuccess ? 0 : SSE_ERR_HIP);
        GemmArgs g{};
        g.A = xq; g.a_scale = xq_s; g.B = m->ptr(Lw.qkv_q); g.b_scale = m->ptr<unsigned char>(Lw.qkv_s);
        g.M = M; g.N = 3 * D; g.K = D; g.rows_per_seg = M; g.lda = D; g.bias = m->ptr<float>(Lw.qkv_b); g.zero = zero;
        g.Ct = qk8; g.c_scale = qks; g.c_scale_rm = 1; g.ldc = 2 * D; g.n_split = 2 * D;
        g.ct2 = v16; g.ldc2 = D; g.vamax = vam; g.vamax_rows = Tq;
        RC(prof(m, s, "gemm_mx:qkv", gflops(g),
                (double)M * D + 3.0 * D * D + (M + 3.0 * D) * D / 32.0 + M * 2.0 * D * (1 + 1.0 / 32) + M * 2.0 * D,
                [&] { return launch_gemm8_mx(g, s); }));
      } else {
        RC(mx_gemm("gemm_mx:qkv", xq, xq_s, Lw.qkv_q, Lw.qkv_s, Lw.qkv_b, 3 * D, D, false, qkv, nullptr, ACT_NONE));
      }
    } else {
      GemmArgs g{};
      g.A = xb; g.B = m->ptr(Lw.qkv_w); g.M = M; g.N = 3 * D; g.K = D; g.rows_per_seg = M; g.lda = D;
      g.bias = m->ptr<float>(Lw.qkv_b); g.Ct = qkv; g.ldc = 3 * D; g.zero = zero;
      if (lnfold && l > 0) {
        g.A = x; g.B = m->ptr(Lw.qkv_wf); g.bias = m->ptr<float>(Lw.qkv_bf); g.acol = m->ptr<float>(Lw.qkv_c);
        g.apart = p2; g.apart_nt = nt; g.ln_eps = eps;
      } else {
        RC((launch_layernorm<R, T>(x, m->ptr<float>(Lw.ln1_w), m->ptr<float>(Lw.ln1_b), M, D, eps, ACT_NONE, nullptr,
                                   xb, s)));
      }
      RC(prof(m, s, "gemm:qkv", gflops(g), gbytes<T>(g), [&] { return launch_gemm<T>(g, AMODE_SEG, 1, s); }));
    }
    GemmArgs g{};
    AttnArgs a{};
    a.qkv = qkv; a.out = ctx; a.T = Tq; a.H = D; a.nh = nh; a.ldq = m->ldq;
    a.q_log2 = m->bf();
    a.scale = a.q_log2 ? 0.6931471805599453f : 1.0f;
    if (f8attn) {
      a.qkv = nullptr; a.qk8 = qk8; a.qks = qks; a.v16 = v16; a.vamax = vam;
      if (f8oproj) { a.out = nullptr; a.out_q = cq; a.out_s = cq_s; }
      RC(prof(m, s, "attn_f8", 4.0 * B * (double)Tq * Tq * D,
              (double)B * Tq * (2.0 * D * (1 + 1.0 / 32) + 2.0 * D + (f8oproj ? D * (1 + 1.0 / 32) : 2.0 * D)),
              [&] { return launch_attention_f8(a, B, s); }));
    } else {
      RC(prof(m, s, "attn", 4.0 * B * (double)Tq * Tq * D, (double)B * Tq * 4.0 * D * sizeof(T),
              [&] { return launch_attention<T>(a, B, s); }));
    }
    if (f8oproj) {
      RC(mx_gemm("gemm_mx:oproj", cq, cq_s, Lw.o_q, Lw.o_s, Lw.o_b, D, D, true, nullptr, nullptr, ACT_NONE));
    } else {
      g = GemmArgs{};
      g.A = ctx; g.B = m->ptr(Lw.o_w); g.M = M; g.N = D; g.K = D; g.rows_per_seg = M; g.lda = D;
      g.bias = m->ptr<float>(Lw.o_b); set_resid(g); g.ldc = D; g.zero = zero;
      if (f1fold) g.opart = p1;
      RC(prof(m, s, "gemm:oproj", gflops(g), gbytes<T>(g), [&] { return launch_gemm<T>(g, AMODE_SEG, 1, s); }));
    }
    if (mx) {
      RC(launch_layernorm_mx<R>(x, m->ptr<float>(Lw.ln2_w), m->ptr<float>(Lw.ln2_b), M, D, eps, xq, xq_s, s));
      RC(mx_gemm("gemm_mx:ffn1", xq, xq_s, Lw.f1_q, Lw.f1_s, Lw.f1_b, F, D, false, fq, fq_s, gelu_rounded_act<T>()));
      RC(mx_gemm("gemm_mx:ffn2", fq, fq_s, Lw.f2_q, Lw.f2_s, Lw.f2_b, D, F, true, nullptr, nullptr, ACT_NONE));
      if (l + 1 < c.layers) RC(sink.emit(l + 1, x));
      continue;
    }
    g = GemmArgs{};
    g.A = xb; g.B = m->ptr(Lw.f1_w); g.M = M; g.N = F; g.K = D; g.rows_per_seg = M; g.lda = D;
    g.bias = m->ptr<float>(Lw.f1_b); g.Ct = ff; g.ldc = F; g.act = gelu_rounded_act<T>(); g.zero = zero;
    if (f1fold) {
      g.A = x; g.B = m->ptr(Lw.f1_wf); g.bias = m->ptr<float>(Lw.f1_bf); g.acol = m->ptr<float>(Lw.f1_c);
      g.apart = p1; g.apart_nt = nt; g.ln_eps = eps;
    } else {
      RC((launch_layernorm<R, T>(x, m->ptr<float>(Lw.ln2_w), m->ptr<float>(Lw.ln2_b), M, D, eps, ACT_NONE, nullptr,
                                 xb, s)));
    }
    RC(prof(m, s, "gemm:ffn1", gflops(g), gbytes<T>(g), [&] { return launch_gemm<T>(g, AMODE_SEG, 1, s); }));
    g = GemmArgs{};
    g.A = ff; g.B = m->ptr(Lw.f2_w); g.M = M; g.N = D; g.K = F; g.rows_per_seg = M; g.lda = F;
    g.bias = m->ptr<float>(Lw.f2_b); set_resid(g); g.ldc = D; g.zero = zero;
    if (lnfold) g.opart = p2;
    RC(prof(m, s, "gemm:ffn2", gflops(g), gbytes<T>(g), [&] { return launch_gemm<T>(g, AMODE_SEG, 1, s); }));
    if (l + 1 < c.layers) RC(sink.emit(l + 1, x));
  }
  // hidden_states[-1] is the post-LN last_hidden_state (HF/utils/output_capturing.py:268-279)
  float* xf = (float*)(ws + w.xf);
  RC((launch_layernorm<R, T>(x, m->ptr<float>(m->enc_ln_w), m->ptr<float>(m->enc_ln_b), M, D, eps, ACT_NONE, xf,
                             dsink ? xb : (T*)nullptr, s)));
  RC(sink.emit(c.layers, xf));
  if (dsink) RC(whisper_decoder<T>(m, xb, B, *dsink, ws, w, s));
  return 0;
}

// SSE_DTYPE_FP16X3 Whisper encoder: the fp32 path with the encoder layers' GEMMs in
// split-fp16 form (as wavlm_forward_x3): pre-LN LayerNorms write the tripled operands, the attention core
// (fp32 softmax, f16 matrix-core products of split operands) writes the out-projection's tripled operand,
// fc1's epilogue the fc2 operand with erf-GELU; log-mel, conv1 / conv2 (exact-f32 MFMA, 0.7 % of the FLOPs),
// the residual stream and the 1-token decoder stay fp32.
int whisper_forward_x3(sse_model* m, const float* wave, int B, int L, const Sink& sink, char* ws, hipStream_t s,
                       const float* mel_hf, const Sink* dsink, const int* lens) {
  const sse_cfg& c = m->cfg;
  Plan p;
  const WhisperWs w = whisper_plan(m, B, p);
  const int D = c.hidden, F = c.ffn, nh = c.heads, Tq = c.max_positions, T2 = 2 * Tq, nm = c.n_mels;
  const int M = B * Tq;
  const float eps = c.ln_eps;
  void* zero = ws + w.zero;
  if (hipMemsetAsync(zero, 0, 256, s) != hipSuccess) return SSE_ERR_HIP;
  float* mel = (float*)(ws + w.mel);
  if (mel_hf)
    RC(launch_mel_to_cl<float>(mel_hf, B, nm, mel, s));
  else
    RC(prof(m, s, "logmel", B * 3000.0 * 5.0 * 200 * 7.64, (double)B * (480000.0 * 4 + 3000.0 * nm * 12.0),
            [&] { return launch_logmel<float>(wave, B, L, nm, nullptr, mel, ws + w.lm, logmel_workspace_bytes(B, nm), s,
                                              lens); }));
  float* h1 = (float*)(ws + w.h1);
  float* x = (float*)(ws + w.x);
  f16* xb = (f16*)(ws + w.xb);
  {
    GemmArgs g{};   // conv1: k3 pad1, 80 -> D, GELU
    g.A = mel; g.B = m->ptr(m->c1_w); g.M = B * T2; g.N = D; g.K = 3 * nm;
    g.rows_per_seg = T2; g.T_in = T2; g.stride = 1; g.pad = 1; g.cin = nm; g.ld_in = nm;
    g.bias = m->ptr<float>(m->c1_b); g.Cf = h1; g.ldc = D; g.act = ACT_GELU; g.zero = zero;
    RC(prof(m, s, "gemm_conv:conv1", gflops(g), gbytes<float>(g, AMODE_CONV),
            [&] { return launch_gemm<float>(g, AMODE_CONV, 1, s); }));
    g = GemmArgs{};   // conv2: k3 s2 pad1, GELU, + embed_positions
    g.A = h1; g.B = m->ptr(m->c2_w); g.M = M; g.N = D; g.K = 3 * D;
    g.rows_per_seg = Tq; g.T_in = T2; g.stride = 2; g.pad = 1; g.cin = D; g.ld_in = D;
    g.bias = m->ptr<float>(m->c2_b); g.resid = m->ptr<float>(m->positions); g.resid_rows = Tq;
    g.Cf = x; g.ldc = D; g.act = ACT_GELU; g.zero = zero;
    RC(prof(m, s, "gemm_conv:conv2", gflops(g), gbytes<float>(g, AMODE_CONV),
            [&] { return launch_gemm<float>(g, AMODE_CONV, 1, s); }));
  }
  RC(sink.emit(0, x));
  float* qkv = (float*)(ws + w.qkv);
  f16* ctx3 = (f16*)(ws + w.ctx);
  f16* ff = (f16*)(ws + w.ff);
  auto gemm3 = [&](const char* tag, GemmArgs& g, int Klog) {   // logical K (the FLOP count), operands 3K
    g.zero = zero;
    g.f16 = 1;
    g.alpha = m->alpha((size_t)((const char*)g.B - m->dmem));
    return prof(m, s, tag, 2.0 * g.M * (double)g.N * Klog, gbytes<bf16>(g), [&] { return launch_gemm8_bf16(g, s); });
  };
  for (int l = 0; l < c.layers; ++l) {
    const LayerW& Lw = m->layers[l];
    RC(launch_layernorm_x3(x, false, m->ptr<float>(Lw.ln1_w), m->ptr<float>(Lw.ln1_b), M, D, eps, nullptr, xb, s));
    GemmArgs g{};
    g.A = xb; g.B = m->ptr(Lw.qkv_w); g.M = M; g.N = 3 * D; g.K = 3 * D; g.rows_per_seg = M; g.lda = 3 * D;
    g.bias = m->ptr<float>(Lw.qkv_b); g.Cf = qkv; g.ldc = 3 * D;
    RC(gemm3("gemm:qkv", g, D));
    AttnArgs a{};
    a.qkv = qkv; a.out = ctx3; a.out3 = 1; a.T = Tq; a.H = D; a.nh = nh; a.ldq = m->ldq; a.scale = 1.0f;
    RC(prof(m, s, "attn", 4.0 * B * (double)Tq * Tq * D, (double)B * Tq * (3.0 * D * 4.0 + 6.0 * D),
            [&] { return launch_attention<float>(a, B, s); }));
    g = GemmArgs{};
    g.A = ctx3; g.B = m->ptr(Lw.o_w); g.M = M; g.N = D; g.K = 3 * D; g.rows_per_seg = M; g.lda = 3 * D;
    g.bias = m->ptr<float>(Lw.o_b); g.resid = x; g.Cf = x; g.ldc = D;
    RC(gemm3("gemm:oproj", g, D));
    RC(launch_layernorm_x3(x, false, m->ptr<float>(Lw.ln2_w), m->ptr<float>(Lw.ln2_b), M, D, eps, nullptr, xb, s));
    g = GemmArgs{};
    g.A = xb; g.B = m->ptr(Lw.f1_w); g.M = M; g.N = F; g.K = 3 * D; g.rows_per_seg = M; g.lda = 3 * D;
    g.bias = m->ptr<float>(Lw.f1_b); g.Ct = ff; g.ct3 = 1; g.ldc = 3 * F; g.act = ACT_GELU;
    RC(gemm3("gemm:ffn1", g, D));
    g = GemmArgs{};
    g.A = ff; g.B = m->ptr(Lw.f2_w); g.M = M; g.N = D; g.K = 3 * F; g.rows_per_seg = M; g.lda = 3 * F;
    g.bias = m->ptr<float>(Lw.f2_b); g.resid = x; g.Cf = x; g.ldc = D;
    RC(gemm3("gemm:ffn2", g, F));
    if (l + 1 < c.layers) RC(sink.emit(l + 1, x));
  }
  // hidden_states[-1] is the post-LN last_hidden_state (HF/utils/output_capturing.py:268-279)
  float* xf = (float*)(ws + w.xf);
  RC((launch_layernorm<float, float>(x, m->ptr<float>(m->enc_ln_w), m->ptr<float>(m->enc_ln_b), M, D, eps, ACT_NONE,
                                     xf, (float*)nullptr, s)));
  RC(sink.emit(c.layers, xf));
  if (dsink) RC(whisper_decoder<float>(m, xf, B, *dsink, ws, w, s));
  return 0;
}

// WavLM embedding batches of at least SPLIT_MIN clips run as two half-batches on two streams (the
// caller's and the model's aux stream): clips are independent, so each half is an ordinary forward
// over its own rows, workspace and output slots, and the two halves' kernels share the CUs -- the last
// partial round of one half's GEMM tiles (447 tiles of the N = 768 residual GEMMs on 256 CUs at B = 256)
// and its latency-bound small kernels are filled with the other half's work.  Bit-identical to the
// single-stream call (every clip's result is independent of the batch it is in).  Not for hidden-state
// calls, Whisper (1500-frame clips already give full rounds) or when OPT_NO_SPLIT is set.
constexpr int SPLIT_MIN = 128;
// parts of a split call: 2 (three or four streams measured slower in rounds 3 and 4)
int split_parts(int) { return 2; }
bool split_applies(const sse_model* m, int B, const Sink* sink) {
  // (Whisper-large-v2 fp8 B = 128 as two streams measured 184.8 vs 178.4 ms/step, round 5: not applied)
  return m->cfg.kind == SSE_KIND_WAVLM && B >= SPLIT_MIN && !sse_opt(OPT_NO_SPLIT) && (!sink || !sink->hs);
}
// clips of part i of P (the first B % P parts one more)
inline int part_size(int B, int P, int i) { return B / P + (i < B % P ? 1 : 0); }
size_t split_ws_bytes(const sse_model* m, int B, int L);
size_t wavlm_ws(const sse_model* m, int B, int L) {
  Plan p;
  if (m->x3()) x3_plan(m, B, L, p); else wavlm_plan(m, B, L, p);
  return p.total;
}

int forward_one(sse_model* m, const float* d_in, int B, int L, const Sink& sink, void* d_ws, hipStream_t s,
                bool from_mel, const Sink* dsink, const int* lens);

int split_forward(sse_model* m, const float* d_in, int B, int L, const Sink& sink, char* ws, hipStream_t s,
                  const int* lens) {
  std::lock_guard<std::mutex> lk(m->split_mu);
  const int P = split_parts(B);
  if (!m->ev_fork && hipEventCreateWithFlags(&m->ev_fork, hipEventDisableTiming) != hipSuccess) {
    m->ev_fork = nullptr;
    return SSE_ERR_HIP;
  }
  for (int i = 0; i < P - 1; ++i) {
    if (!m->aux[i]) {
      if (hipStreamCreateWithFlags(&m->aux[i], hipStreamNonBlocking) != hipSuccess) { m->aux[i] = nullptr; return SSE_ERR_HIP; }
      if (hipEventCreateWithFlags(&m->ev_join[i], hipEventDisableTiming) != hipSuccess) {
        m->ev_join[i] = nullptr;
        return SSE_ERR_HIP;
      }
    }
  }
  // CU-masked halves (A/B option): each half-batch on its own half of the CUs, both forked from and joined to s
  const int mk = P == 2 ? sse_opt(OPT_SPLIT_CUMASK) : 0;
  if (mk && m->mkind != mk) {
    for (int i = 0; i < 2; ++i) {
      if (m->mstream[i]) {
        unregister_mask_stream(m->mstream[i]);
        (void)hipStreamDestroy(m->mstream[i]);
        m->mstream[i] = nullptr;
      }
      if (!m->mjoin[i] && hipEventCreateWithFlags(&m->mjoin[i], hipEventDisableTiming) != hipSuccess) {
        m->mjoin[i] = nullptr;
        return SSE_ERR_HIP;
      }
    }
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, m->device) != hipSuccess || n <= 0 || n > 1024)
      return SSE_ERR_HIP;
    for (int i = 0; i < 2; ++i) {
      std::vector<uint32_t> mask((n + 31) / 32, 0u);
      int cnt = 0;
      for (int c = 0; c < n; ++c) {
        const bool mine = mk == 1 ? ((c < n / 2) == (i == 0)) : ((c & 1) == i);
        if (mine) {
          mask[c >> 5] |= 1u << (c & 31);
          ++cnt;
        }
      }
      if (hipExtStreamCreateWithCUMask(&m->mstream[i], (uint32_t)mask.size(), mask.data()) != hipSuccess) {
        m->mstream[i] = nullptr;
        return SSE_ERR_HIP;
      }
      register_mask_stream(m->mstream[i], cnt);
    }
    m->mkind = mk;
  }
  if (hipEventRecord(m->ev_fork, s) != hipSuccess) return SSE_ERR_HIP;
  int rc = 0, b0 = 0;
  size_t off = 0;
  for (int i = 0; i < P; ++i) {
    const int Bi = part_size(B, P, i);
    hipStream_t si = mk ? m->mstream[i] : (i ? m->aux[i - 1] : s);
    if ((i || mk) && hipStreamWaitEvent(si, m->ev_fork, 0) != hipSuccess) return SSE_ERR_HIP;
    Sink sk = sink;
    sk.B = Bi;
    sk.pooled = sink.pooled + (size_t)b0 * sink.n_ids * sink.H;
    sk.s = si;
    const int r = forward_one(m, d_in + (size_t)b0 * L, Bi, L, sk, ws + off, si, false, nullptr, lens ? lens + b0 : nullptr);
    rc = rc ? rc : r;
    off += (wavlm_ws(m, Bi, L) + 255) & ~(size_t)255;
    b0 += Bi;
  }
  // the joins are recorded whatever happened, so the caller's stream never runs ahead of aux work
  if (mk) {
    for (int i = 0; i < 2; ++i)
      if (hipEventRecord(m->mjoin[i], m->mstream[i]) != hipSuccess || hipStreamWaitEvent(s, m->mjoin[i], 0) != hipSuccess)
        return SSE_ERR_HIP;
    return rc;
  }
  for (int i = 0; i < P - 1; ++i)
    if (hipEventRecord(m->ev_join[i], m->aux[i]) != hipSuccess || hipStreamWaitEvent(s, m->ev_join[i], 0) != hipSuccess)
      return SSE_ERR_HIP;
  return rc;
}

size_t split_ws_bytes(const sse_model* m, int B, int L) {
  const int P = split_parts(B);
  size_t t = 0;
  for (int i = 0; i < P; ++i) t += (wavlm_ws(m, part_size(B, P, i), L) + 255) & ~(size_t)255;
  return t;
}

int forward_any(sse_model* m, const float* d_in, int B, int L, const Sink& sink, void* d_ws, size_t ws_bytes,
                hipStream_t s, bool from_mel, const Sink* dsink, const int* lens);

// fp16-range dtypes: every value the call wrote is scanned and the handle's range flag raised on a
// non-finite one (sse_check_range reports it)
int forward(sse_model* m, const float* d_in, int B, int L, const Sink& sink, void* d_ws, size_t ws_bytes,
            hipStream_t s, bool from_mel = false, const Sink* dsink = nullptr, const int* lens = nullptr) {
  const int rc = forward_any(m, d_in, B, L, sink, d_ws, ws_bytes, s, from_mel, dsink, lens);
  if (rc || !(m->h16() || m->x3())) return rc;
  int* flag = (int*)(m->dmem + m->status);
  if (sink.pooled) RC(launch_finite_flag(sink.pooled, (long long)B * sink.n_ids * sink.H, flag, s));
  if (sink.hs) RC(launch_finite_flag(sink.hs, (long long)(m->cfg.layers + 1) * B * sink.T * sink.H, flag, s));
  return 0;
}

int forward_any(sse_model* m, const float* d_in, int B, int L, const Sink& sink, void* d_ws, size_t ws_bytes,
                hipStream_t s, bool from_mel, const Sink* dsink, const int* lens) {
  if (!m || !d_in || B <= 0 || L <= 0) return SSE_ERR_INVALID;
  if (ws_bytes < sse_workspace_bytes(m, B, L)) return SSE_ERR_WORKSPACE;
  if (!from_mel && !dsink && split_applies(m, B, &sink)) {
    if (wavlm_frames(m->cfg, L, nullptr) <= 0) return SSE_ERR_INVALID;
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess) return SSE_ERR_HIP;
    if (dev != m->device && hipSetDevice(m->device) != hipSuccess) return SSE_ERR_HIP;
    const int rc = split_forward(m, d_in, B, L, sink, (char*)d_ws, s, lens);
    if (dev != m->device) (void)hipSetDevice(dev);
    return rc;
  }
  return forward_one(m, d_in, B, L, sink, d_ws, s, from_mel, dsink, lens);
}

int forward_one(sse_model* m, const float* d_in, int B, int L, const Sink& sink, void* d_ws, hipStream_t s,
                bool from_mel, const Sink* dsink, const int* lens) {
  if (m->cfg.kind == SSE_KIND_WAVLM && wavlm_frames(m->cfg, L, nullptr) <= 0) return SSE_ERR_INVALID;
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) return SSE_ERR_HIP;
  if (dev != m->device && hipSetDevice(m->device) != hipSuccess) return SSE_ERR_HIP;
  int rc;
  if (m->cfg.kind == SSE_KIND_WAVLM && m->x3())
    rc = wavlm_forward_x3(m, d_in, B, L, sink, (char*)d_ws, s, lens);
  else if (m->cfg.kind == SSE_KIND_WAVLM)
    rc = m->bf()    ? wavlm_forward<bf16>(m, d_in, B, L, sink, (char*)d_ws, s, lens)
         : m->h16() ? wavlm_forward<f16>(m, d_in, B, L, sink, (char*)d_ws, s, lens)
                    : wavlm_forward<float>(m, d_in, B, L, sink, (char*)d_ws, s, lens);
  else if (m->x3())
    rc = whisper_forward_x3(m, d_in, B, L, sink, (char*)d_ws, s, from_mel ? d_in : nullptr, dsink, lens);
  else
    rc = m->bf() ? whisper_forward<bf16>(m, d_in, B, L, sink, (char*)d_ws, s, from_mel ? d_in : nullptr, dsink, lens)
                 : whisper_forward<float>(m, d_in, B, L, sink, (char*)d_ws, s, from_mel ? d_in : nullptr, dsink, lens);
  if (dev != m->device) (void)hipSetDevice(dev);
  return rc;
}

int hs_frames(const sse_model* m, int L) {
  return m->cfg.kind == SSE_KIND_WAVLM ? wavlm_frames(m->cfg, L, nullptr) : m->cfg.max_positions;
}

}  // namespace

// ======================================= C-ABI ==========================================
extern "C" {

const char* sse_version(void) { return SSE_VERSION; }

int sse_set_option(const char* name, int value) {
  for (int i = 0; name && i < OPT_COUNT; ++i)
    if (!std::strcmp(name, g_opt_name[i]))
      return value < 0 || value > g_opt_max[i] ? SSE_ERR_INVALID : __atomic_exchange_n(&g_opt[i], value, __ATOMIC_RELAXED);
  return SSE_ERR_INVALID;
}

int sse_get_option(const char* name) {
  for (int i = 0; name && i < OPT_COUNT; ++i)
    if (!std::strcmp(name, g_opt_name[i])) return sse_opt(i);
  return SSE_ERR_INVALID;
}

const char* sse_strerror(int err) {
  switch (err) {
    case SSE_OK: return "ok";
    case SSE_ERR_INVALID: return "invalid argument";
    case SSE_ERR_HIP: return "HIP runtime error";
    case SSE_ERR_UNSUPPORTED: return "unsupported shape";
    case SSE_ERR_WORKSPACE: return "workspace too small";
    case SSE_ERR_WEIGHTS: return "weight blob size does not match the config";
    case SSE_ERR_OOM: return "HIP out of memory";
    case SSE_ERR_RANGE: return "non-finite output: an fp16 activation overflowed (|x| >= 65504)";
    default: return "unknown error";
  }
}

int sse_rel_bucket(int d, int num_buckets, int max_distance) { return rel_bucket(d, num_buckets, max_distance); }

int sse_mel_filters(int n_mels, float* out) {
  if (n_mels <= 0 || !out) return SSE_ERR_INVALID;
  auto h2m = [](double f) { return f >= 1000.0 ? 15.0 + std::log(f / 1000.0) * (27.0 / std::log(6.4)) : 3.0 * f / 200.0; };
  auto m2h = [](double m) { return m >= 15.0 ? 1000.0 * std::exp((std::log(6.4) / 27.0) * (m - 15.0)) : 200.0 * m / 3.0; };
  const int NF = 201;
  const double mmin = h2m(0.0), mmax = h2m(8000.0), step = (mmax - mmin) / (n_mels + 1);
  for (int f = 0; f < NF; ++f)
    for (int m = 0; m < n_mels; ++m) {
      const double f0 = m2h(mmin + step * m), f1 = m2h(mmin + step * (m + 1)), f2 = m2h(mmin + step * (m + 2));
      const double ff = 8000.0 * f / (NF - 1);
      double v = std::fmin((ff - f0) / (f1 - f0), (f2 - ff) / (f2 - f1));
      v = v > 0.0 ? v : 0.0;
      out[f * n_mels + m] = (float)(v * (2.0 / (f2 - f0)));
    }
  return SSE_OK;
}

size_t sse_weight_floats(const sse_cfg* cfg) {
  if (!cfg_valid(cfg)) return 0;
  sse_model tmp{};
  tmp.cfg = *cfg;
  Blob bl{nullptr, (size_t)-1};
  Arena ar;
  const int rc = cfg->kind == SSE_KIND_WAVLM ? build_wavlm(&tmp, bl, ar) : build_whisper(&tmp, bl, ar);
  return rc == SSE_OK ? bl.off : 0;
}

int sse_model_create(const sse_cfg* cfg, const float* host_weights, size_t nbytes, int device, int dtype,
                     sse_model** out) {
  if (!out || !host_weights || !cfg_valid(cfg) ||
      (dtype != SSE_DTYPE_F32 && dtype != SSE_DTYPE_BF16 && dtype != SSE_DTYPE_FP8 && dtype != SSE_DTYPE_FP16X3 &&
       dtype != SSE_DTYPE_FP16))
    return SSE_ERR_INVALID;
  // fp16: WavLM whose every GEMM fits the 8-phase kernels and whose positional conv has 48- or 64-channel
  // groups (the dedicated kernel; WavLM-base / -large) -- the grouped-GEMM fallback has no fp16 form
  if (dtype == SSE_DTYPE_FP16 &&
      (cfg->kind != SSE_KIND_WAVLM || cfg->hidden % 256 || cfg->ffn % 256 ||
       (cfg->hidden / cfg->pos_groups != 48 && cfg->hidden / cfg->pos_groups != 64)))
    return SSE_ERR_UNSUPPORTED;
  // split-fp16: WavLM-base ("group" frontend, post-LN), WavLM-large ("layer" frontend, stable-LN) and the
  // Whisper encoder; every split GEMM N % 256 == 0
  if (dtype == SSE_DTYPE_FP16X3 && (cfg->hidden % 256 || cfg->ffn % 256 ||
                                    (cfg->kind == SSE_KIND_WAVLM ? cfg->conv_dim[0] != 512 : cfg->kind != SSE_KIND_WHISPER)))
    return SSE_ERR_UNSUPPORTED;
  // MX-fp8 GEMMs: N % 256 and K % 128 for QKV (3D x D), fc1 (F x D), fc2 (D x F)
  if (dtype == SSE_DTYPE_FP8 && (cfg->kind != SSE_KIND_WHISPER || cfg->hidden % 256 || cfg->ffn % 256))
    return SSE_ERR_UNSUPPORTED;
  *out = nullptr;
  const size_t need = sse_weight_floats(cfg);
  if (need == 0 || nbytes != need * 4) return SSE_ERR_WEIGHTS;
  sse_model* m = new (std::nothrow) sse_model();
  if (!m) return SSE_ERR_OOM;
  m->cfg = *cfg;
  m->device = device;
  m->dtype = dtype;
  Blob bl{host_weights, need};
  Arena ar;
  const int rc = cfg->kind == SSE_KIND_WAVLM ? build_wavlm(m, bl, ar) : build_whisper(m, bl, ar);
  if (rc != SSE_OK || bl.off != need) { delete m; return SSE_ERR_WEIGHTS; }
  m->zero = ar.put(nullptr, 256);
  m->status = ar.put(nullptr, 256);
  m->x3_alpha = ar.alpha;
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) { delete m; return SSE_ERR_HIP; }
  m->dbytes = ar.size;
  if (hipMalloc((void**)&m->dmem, ar.size) != hipSuccess) {
    (void)hipSetDevice(prev);
    delete m;
    return SSE_ERR_OOM;
  }
  std::vector<char> staging(ar.size, 0);
  for (auto& pr : ar.pending) std::memcpy(staging.data() + pr.first, pr.second.data(), pr.second.size());
  const bool okc = hipMemcpy(m->dmem, staging.data(), ar.size, hipMemcpyHostToDevice) == hipSuccess;
  (void)hipSetDevice(prev);
  if (!okc) { (void)hipFree(m->dmem); delete m; return SSE_ERR_HIP; }
  *out = m;
  return SSE_OK;
}

void sse_model_destroy(sse_model* m) {
  if (!m) return;
  for (auto e : m->prof.ev) (void)hipEventDestroy(e);
  if (m->ev_fork) (void)hipEventDestroy(m->ev_fork);
  for (int i = 0; i < sse_model::MAX_PARTS - 1; ++i) {
    if (m->ev_join[i]) (void)hipEventDestroy(m->ev_join[i]);
    if (m->aux[i]) (void)hipStreamDestroy(m->aux[i]);
  }
  for (int i = 0; i < 2; ++i) {
    if (m->mjoin[i]) (void)hipEventDestroy(m->mjoin[i]);
    if (m->mstream[i]) {
      unregister_mask_stream(m->mstream[i]);
      (void)hipStreamDestroy(m->mstream[i]);
    }
  }
  if (m->dmem) {
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(m->device);
    (void)hipFree(m->dmem);
    (void)hipSetDevice(prev);
  }
  delete m;
}

int sse_output_frames(const sse_model* m, int L) {
  if (!m || L <= 0) return SSE_ERR_INVALID;
  return hs_frames(m, L);
}

size_t sse_workspace_bytes(const sse_model* m, int B, int L) {
  if (!m || B <= 0 || L <= 0) return 0;
  Plan p;
  if (m->cfg.kind == SSE_KIND_WAVLM) {
    if (wavlm_frames(m->cfg, L, nullptr) <= 0) return 0;
    const size_t one = wavlm_ws(m, B, L);
    if (split_applies(m, B, nullptr)) {   // the parts' workspaces (split_forward); also covers one stream
      const size_t parts = split_ws_bytes(m, B, L);
      return parts > one ? parts : one;
    }
    return one;
  } else {
    whisper_plan(m, B, p);
  }
  return p.total;
}

size_t sse_logmel_workspace_bytes(int B, int n_mels) { return logmel_workspace_bytes(B, n_mels); }

int sse_logmel(const float* d_wave, int B, int L, int n_mels, float* d_mel, void* d_ws, size_t ws_bytes,
               void* stream) {
  if (!d_wave || !d_mel || !d_ws) return SSE_ERR_INVALID;
  return launch_logmel<float>(d_wave, B, L, n_mels, d_mel, (float*)nullptr, d_ws, ws_bytes, (hipStream_t)stream);
}

int sse_check_range(sse_model* m, void* stream) {
  if (!m) return SSE_ERR_INVALID;
  if (!(m->h16() || m->x3())) return SSE_OK;
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(m->device) != hipSuccess) return SSE_ERR_HIP;
  int v = 0;
  int* flag = (int*)(m->dmem + m->status);
  bool ok = hipStreamSynchronize((hipStream_t)stream) == hipSuccess &&
            hipMemcpy(&v, flag, sizeof(int), hipMemcpyDeviceToHost) == hipSuccess;
  if (ok && v) ok = hipMemset(flag, 0, sizeof(int)) == hipSuccess;
  (void)hipSetDevice(prev);
  if (!ok) return SSE_ERR_HIP;
  return v ? SSE_ERR_RANGE : SSE_OK;
}

int sse_embed(sse_model* m, const float* d_in, int B, int L, const int32_t* layer_ids, int n_layers, float* d_out,
              void* d_ws, size_t ws_bytes, void* stream) {
  if (!m || !layer_ids || n_layers <= 0 || !d_out) return SSE_ERR_INVALID;
  for (int i = 0; i < n_layers; ++i)
    if (layer_ids[i] < 0 || layer_ids[i] > m->cfg.layers) return SSE_ERR_INVALID;
  Sink sk{layer_ids, n_layers, d_out, nullptr, B, hs_frames(m, L), m->cfg.hidden, (hipStream_t)stream};
  return forward(m, d_in, B, L, sk, d_ws, ws_bytes, (hipStream_t)stream);
}

int sse_embed_ragged(sse_model* m, const float* d_in, const int32_t* d_lengths, int B, int L, const int32_t* layer_ids,
                     int n_layers, float* d_out, void* d_ws, size_t ws_bytes, void* stream) {
  if (!m || !d_lengths || !layer_ids || n_layers <= 0 || !d_out) return SSE_ERR_INVALID;
  for (int i = 0; i < n_layers; ++i)
    if (layer_ids[i] < 0 || layer_ids[i] > m->cfg.layers) return SSE_ERR_INVALID;
  Sink sk{layer_ids, n_layers, d_out, nullptr, B, hs_frames(m, L), m->cfg.hidden, (hipStream_t)stream};
  return forward(m, d_in, B, L, sk, d_ws, ws_bytes, (hipStream_t)stream, false, nullptr, (const int*)d_lengths);
}

int sse_hidden_states(sse_model* m, const float* d_in, int B, int L, float* d_hs, void* d_ws, size_t ws_bytes,
                      void* stream) {
  if (!m || !d_hs) return SSE_ERR_INVALID;
  Sink sk{nullptr, 0, nullptr, d_hs, B, hs_frames(m, L), m->cfg.hidden, (hipStream_t)stream};
  return forward(m, d_in, B, L, sk, d_ws, ws_bytes, (hipStream_t)stream);
}

int sse_whisper_hidden_states_from_mel(sse_model* m, const float* d_mel, int B, float* d_hs, void* d_ws,
                                       size_t ws_bytes, void* stream) {
  if (!m || !d_hs || m->cfg.kind != SSE_KIND_WHISPER) return SSE_ERR_INVALID;
  Sink sk{nullptr, 0, nullptr, d_hs, B, m->cfg.max_positions, m->cfg.hidden, (hipStream_t)stream};
  return forward(m, d_mel, B, 2 * m->cfg.max_positions, sk, d_ws, ws_bytes, (hipStream_t)stream, true);
}

int sse_whisper_embed(sse_model* m, const float* d_wave, int B, int L, const int32_t* enc_ids, int n_enc,
                      float* d_enc_out, const int32_t* dec_ids, int n_dec, float* d_dec_out, void* d_ws,
                      size_t ws_bytes, void* stream) {
  if (!m || m->cfg.kind != SSE_KIND_WHISPER || n_enc < 0 || n_dec < 0 || (n_enc && (!enc_ids || !d_enc_out)) ||
      (n_dec && (!dec_ids || !d_dec_out)) || (n_dec && m->cfg.decoder_layers <= 0))
    return SSE_ERR_INVALID;
  for (int i = 0; i < n_enc; ++i)
    if (enc_ids[i] < 0 || enc_ids[i] > m->cfg.layers) return SSE_ERR_INVALID;
  for (int i = 0; i < n_dec; ++i)
    if (dec_ids[i] < 0 || dec_ids[i] > m->cfg.decoder_layers) return SSE_ERR_INVALID;
  Sink sk{enc_ids, n_enc, d_enc_out, nullptr, B, m->cfg.max_positions, m->cfg.hidden, (hipStream_t)stream};
  Sink dk{dec_ids, n_dec, d_dec_out, nullptr, B, 1, m->cfg.hidden, (hipStream_t)stream};
  return forward(m, d_wave, B, L, sk, d_ws, ws_bytes, (hipStream_t)stream, false, n_dec ? &dk : nullptr);
}

int sse_whisper_decoder_hidden_states(sse_model* m, const float* d_enc, int B, float* d_hs, void* d_ws,
                                      size_t ws_bytes, void* stream) {
  if (!m || !d_enc || !d_hs || B <= 0 || m->cfg.kind != SSE_KIND_WHISPER || m->cfg.decoder_layers <= 0)
    return SSE_ERR_INVALID;
  if (ws_bytes < sse_workspace_bytes(m, B, 2 * m->cfg.max_positions)) return SSE_ERR_WORKSPACE;
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) return SSE_ERR_HIP;
  if (dev != m->device && hipSetDevice(m->device) != hipSuccess) return SSE_ERR_HIP;
  hipStream_t s = (hipStream_t)stream;
  Plan p;
  const WhisperWs w = whisper_plan(m, B, p);
  char* ws = (char*)d_ws;
  Sink dk{nullptr, 0, nullptr, d_hs, B, 1, m->cfg.hidden, s};
  const long long n = (long long)B * m->cfg.max_positions * m->cfg.hidden;
  int rc = hipMemsetAsync(ws + w.zero, 0, 256, s) == hipSuccess ? 0 : SSE_ERR_HIP;
  if (!rc) {
    if (m->bf()) {
      rc = launch_cast<bf16>(d_enc, n, (bf16*)(ws + w.xb), s);
      if (!rc) rc = whisper_decoder<bf16>(m, (const bf16*)(ws + w.xb), B, dk, ws, w, s);
    } else {
      rc = whisper_decoder<float>(m, d_enc, B, dk, ws, w, s);
    }
  }
  if (dev != m->device) (void)hipSetDevice(dev);
  return rc;
}

int sse_profile_start(sse_model* m, int max_launches) {
  if (!m || max_launches <= 0) return SSE_ERR_INVALID;
  auto& P = m->prof;
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(m->device) != hipSuccess) return SSE_ERR_HIP;
  while ((int)P.ev.size() < 2 * max_launches) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) { (void)hipSetDevice(prev); return SSE_ERR_HIP; }
    P.ev.push_back(e);
  }
  (void)hipSetDevice(prev);
  P.on = true;
  P.used = 0;
  P.tag.clear(); P.flops.clear(); P.bytes.clear();
  return SSE_OK;
}

int sse_profile_read(sse_model* m, int cap, char* tags, float* ms, double* flops, double* bytes) {
  if (!m || cap < 0) return SSE_ERR_INVALID;
  auto& P = m->prof;
  const int n = (int)P.tag.size();
  // launches may sit on two streams (split_forward): wait for every recorded end event
  for (int i = 0; i < n; ++i)
    if (hipEventSynchronize(P.ev[2 * i + 1]) != hipSuccess) return SSE_ERR_HIP;
  for (int i = 0; i < n && i < cap; ++i) {
    float t = 0.f;
    if (hipEventElapsedTime(&t, P.ev[2 * i], P.ev[2 * i + 1]) != hipSuccess) return SSE_ERR_HIP;
    if (ms) ms[i] = t;
    if (flops) flops[i] = P.flops[i];
    if (bytes) bytes[i] = P.bytes[i];
    if (tags) { std::strncpy(tags + 32 * i, P.tag[i].c_str(), 31); tags[32 * i + 31] = 0; }
  }
  P.used = 0;
  P.tag.clear(); P.flops.clear(); P.bytes.clear();
  return n;
}

int sse_profile_stop(sse_model* m) {
  if (!m) return SSE_ERR_INVALID;
  m->prof.on = false;
  m->prof.used = 0;
  m->prof.tag.clear(); m->prof.flops.clear(); m->prof.bytes.clear();
  return SSE_OK;
}

size_t sse_normalize_workspace_bytes(int B) { return (size_t)B * 8; }

int sse_resample_length(int L, int orig_freq, int new_freq) {
  if (L <= 0 || orig_freq <= 0 || new_freq <= 0) return SSE_ERR_INVALID;
  return orig_freq == new_freq ? L : resample_length(L, orig_freq, new_freq);
}

size_t sse_resample_workspace_bytes(int B, int L, int orig_freq, int new_freq) {
  if (B <= 0 || L <= 0 || orig_freq <= 0 || new_freq <= 0) return 0;
  return orig_freq == new_freq ? 256 : resample_workspace_bytes(B, L, orig_freq, new_freq);
}

int sse_resample(const float* d_in, int B, int L, int orig_freq, int new_freq, float* d_out, void* d_ws,
                 size_t ws_bytes, void* stream) {
  if (!d_in || !d_out || !d_ws) return SSE_ERR_INVALID;
  const int rc = launch_resample(d_in, B, L, orig_freq, new_freq, d_out, d_ws, ws_bytes, (hipStream_t)stream);
  return rc == -4 ? SSE_ERR_WORKSPACE : (rc == -1 ? SSE_ERR_INVALID : (rc ? SSE_ERR_HIP : SSE_OK));
}

int sse_augment(const float* d_in, float* d_out, int B, int L, const int32_t* d_kind, const float* d_factor,
                const int64_t* d_stream, uint64_t seed, void* stream) {
  if (!d_in || !d_out || !d_kind || !d_factor || !d_stream) return SSE_ERR_INVALID;
  const int rc = launch_augment(d_in, d_out, B, L, (const int*)d_kind, d_factor, (const long long*)d_stream, seed,
                                (hipStream_t)stream);
  return rc == -1 ? SSE_ERR_INVALID : (rc ? SSE_ERR_HIP : SSE_OK);
}

size_t sse_pitch_shift_workspace_bytes(int B, int L, int sample_rate, int n_steps) {
  if (B <= 0 || L <= 256 || sample_rate <= 0 || n_steps < -48 || n_steps > 48) return 0;
  return pitch_shift_workspace_bytes(B, L, sample_rate, n_steps);
}

int sse_pitch_shift(const float* d_in, int B, int L, int sample_rate, int n_steps, float* d_out, void* d_ws,
                    size_t ws_bytes, void* stream) {
  if (!d_in || !d_out || !d_ws) return SSE_ERR_INVALID;
  const int rc = launch_pitch_shift(d_in, B, L, sample_rate, n_steps, d_out, d_ws, ws_bytes, (hipStream_t)stream);
  return rc == -4 ? SSE_ERR_WORKSPACE : (rc == -1 ? SSE_ERR_INVALID : (rc ? SSE_ERR_HIP : SSE_OK));
}

int sse_mono(const float* d_in, int B, int C, int L, float* d_out, void* stream) {
  if (!d_in || !d_out) return SSE_ERR_INVALID;
  const int rc = launch_mono(d_in, B, C, L, d_out, (hipStream_t)stream);
  return rc == -1 ? SSE_ERR_INVALID : (rc ? SSE_ERR_HIP : SSE_OK);
}

int sse_attention(const void* d_qkv, void* d_out, int B, int T, int H, int nh, int ldq, float scale, int q_log2,
                  void* stream) {
  if (!d_qkv || !d_out || B <= 0 || T <= 0 || nh <= 0 || H != nh * 64 || ldq < 3 * H || ldq % 8) return SSE_ERR_INVALID;
  // q_log2: the scores are already log2-domain logits, which every kernel reads as scale = ln 2; any other
  // scale would be honoured by the short-T kernels (T <= 160) and ignored by the 32x32 flash kernel
  if (q_log2 && scale != 0.6931471805599453f) return SSE_ERR_INVALID;
  AttnArgs a{};
  a.qkv = d_qkv; a.out = d_out; a.T = T; a.H = H; a.nh = nh; a.ldq = ldq; a.scale = scale; a.q_log2 = q_log2 ? 1 : 0;
  return launch_attention<bf16>(a, B, (hipStream_t)stream) ? SSE_ERR_HIP : SSE_OK;
}

int sse_attention_f8(const uint8_t* d_qk, const uint8_t* d_qk_scale, const void* d_v, const uint32_t* d_vamax,
                     void* d_out, int B, int T, int H, int nh, void* stream) {
  if (!d_qk || !d_qk_scale || !d_v || !d_vamax || !d_out || B <= 0 || T <= 0 || nh <= 0 || H != nh * 64)
    return SSE_ERR_INVALID;
  AttnArgs a{};
  a.out = d_out; a.T = T; a.H = H; a.nh = nh; a.ldq = 2 * H; a.scale = 0.6931471805599453f; a.q_log2 = 1;
  a.qk8 = d_qk; a.qks = d_qk_scale; a.v16 = d_v; a.vamax = d_vamax;
  const int rc = launch_attention_f8(a, B, (hipStream_t)stream);
  return rc == -3 ? SSE_ERR_INVALID : (rc ? SSE_ERR_HIP : SSE_OK);
}

int sse_attention_f8_mx(const uint8_t* d_qk, const uint8_t* d_qk_scale, const void* d_v, const uint32_t* d_vamax,
                        uint8_t* d_out_q, uint8_t* d_out_scale, int B, int T, int H, int nh, void* stream) {
  if (!d_qk || !d_qk_scale || !d_v || !d_vamax || !d_out_q || !d_out_scale || B <= 0 || T <= 0 || nh <= 0 ||
      H != nh * 64 || H % 128)
    return SSE_ERR_INVALID;
  AttnArgs a{};
  a.T = T; a.H = H; a.nh = nh; a.ldq = 2 * H; a.scale = 0.6931471805599453f; a.q_log2 = 1;
  a.qk8 = d_qk; a.qks = d_qk_scale; a.v16 = d_v; a.vamax = d_vamax; a.out_q = d_out_q; a.out_s = d_out_scale;
  const int rc = launch_attention_f8(a, B, (hipStream_t)stream);
  return rc == -3 ? SSE_ERR_INVALID : (rc ? SSE_ERR_HIP : SSE_OK);
}

int sse_gemm(int dtype, const void* d_a, const void* d_b, const float* d_bias, const float* d_resid, float* d_cf,
             void* d_ct, int M, int N, int K, int act, const void* d_zero, void* stream) {
  if (!d_a || !d_b || !d_zero || M <= 0 || N <= 0 || K <= 0 || (!d_cf && !d_ct)) return SSE_ERR_INVALID;
  GemmArgs g{};
  g.A = d_a; g.B = d_b; g.M = M; g.N = N; g.K = K; g.rows_per_seg = M; g.lda = K;
  g.bias = d_bias; g.resid = d_resid; g.Cf = d_cf; g.Ct = d_ct; g.ldc = N; g.act = act; g.zero = d_zero;
  return dtype == SSE_DTYPE_BF16 ? launch_gemm_bf16(g, AMODE_SEG, 1, (hipStream_t)stream)
                                 : launch_gemm_f32(g, AMODE_SEG, 1, (hipStream_t)stream);
}

int sse_gemm_ex(const sse_gemm_desc* d, void* stream) {
  if (!d || !d->a || !d->b || !d->zero || d->M <= 0 || d->N <= 0 || d->K <= 0 || (!d->cf && !d->ct) ||
      d->ldc < (d->n_split ? d->n_split : d->N))
    return SSE_ERR_INVALID;
  if (d->dtype != SSE_DTYPE_BF16 && d->dtype != SSE_DTYPE_FP16 && d->dtype != SSE_DTYPE_F32 && d->dtype != SSE_DTYPE_FP8)
    return SSE_ERR_INVALID;
  if (d->dtype == SSE_DTYPE_FP8) {
    if (!d->a_scale || !d->b_scale || d->ldc != (d->n_split ? d->n_split : d->N) || d->apart || d->rpart || d->opart)
      return SSE_ERR_INVALID;
    if (d->N % 256 || d->K % 128) return SSE_ERR_UNSUPPORTED;
    GemmArgs g{};
    g.A = d->a; g.a_scale = d->a_scale; g.B = d->b; g.b_scale = d->b_scale; g.M = d->M; g.N = d->N; g.K = d->K;
    g.rows_per_seg = d->M; g.lda = d->K; g.bias = d->bias; g.resid = d->resid; g.resid_t = (const bf16*)d->resid_t;
    g.Cf = d->cf; g.Ct = d->ct; g.ldc = d->ldc; g.act = d->act; g.zero = d->zero;
    g.c_scale = d->c_scale; g.c_scale_rm = d->c_scale_rm; g.vamax = d->vamax; g.vamax_rows = d->vamax_rows;
    g.ct2 = d->ct2; g.n_split = d->n_split; g.ldc2 = d->ldc2;
    const int rc = launch_gemm8_mx(g, (hipStream_t)stream);
    return rc == -3 ? SSE_ERR_INVALID : (rc ? SSE_ERR_HIP : SSE_OK);
  }
  if ((d->apart != nullptr) != (d->acol != nullptr) || (d->rpart && (!d->rln_w || !d->rln_b)) ||
      (d->resid && d->resid_t) || (d->rpart && !d->resid && !d->resid_t))
    return SSE_ERR_INVALID;
  GemmArgs g{};
  g.A = d->a; g.B = d->b; g.M = d->M; g.N = d->N; g.K = d->K; g.rows_per_seg = d->M; g.lda = d->K;
  g.bias = d->bias; g.act = d->act; g.Cf = d->cf; g.Ct = d->ct; g.ldc = d->ldc; g.zero = d->zero;
  g.acol = d->acol; g.apart = (const float2*)d->apart; g.apart_nt = d->apart_nt; g.ln_eps = d->ln_eps;
  g.resid = d->resid; g.resid_t = (const bf16*)d->resid_t;
  g.rpart = (const float2*)d->rpart; g.rpart_nt = d->rpart ? 3 : 0; g.rln_w = d->rln_w; g.rln_b = d->rln_b;
  g.opart = (float2*)d->opart;
  hipStream_t s = (hipStream_t)stream;
  const int rc = d->dtype == SSE_DTYPE_BF16   ? launch_gemm<bf16>(g, AMODE_SEG, 1, s)
                 : d->dtype == SSE_DTYPE_FP16 ? launch_gemm<f16>(g, AMODE_SEG, 1, s)
                                              : launch_gemm<float>(g, AMODE_SEG, 1, s);
  return rc == -3 ? SSE_ERR_INVALID : (rc ? SSE_ERR_HIP : SSE_OK);
}

int sse_gemm_lnfold(const void* d_a, const void* d_b, const float* d_bias, const float* d_acol, const float* d_apart,
                    void* d_ct, int M, int N, int K, int act, float eps, const void* d_zero, void* stream) {
  if (!d_a || !d_b || !d_acol || !d_apart || !d_ct || !d_zero || M <= 0 || N <= 0 || K != 768) return SSE_ERR_INVALID;
  GemmArgs g{};
  g.A = d_a; g.B = d_b; g.M = M; g.N = N; g.K = K; g.rows_per_seg = M; g.lda = K;
  g.bias = d_bias; g.Ct = d_ct; g.ldc = N; g.act = act; g.zero = d_zero;
  g.acol = d_acol; g.apart = (const float2*)d_apart; g.apart_nt = 3; g.ln_eps = eps;
  return launch_gemm_bf16(g, AMODE_SEG, 1, (hipStream_t)stream);
}

size_t sse_mx_scale_bytes(int R, int K) {
  if (R <= 0 || K <= 0 || K % 128) return 0;
  return (size_t)mx_scale_bytes(R, K);
}

long long sse_mx_scale_offset(int role, int r, int b, int K) {
  if (r < 0 || b < 0 || K <= 0 || K % 128 || b >= K / 32) return -1;
  return role ? mx_b_scale_off(r, b, K / 128) : mx_a_scale_off(r, b, K / 128);
}

int sse_mx_quantize(const float* d_x, int R, int K, int role, uint8_t* d_q, uint8_t* d_scale, void* stream) {
  if (!d_x || !d_q || !d_scale || R <= 0 || K <= 0 || K % 128 || (role != 0 && role != 1)) return SSE_ERR_INVALID;
  return launch_mx_quantize(d_x, R, K, role, d_q, d_scale, (hipStream_t)stream) ? SSE_ERR_HIP : SSE_OK;
}

int sse_layernorm_mx(const void* d_x, const float* d_w, const float* d_b, int R, int H, float eps, uint8_t* d_q,
                     uint8_t* d_scale, void* stream) {
  if (!d_x || !d_w || !d_b || !d_q || !d_scale || R <= 0 || H <= 0 || H % 128 || H > 2048) return SSE_ERR_INVALID;
  return launch_layernorm_mx<bf16>((const bf16*)d_x, d_w, d_b, R, H, eps, d_q, d_scale, (hipStream_t)stream) ? SSE_ERR_HIP
                                                                                                            : SSE_OK;
}

int sse_mx_quantize_host(const float* x, int R, int K, int role, uint8_t* q, uint8_t* scale) {
  if (!x || !q || !scale || R <= 0 || K <= 0 || K % 128 || (role != 0 && role != 1)) return SSE_ERR_INVALID;
  mx_quantize_rows(x, R, K, role, q, scale);
  return SSE_OK;
}

int sse_gemm_mx(const uint8_t* d_a, const uint8_t* d_a_scale, const uint8_t* d_b, const uint8_t* d_b_scale,
                const float* d_bias, const float* d_resid, float* d_cf, void* d_ct, uint8_t* d_c_scale, int M, int N,
                int K, int act, void* stream) {
  if (!d_a || !d_a_scale || !d_b || !d_b_scale || M <= 0 || N <= 0 || K <= 0 || (!d_cf && !d_ct)) return SSE_ERR_INVALID;
  if (N % 256 || K % 128) return SSE_ERR_UNSUPPORTED;
  if (d_c_scale && (d_cf || !d_ct || d_resid)) return SSE_ERR_INVALID;
  if (d_resid && d_ct) return SSE_ERR_UNSUPPORTED;
  GemmArgs g{};
  g.A = d_a; g.a_scale = d_a_scale; g.B = d_b; g.b_scale = d_b_scale; g.M = M; g.N = N; g.K = K;
  g.rows_per_seg = M; g.lda = K; g.bias = d_bias; g.resid = d_resid; g.Cf = d_cf; g.Ct = d_ct; g.c_scale = d_c_scale;
  g.ldc = N; g.act = act;
  return launch_gemm8_mx(g, (hipStream_t)stream) ? SSE_ERR_HIP : SSE_OK;
}

int sse_normalize(const float* d_in, int B, int L, float* d_out, void* d_ws, size_t ws_bytes, void* stream) {
  if (!d_in || !d_out || !d_ws || B <= 0 || L <= 0) return SSE_ERR_INVALID;
  if (ws_bytes < (size_t)B * 8) return SSE_ERR_WORKSPACE;
  RC(launch_wave_stats(d_in, B, L, (float*)d_ws, (hipStream_t)stream));
  return launch_normalize_apply(d_in, B, L, (const float*)d_ws, d_out, (hipStream_t)stream);
}

}  // extern "C"
