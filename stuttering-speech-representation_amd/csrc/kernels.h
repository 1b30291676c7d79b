// Launcher declarations for kernels_misc.hip (host orchestration in sse_model.hip).
#pragma once
#include "common.h"

// lens (ragged batches, device, optional): samples of each clip [B]; L is the row stride
int launch_wave_stats(const float* x, int B, int L, float* out, hipStream_t s, const int* lens = nullptr);

size_t conv0_moments_bytes(int B);
// t0len (ragged batches, device, optional): conv0 frames of each clip [B] (GroupNorm statistics
// over the clip's own frames); T0 is the row stride
template <typename TO>
int launch_conv0_gn(const float* x, int B, int L, const float* norm, const float* w0, const float* b0, int C,
                    int k0, int s0, int T0, const float* gamma, const float* beta, float eps, double* mom,
                    float2* ss, TO* out, hipStream_t s, const int* t0len = nullptr);

// ragged batches: per-clip frame counts after each conv layer, from the sample counts
struct ClipFrames {
  int n_conv, kernel[8], stride[8];
};
// L: the batch's row length in samples (lengths are clamped to [0, L] on the device)
int launch_clip_frames(const int* lens, int B, int L, ClipFrames cf, int* t0, int* tf, hipStream_t s);
// zero rows t >= tlen[b] of x [B][T][H] (ragged batches: the padded positional conv must read zeros)
template <typename TE>
int launch_mask_rows(TE* x, int B, int T, int H, const int* tlen, hipStream_t s);

template <typename TO>
int launch_conv0_ln(const float* x, int B, int L, const float* norm, const float* w0, const float* b0, int C, int k0,
                    int s0, int T0, const float* lnw, const float* lnb, float eps, TO* out, hipStream_t s);

template <typename TO>
int launch_conv0_raw(const float* x, int B, int L, const float* norm, const float* w0, const float* b0, int C,
                     int k0, int s0, int T0, TO* out, hipStream_t s);

template <typename TI, typename TO>
int launch_layernorm(const TI* in, const float* w, const float* b, int rows, int H, float eps, int act,
                     float* out_f, TO* out_t, hipStream_t s, float2* stats = nullptr);

// split-fp16 (SSE_DTYPE_FP16X3) operands: tripled rows [hi | lo' | hi] (common.h x3_split4)
// act: ACT_NONE or ACT_GELU (erf, fp32 input only: the "layer" conv frontend's LN + GELU)
int launch_layernorm_x3(const void* in, bool in3, const float* w, const float* b, int rows, int H, float eps,
                        float* out_f, f16* out3, hipStream_t s, int act = ACT_NONE);
int launch_split3(const float* x, long long rows, int C, f16* y, hipStream_t s);
int launch_conv0_ln_x3(const float* x, int B, int L, const float* norm, const float* w0, const float* b0, int C,
                       int k0, int s0, int T0, const float* lnw, const float* lnb, float eps, f16* out3, hipStream_t s);
int launch_conv0_gn_x3(const float* x, int B, int L, const float* norm, const float* w0, const float* b0, int C,
                       int k0, int s0, int T0, const float* gamma, const float* beta, float eps, double* mom,
                       float2* ss, f16* out3, hipStream_t s, const int* t0len);

// MX-fp8 (e4m3 + E8M0 per 32 K-elements) GEMM operands, layouts in common.h
template <typename TI>
int launch_layernorm_mx(const TI* in, const float* w, const float* b, int rows, int H, float eps,
                        unsigned char* q, unsigned char* scale, hipStream_t s);
int launch_mx_quantize(const float* x, int R, int K, int role, unsigned char* q, unsigned char* scale, hipStream_t s);

// kernels_posconv.hip: WavLM positional conv (bf16 path); -3 = shape not covered (use the GEMM)
// split-fp16 positional conv (SSE_DTYPE_FP16X3): fp32 xt / x, W = planes [wh][wl] of w / alpha
int launch_posconv_x3(const float* xt, const f16* W, float alpha, const float* bias, float* x, int B, int T, int H,
                      int G, int K, int pad, hipStream_t s);
int launch_posconv_bf16(const bf16* xt, const bf16* W, const float* bias, float* x, int B, int T, int H, int G, int K,
                        int pad, hipStream_t s, bool h16 = false);   // h16: xt / W are fp16

// st: per-row (mean, rstd), or part: per-256-column partials [rows][nt] (ln_part_stats): each element
// is LayerNorm'd with (w, b) before the mean.  tlen (ragged batches): the mean runs over each clip's
// own frames; T is the row stride.
template <typename TI>
int launch_pool_mean(const TI* x, int B, int T, int H, float* out, long long out_stride, hipStream_t s,
                     const float2* st = nullptr, const float* w = nullptr, const float* b = nullptr,
                     const float2* part = nullptr, int nt = 0, float eps = 0.f, const int* tlen = nullptr);

struct AttnArgs {
  const void* qkv;       // [B*T][ldq]  (q | k | v | WavLM gate projection | pad), element type T
  void* out;             // [B*T][H]
  int T, H, nh, ldq;
  float scale;           // applied to q.k (WavLM 1/sqrt(d); Whisper 1, q pre-scaled in weights)
  // WavLM gated relative-position bias (null for Whisper): the QKV GEMM also produced the
  // per-head gru_rel_pos_linear outputs rp[t][h][0..7] at column 3H + 8h (bias included)
  const float* gconst;   // [nh]
  const float* relb;     // [nh][2*maxd+1], index d + maxd
  int maxd;
  const int* tlen;       // ragged batch: frames of each clip [B] (T is then the per-clip row stride)
  int min_t;             // flash kernel: clips of at most min_t frames are skipped (ragged batches whose
                         // short clips run on the short-T kernel, exactly as when run alone)
  int q_log2;            // q carries scale * log2(e) (Whisper bf16 / fp8 encoder): scale = ln 2, and the
                         // flash3 kernel (which requires it) takes the scores as log2-domain logits
  int out3;              // fp32 kernel: write the output tripled for a split-fp16 GEMM ([hi | lo' | hi],
                         // rows of 3H fp16, x3_split4) instead of fp32 (SSE_DTYPE_FP16X3)
  // fp8 Whisper attention (launch_attention_f8; qkv unused): Q | K MX-fp8 [B*T][2H] bytes (q carries
  // scale * log2 e: q_log2), their E8M0 scales row-major [B*T][2H / 32]; V bf16 [B*T][H]; vamax [B][H]
  // the float bits of max |V| per (clip, column) (the V GEMM's GemmArgs::vamax)
  const unsigned char* qk8;
  const unsigned char* qks;
  const void* v16;
  const unsigned* vamax;
  // fp8 attention, optional MX-fp8 output instead of bf16 `out` (round 6: the out-projection's A operand):
  // e4m3 [B*T][H] and E8M0 scales in the MX GEMM's A layout for K = H (mx_a_scale_off)
  unsigned char* out_q;
  unsigned char* out_s;
};
int launch_attention_f8(const AttnArgs& a, int B, hipStream_t s);
template <typename T>
int launch_attention(const AttnArgs& a, int B, hipStream_t s);

template <typename TE>
int launch_xattn1(const TE* q, const TE* kv, int B, int T, int D, int nh, TE* out, hipStream_t s);
int launch_bcast_rows(const float* v, int D, int B, float* out, hipStream_t s);
int launch_finite_flag(const float* x, long long n, int* flag, hipStream_t s);   // sse_check_range
template <typename TO, typename TI = float>
int launch_cast(const TI* x, long long n, TO* y, hipStream_t s);

// kernels_ingest.hip
int resample_length(int L, int orig_freq, int new_freq);
size_t resample_workspace_bytes(int B, int L, int orig_freq, int new_freq);
int launch_resample(const float* x, int B, int L, int orig_freq, int new_freq, float* y, void* ws, size_t ws_bytes,
                    hipStream_t s);
int launch_mono(const float* x, int B, int C, int L, float* y, hipStream_t s);
int launch_augment(const float* x, float* y, int B, int L, const int* kind, const float* factor,
                   const long long* stream, uint64_t seed, hipStream_t s);

// kernels_pitch.hip (model_training_01's pitch branch)
size_t pitch_shift_workspace_bytes(int B, int L, int sr, int n_steps);
int launch_pitch_shift(const float* x, int B, int L, int sr, int n_steps, float* y, void* ws, size_t ws_bytes,
                       hipStream_t s);
