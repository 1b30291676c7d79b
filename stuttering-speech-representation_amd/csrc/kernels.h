// Launcher declarations for kernels_misc.hip (host orchestration in sse_model.hip).
#pragma once
#include "common.h"

int launch_wave_stats(const float* x, int B, int L, float* out, hipStream_t s);

int conv0_chunks(int T0);
template <typename TO>
int launch_conv0_gn(const float* x, int B, int L, const float* norm, const float* w0, const float* b0, int C,
                    int k0, int s0, int T0, const float* gamma, const float* beta, float eps, double2* part,
                    float2* ss, TO* out, hipStream_t s);

template <typename TI, typename TO>
int launch_layernorm(const TI* in, const float* w, const float* b, int rows, int H, float eps, int act,
                     float* out_f, TO* out_t, hipStream_t s);

int launch_pool_mean(const float* x, int B, int T, int H, float* out, long long out_stride, hipStream_t s);

struct AttnArgs {
  const void* qkv;       // [B*T][3H]  (q | k | v), element type T
  void* out;             // [B*T][H]
  int T, H, nh;
  float scale;           // applied to q.k (WavLM 1/sqrt(d); Whisper 1, q pre-scaled in weights)
  // WavLM gated relative-position bias (all null for Whisper)
  const float* gx;       // [B*T][H] fp32 gate input (the attention input hidden state)
  const float* gw;       // [8][64]
  const float* gb;       // [8]
  const float* gconst;   // [nh]
  const float* relb;     // [nh][2*maxd+1], index d + maxd
  int maxd;
};
template <typename T>
int launch_attention(const AttnArgs& a, int B, hipStream_t s);
