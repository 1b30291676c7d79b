#pragma once
#include "common.h"

constexpr int LM_NFFT = 400;   // Whisper STFT: 400-point frames, hop 160, 201 bins
constexpr int LM_MAXMEL = 128;   // n_mels: 80 (v1/v2) or 128 (v3)

size_t logmel_workspace_bytes(int B, int n_mels);
// x [B][L] fp32 -> out_hf [B][n_mels][3000] fp32 (optional) and out_cl [B][3000][n_mels] (optional);
// lens (ragged batch, device, optional): samples of each clip, zeros after (the feature extractor's padding)
template <typename TO>
int launch_logmel(const float* x, int B, int L, int n_mels, float* out_hf, TO* out_cl, void* ws, size_t ws_bytes,
                  hipStream_t s, const int* lens = nullptr);
// HF-layout mel [B][n_mels][3000] fp32 -> channels-last [B][3000][n_mels]
template <typename TO>
int launch_mel_to_cl(const float* mel_hf, int B, int n_mels, TO* out_cl, hipStream_t s);
// y = (x - st[b].mean) * st[b].rstd
int launch_normalize_apply(const float* x, int B, int L, const float* st, float* y, hipStream_t s);
