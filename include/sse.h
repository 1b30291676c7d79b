/*
 * sse.h — C-ABI of libsse.so, the MI355X (gfx950) speech-embedding extractor.
 *
 * The reference (warren-machy/stuttering-speech-representation) has no native FFI: its
 * operator API for the hot path is the HF object pair handed to its glue functions
 * (SURVEY.md §8(b)).  Each entry point below replaces one piece of that Python surface:
 *
 *   sse_model_create    <- WavLMModel.from_pretrained(...).to(device)      REF/WavLM_embeddings.py:482-483
 *                          WhisperModel.from_pretrained(...).to(device)    REF/whisper_embeddings_large.py:437-438
 *   sse_logmel          <- WhisperProcessor(audio, sampling_rate=16000)   REF/whisper_embeddings_large.py:242-246
 *                          (HF/models/whisper/feature_extraction_whisper.py:135-168)
 *   sse_embed           <- fe(audio) -> model(..., output_hidden_states=True) -> torch.mean(hs[idx], dim=1)
 *                          REF/WavLM_embeddings.py:289-323, REF/whisper_embeddings_large.py:242-281
 *   sse_hidden_states   <- model(input_values, output_hidden_states=True).hidden_states
 *                          REF/WavLM_embeddings.py:249-265 (get_model_layer_info), :302-310
 *   sse_model_destroy   <- del model / torch.cuda.empty_cache()            REF/WavLM_embeddings.py:630
 *
 * Conventions: plain pointers and sizes only.  Every d_* pointer is DEVICE memory owned by
 * the caller; the handle owns only the weights and derived tables.  Calls other than
 * sse_model_create / sse_model_destroy are asynchronous on `stream` (a hipStream_t, passed
 * as void*; NULL = the legacy default stream) and perform no host synchronisation, so they
 * may be captured into a hipGraph.  Return value 0 = success, negative = error (see
 * sse_strerror).  A handle is bound to one device; concurrent calls are safe on distinct
 * streams with distinct workspaces.
 */
#ifndef SSE_H
#define SSE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum sse_kind { SSE_KIND_WAVLM = 0, SSE_KIND_WHISPER = 1 };
/* SSE_DTYPE_FP8 (Whisper): bf16 activations, the encoder layers' QKV / fc1 / fc2 GEMMs in MX-fp8
 * (OCP e4m3 operands, one E8M0 scale per 32 K-elements, BASELINE configs[4] "fp8 MFMA encoder"). */
/* SSE_DTYPE_FP16X3 (WavLM with the "group" frontend and post-LN encoder, i.e. WavLM-base): the
 * fp32 path with every dense GEMM / strided conv on the fp16 matrix cores in split form: operands
 * x = hi + lo (two fp16, the lo plane carried scaled by 2^11 and the weights by a power of two so no
 * operand is an fp16 subnormal), products hi*hi + lo*hi + hi*lo accumulated in fp32 (~22 significant
 * bits per operand) -- fp32-class embeddings (<= 1e-4 rel-L2, also with outlier-channel weights) at
 * ~1/3 of the bf16 GEMM rate, with conv0, the positional conv and the attention core in exact fp32.
 * Activations must stay inside the fp16 range (|x| < 65504): a non-finite output is reported by
 * sse_check_range as SSE_ERR_RANGE. */
/* SSE_DTYPE_FP16 (WavLM-base / -large): the bf16 path's kernels and data flow with fp16 instead of bf16 activations,
 * weights and MFMA operands -- the same matrix-core rate, 8 more mantissa bits per operand (emulated
 * ideal-operand error on outlier-channel weights 0.017 rel-L2 vs 0.226 for bf16, oracle/emulate.py).
 * Range as FP16X3 (|x| < 65504, checked by sse_check_range). */
enum sse_dtype { SSE_DTYPE_F32 = 0, SSE_DTYPE_BF16 = 1, SSE_DTYPE_FP8 = 2, SSE_DTYPE_FP16X3 = 3, SSE_DTYPE_FP16 = 4 };
enum sse_err {
  SSE_OK = 0,
  SSE_ERR_INVALID = -1,      /* bad argument / null pointer / bad layer index         */
  SSE_ERR_HIP = -2,          /* a HIP runtime call failed (launch, copy, malloc)       */
  SSE_ERR_UNSUPPORTED = -3,  /* shape outside what the kernels implement              */
  SSE_ERR_WORKSPACE = -4,    /* ws_bytes < sse_workspace_bytes(...)                    */
  SSE_ERR_WEIGHTS = -5,      /* host weight blob size does not match the config        */
  SSE_ERR_OOM = -6,          /* device allocation failed (torch.OutOfMemoryError twin) */
  SSE_ERR_RANGE = -7         /* an fp16-range path produced a non-finite output (sse_check_range) */
};

/* Model shape.  Field meaning follows the HF configs (WavLMConfig / WhisperConfig). */
typedef struct sse_cfg {
  int32_t kind;              /* sse_kind                                              */
  int32_t hidden;            /* hidden_size / d_model                                 */
  int32_t layers;            /* num_hidden_layers / encoder_layers                    */
  int32_t heads;             /* num_attention_heads / encoder_attention_heads         */
  int32_t ffn;               /* intermediate_size / encoder_ffn_dim                   */
  /* WavLM conv feature encoder */
  int32_t n_conv;            /* 7                                                     */
  int32_t conv_dim[8];
  int32_t conv_kernel[8];
  int32_t conv_stride[8];
  int32_t conv_bias;         /* 0/1                                                   */
  int32_t feat_norm_layer;   /* 0: GroupNorm on conv0 ("group"); 1: LN after each conv */
  int32_t stable_layer_norm; /* 0: post-LN encoder (base); 1: pre-LN + final LN (large) */
  int32_t pos_kernel;        /* 128                                                   */
  int32_t pos_groups;        /* 16                                                    */
  int32_t num_buckets;       /* 320                                                   */
  int32_t max_distance;      /* 800                                                   */
  int32_t do_normalize;      /* Wav2Vec2FeatureExtractor.do_normalize                 */
  /* Whisper */
  int32_t n_mels;            /* 80                                                    */
  int32_t max_positions;     /* 1500                                                  */
  float ln_eps;              /* 1e-5                                                  */
  /* Whisper 1-token decoder pass (REF/whisper_embeddings_large.py:257-262); 0 = encoder only */
  int32_t decoder_layers;
  int32_t dec_ffn;           /* decoder_ffn_dim                                       */
} sse_cfg;

typedef struct sse_model sse_model;

/* Number of fp32 values the weight blob must hold for `cfg` (canonical HF-key order,
 * mirrored by config.param_specs() on the host side). */
size_t sse_weight_floats(const sse_cfg* cfg);

/* Upload + repack weights (weight-norm folded, conv kernels reshaped to [out][k*in],
 * QKV concatenated, bf16 / fp16 cast for SSE_DTYPE_BF16 / SSE_DTYPE_FP16, relative-position bias table
 * precomputed).  Synchronous.  `host_weights` is fp32, `nbytes` = 4 * sse_weight_floats. */
int sse_model_create(const sse_cfg* cfg, const float* host_weights, size_t nbytes,
                     int device, int dtype, sse_model** out);
void sse_model_destroy(sse_model* m);

/* Frames the encoder produces for L input samples (WavLM conv stack; Whisper: 1500). */
int sse_output_frames(const sse_model* m, int L);

/* Device workspace needed by sse_embed / sse_hidden_states for B clips of L samples. */
size_t sse_workspace_bytes(const sse_model* m, int B, int L);

/* Whisper front end: d_wave [B][L] fp32 (L <= 480000, zero-padded to 30 s like
 * WhisperFeatureExtractor) -> d_mel [B][n_mels][3000] fp32, n_mels in [64, 128] (80: v1/v2,
 * 128: v3; SSE_ERR_INVALID otherwise).  Needs sse_logmel_workspace_bytes(B, n_mels) of workspace. */
size_t sse_logmel_workspace_bytes(int B, int n_mels);
int sse_logmel(const float* d_wave, int B, int L, int n_mels, float* d_mel,
               void* d_ws, size_t ws_bytes, void* stream);

/* Fused embedding path: d_in = raw 16 kHz waves [B][L] fp32 (WavLM and Whisper; Whisper
 * computes its log-mel in-stream) -> d_out [B][n_layers][hidden] fp32, the time-mean of
 * hidden_states[layer_ids[i]]. */
int sse_embed(sse_model* m, const float* d_in, int B, int L, const int32_t* layer_ids,
              int n_layers, float* d_out, void* d_ws, size_t ws_bytes, void* stream);

/* Ragged batch (REF/WavLM_embeddings.py:284-307 embeds every file at its own length): d_in [B][L]
 * fp32 holds each clip in the first d_lengths[b] samples of its row (device int32 [B], 1..L; WavLM:
 * >= 400 samples, the conv receptive field).  Each clip's embedding equals that clip run alone:
 * WavLM's GroupNorm statistics, attention keys, positional-conv padding and time-means cover the
 * clip's own frames; Whisper pads each clip with zeros to 30 s as the feature extractor does.
 * Bit-identical to the per-clip call (a batch with clips on both sides of WavLM's 160-frame
 * attention split runs each clip on the kernel it runs alone).  The library clamps each length to [0, L]
 * on the device (no kernel reads past its clip's row whatever the caller passes); a WavLM clip
 * under 400 samples has no frames and its embedding slots are written as zeros (the Python
 * wrapper rejects such clips before the call, as the reference's forward would raise). */
int sse_embed_ragged(sse_model* m, const float* d_in, const int32_t* d_lengths, int B, int L,
                     const int32_t* layer_ids, int n_layers, float* d_out, void* d_ws, size_t ws_bytes,
                     void* stream);

/* Range check of the fp16-range dtypes (SSE_DTYPE_FP16, SSE_DTYPE_FP16X3): every sse_embed /
 * sse_embed_ragged / sse_hidden_states call on such a model also scans the fp32 values it wrote and
 * raises a device flag when one is non-finite (an fp16 activation overflowed: |x| >= 65504 somewhere
 * in the forward).  sse_check_range synchronises `stream`, reads and clears the flag and returns
 * SSE_ERR_RANGE if it was raised since the last check (0 otherwise; always 0 for other dtypes).  The
 * flag is per handle: with concurrent streams, check after joining them. */
int sse_check_range(sse_model* m, void* stream);

/* Same forward, materialising every hidden state: d_hs [layers+1][B][T][hidden] fp32. */
int sse_hidden_states(sse_model* m, const float* d_in, int B, int L, float* d_hs,
                      void* d_ws, size_t ws_bytes, void* stream);

/* Whisper encoder from an HF-layout log-mel (model.encoder(input_features) twin,
 * REF/whisper_embeddings_large.py:250-254): d_mel [B][n_mels][3000] fp32 ->
 * d_hs [layers+1][B][1500][hidden] fp32.  Workspace: sse_workspace_bytes(m, B, 480000). */
int sse_whisper_hidden_states_from_mel(sse_model* m, const float* d_mel, int B, float* d_hs, void* d_ws,
                                       size_t ws_bytes, void* stream);

/* Whisper encoder AND decoder embeddings in one call (extract_whisper_embeddings_fixed,
 * REF/whisper_embeddings_large.py:234-299): waves [B][L] -> d_enc_out [B][n_enc][hidden]
 * (time-means of encoder hidden states) and d_dec_out [B][n_dec][hidden] (decoder hidden
 * states of the single input token id 0; needs cfg.decoder_layers > 0). */
int sse_whisper_embed(sse_model* m, const float* d_wave, int B, int L, const int32_t* enc_ids, int n_enc,
                      float* d_enc_out, const int32_t* dec_ids, int n_dec, float* d_dec_out, void* d_ws,
                      size_t ws_bytes, void* stream);
/* model.decoder(input_ids=zeros([B,1]), encoder_hidden_states=enc) twin: d_enc [B][1500][hidden]
 * fp32 (the encoder's last_hidden_state) -> d_hs [decoder_layers+1][B][hidden] fp32. */
int sse_whisper_decoder_hidden_states(sse_model* m, const float* d_enc, int B, float* d_hs, void* d_ws,
                                      size_t ws_bytes, void* stream);

/* ---- ingest ----
 * Mono mix: torch.mean(waveform, dim=0) of load_audio (REF/WavLM_embeddings.py:103-105,
 * REF/whisper_embeddings_large.py:78-96): d_in [B][C][L] -> d_out [B][L]. */
int sse_mono(const float* d_in, int B, int C, int L, float* d_out, void* stream);
/* torchaudio.transforms.Resample(orig_freq, new_freq) (default sinc_interp_hann, width 6, rolloff
 * 0.99) of load_audio (REF/WavLM_embeddings.py:107-110): d_in [B][L] -> d_out [B][Lo],
 * Lo = sse_resample_length(L, orig, new) = ceil(new*L/orig). */
int sse_resample_length(int L, int orig_freq, int new_freq);
size_t sse_resample_workspace_bytes(int B, int L, int orig_freq, int new_freq);
int sse_resample(const float* d_in, int B, int L, int orig_freq, int new_freq, float* d_out, void* d_ws,
                 size_t ws_bytes, void* stream);

/* Pointwise part of augment_audio (REF/model_training_1.py:167-214), one
 * clip per row of d_in [B][L]: kind 0 none, 1 noise (x + N(0,1)*factor, N from the counter-hash
 * Gaussian stream d_stream[b] of `seed`), 2 volume (x*factor), 3 clamp only (after the speed
 * round trip, done with sse_resample); every kind ends in clamp(-1, 1). */
int sse_augment(const float* d_in, float* d_out, int B, int L, const int32_t* d_kind, const float* d_factor,
                const int64_t* d_stream, uint64_t seed, void* stream);

/* Pitch branch of augment_audio (REF/model_training_01.py:172-177): torchaudio.transforms.
 * PitchShift(sample_rate, n_steps) with its defaults (bins_per_octave 12, n_fft 512, hop 128,
 * periodic Hann) = STFT -> phase vocoder (rate 2^(-n_steps/12)) -> iSTFT (length round(L/rate))
 * -> resample int(sample_rate/rate) -> sample_rate -> truncate / zero-pad to L.  d_in, d_out
 * [B][L] (all clips share n_steps); L must exceed 256 (torch.stft's reflect padding, the
 * reference raises and keeps the original clip).  No clamp: sse_augment kind 3 follows. */
size_t sse_pitch_shift_workspace_bytes(int B, int L, int sample_rate, int n_steps);
int sse_pitch_shift(const float* d_in, int B, int L, int sample_rate, int n_steps, float* d_out, void* d_ws,
                    size_t ws_bytes, void* stream);

/* Wav2Vec2FeatureExtractor zero_mean_unit_var_norm on device (feature_extraction_wav2vec2.py:94):
 * d_out[b] = (d_in[b] - mean_b) / sqrt(var_b + 1e-7).  Workspace: 8 * B bytes. */
int sse_normalize(const float* d_in, int B, int L, float* d_out, void* d_ws, size_t ws_bytes, void* stream);

size_t sse_normalize_workspace_bytes(int B);

/* Live per-launch timing for benchmarks: after sse_profile_start every kernel launch of
 * sse_embed / sse_hidden_states is bracketed by two hipEvents on the caller's stream
 * (at most max_launches per read).  sse_profile_read synchronises on the last event and
 * returns the number of launches n, filling per launch: tag (32 chars, "<kernel>:<role>"),
 * elapsed ms, algorithmic FLOPs and algorithmic bytes; then clears the record. */
int sse_profile_start(sse_model* m, int max_launches);
int sse_profile_read(sse_model* m, int cap, char* tags, float* ms, double* flops, double* bytes);
int sse_profile_stop(sse_model* m);

/* The MFMA GEMM the path is built on, exposed for kernel tests and microbenchmarks:
 * C[M][N] = A[M][K] . B[N][K]^T (+bias[N]) (GELU if act == 1) (+resid[M][N] fp32), written to
 * d_cf (fp32) and/or d_ct (bf16 or fp32 = dtype).  A, B in the dtype; d_zero >= 64 zero bytes. */
int sse_gemm(int dtype, const void* d_a, const void* d_b, const float* d_bias, const float* d_resid, float* d_cf,
             void* d_ct, int M, int N, int K, int act, const void* d_zero, void* stream);

/* The Whisper (no-bias) flash attention of the bf16 / fp8 encoder (test hook): d_out bf16 [B*T][H] =
 * softmax(scale * q k^T) v per head (nh heads of 64), q | k | v the bf16 rows of d_qkv [B*T][ldq]
 * (q at column 0, k at H, v at 2H).  q_log2 = 1: q already carries scale' * log2(e) and scale must be
 * ln 2 = 0.6931471805599453f (else SSE_ERR_INVALID; the encoder's layout; the 32x32 kernel, option attn_long
 * picks the variant); q_log2 = 0: any scale, the 16x16 kernel.  REF/whisper_embeddings_large.py:250 -> HF WhisperAttention (SDPA). */
int sse_attention(const void* d_qkv, void* d_out, int B, int T, int H, int nh, int ldq, float scale, int q_log2,
                  void* stream);

/* The fp8 encoder's attention (test hook; the SSE_DTYPE_FP8 Whisper path's default, option fp8_attn_bf16 = 1
 * keeps the bf16 one): d_out bf16 [B*T][H] = softmax(q k^T) v per head (nh heads of 64; q carries the softmax
 * scale * log2(e), so the scores are log2-domain logits), q | k MX-fp8 [B*T][2H] e4m3 with their E8M0 scales
 * row-major [B*T][2H / 32] (blocks of 32 columns: the c_scale_rm output of sse_gemm_ex), v bf16 [B*T][H],
 * d_vamax [B][H] the float bits of max |bf16 v| per (clip, column) (the vamax output of sse_gemm_ex).  Both
 * products on the block-scaled fp8 MFMA: P in e4m3, V in e4m3 with one power-of-two scale per (clip, head).
 * REF/whisper_embeddings_large.py:250-254 (fp8 encoder) -> HF WhisperAttention (SDPA). */
int sse_attention_f8(const uint8_t* d_qk, const uint8_t* d_qk_scale, const void* d_v, const uint32_t* d_vamax,
                     void* d_out, int B, int T, int H, int nh, void* stream);

/* sse_attention_f8 with the output as MX-fp8 (test hook; round 6: with option f8_oproj = 1 the SSE_DTYPE_FP8
 * Whisper path's attention writes this and its out-projection runs on the MX GEMM): d_out_q e4m3 [B*T][H], d_out_scale the E8M0 exponents of every 32-column block in the MX GEMM's
 * A-operand layout for K = H (sse_mx_scale_bytes(B*T, H) bytes; the layout sse_mx_quantize role 0 writes).  Each
 * block's exponent is the smallest E with max |o| <= 448 * 2^E over its fp32 outputs, each code RNE(o * 2^-E).
 * H % 128 == 0.  Same reference line as sse_attention_f8. */
int sse_attention_f8_mx(const uint8_t* d_qk, const uint8_t* d_qk_scale, const void* d_v, const uint32_t* d_vamax,
                        uint8_t* d_out_q, uint8_t* d_out_scale, int B, int T, int H, int nh, void* stream);

/* Every epilogue form of the path's GEMMs behind one test hook (guard-band and epilogue tests; no
 * reference counterpart).  C[M][N] = A[M][K] . B[N][K]^T with, by the non-null fields:
 *   bias[N]; act (0 none, 1 erf-GELU, 2 the bf16 path's GELU);
 *   apart / acol / apart_nt: the folded LayerNorm of A (rstd_m (acc - mean_m acol[n]) + bias[n], (mean, rstd)
 *     from apart [M][apart_nt] float2 partials, eps ln_eps);
 *   resid [M][ldc] fp32, or resid_t [M][ldc] 16-bit (the bf16 / fp16 residual stream), optionally
 *     LayerNorm'd in the epilogue from rpart [M][3] float2 partials and rln_w / rln_b [N];
 *   opart [M][N / 256] float2: (mean, M2) of every 256 output columns of each written row;
 * written to cf (fp32) and / or ct (dtype: bf16, fp16 or fp32) with row stride ldc >= N.  dtype:
 * SSE_DTYPE_BF16, SSE_DTYPE_FP16 (fp16 operands, 8-phase kernels only), SSE_DTYPE_F32, or SSE_DTYPE_FP8: a / b
 * MX-fp8 operands with their tiled scales a_scale / b_scale (sse_mx_quantize), ldc == N, out bf16 ct (optionally
 * with the bf16 residual stream resid_t, in place as the Whisper fc2 runs it) or fp32 cf.  The dispatch is the
 * model's own (launch_gemm<T> / launch_gemm8_mx): a combination no kernel takes returns SSE_ERR_INVALID. */
typedef struct sse_gemm_desc {
  int dtype, M, N, K, ldc, act, apart_nt;
  float ln_eps;
  const void* a;
  const void* b;
  const float* bias;
  const float* acol;
  const float* apart;
  const float* resid;
  const void* resid_t;
  const float* rpart;
  const float* rln_w;
  const float* rln_b;
  float* opart;
  float* cf;
  void* ct;
  const void* zero;   /* >= 64 zero bytes of device memory */
  const uint8_t* a_scale;   /* SSE_DTYPE_FP8 only */
  const uint8_t* b_scale;
  /* SSE_DTYPE_FP8 outputs of the fp8 attention's operands: c_scale != NULL makes ct MX-fp8 (e4m3) with its
   * scales in c_scale, row-major [M][N / 32] when c_scale_rm = 1 (else the tiled A layout of a following GEMM);
   * vamax != NULL (bf16 ct): atomicMax of the float bits of max |bf16 C[m][n]| over each segment of vamax_rows
   * rows into vamax [M / vamax_rows][N] (zeroed by the caller) */
  uint8_t* c_scale;
  uint32_t* vamax;
  int c_scale_rm, vamax_rows;
  /* n_split > 0 (SSE_DTYPE_FP8, the encoder's fused QKV form): columns [0, n_split) go to ct as MX-fp8 with
   * row-major c_scale (c_scale_rm = 1, ldc = n_split), columns [n_split, N) to ct2 [M][ldc2] bf16 (column
   * n - n_split) with their vamax [M / vamax_rows][N - n_split] */
  void* ct2;
  int n_split, ldc2;
} sse_gemm_desc;
int sse_gemm_ex(const sse_gemm_desc* d, void* stream);

/* The folded-LayerNorm GEMM of the bf16 post-LN path (test hook): d_ct bf16 [M][N] =
 * act(rstd_m * (A B^T)[m][n] + bias[n] - rstd_m mean_m acol[n]), (mean_m, rstd_m) combined from the
 * per-256-column partials d_apart [M][3] (float2 (mean, M2)) with eps; K = 768 (three column tiles),
 * act 0 none / 2 the bf16 path's GELU. */
int sse_gemm_lnfold(const void* d_a, const void* d_b, const float* d_bias, const float* d_acol, const float* d_apart,
                    void* d_ct, int M, int N, int K, int act, float eps, const void* d_zero, void* stream);

/* MX-fp8 operands (SSE_DTYPE_FP8): e4m3 bytes [R][K] (K % 128 == 0) plus E8M0 scales, one per 32
 * consecutive K elements, in the tiled layout the GEMM stages (role 0: A operand / activations,
 * role 1: B operand / weights [N][K]); sse_mx_scale_bytes(R, K) bytes.  Quantisation: block
 * exponent E = the smallest with max|x| <= 448 * 2^E, q = RNE_e4m3(x * 2^-E). */
size_t sse_mx_scale_bytes(int R, int K);
/* byte offset of the scale of (row r, block b = k / 32) in the role's layout */
long long sse_mx_scale_offset(int role, int r, int b, int K);
int sse_mx_quantize(const float* d_x, int R, int K, int role, uint8_t* d_q, uint8_t* d_scale, void* stream);
/* LayerNorm of bf16 rows d_x [R][H] (fp32 statistics, affine d_w / d_b) quantised to MX-fp8 in the A layout
 * (the fp8 Whisper encoder's QKV / fc1 operand: REF/whisper_embeddings_large.py:250-254 -> HF WhisperEncoderLayer
 * self_attn_layer_norm / final_layer_norm); H % 128 == 0, H <= 2048.  Test hook. */
int sse_layernorm_mx(const void* d_x, const float* d_w, const float* d_b, int R, int H, float eps, uint8_t* d_q,
                     uint8_t* d_scale, void* stream);
/* C[M][N] = dequant(A)[M][K] . dequant(B)[N][K]^T (+bias) (GELU: act 1 erf, 2 bf16-path form)
 * (+resid fp32) -> d_cf fp32, or d_ct bf16, or (d_c_scale != NULL) d_ct MX-fp8 in the A layout of
 * a GEMM with K = N.  M > 0, N % 256 == 0, K % 128 == 0. */
int sse_gemm_mx(const uint8_t* d_a, const uint8_t* d_a_scale, const uint8_t* d_b, const uint8_t* d_b_scale,
                const float* d_bias, const float* d_resid, float* d_cf, void* d_ct, uint8_t* d_c_scale, int M, int N,
                int K, int act, void* stream);

/* Host-only helpers (no device work; usable without a GPU). */
/* The quantiser above on the host (what sse_model_create applies to the weights). */
int sse_mx_quantize_host(const float* x, int R, int K, int role, uint8_t* q, uint8_t* scale);
const char* sse_strerror(int err);
/* WavLM relative-position bucket of distance d = key - query (HF _relative_positions_bucket). */
int sse_rel_bucket(int d, int num_buckets, int max_distance);
/* Whisper Slaney mel filter bank, [n_freq = 201][n_mels] fp32 as HF casts it. */
int sse_mel_filters(int n_mels, float* out);
/* Library version string. */
const char* sse_version(void);

/* Kernel-selection switches for A/B equality tests (no reference counterpart; the library never
 * reads the environment).  Process-wide; 0 is the production choice for every name:
 *   "gemm_cfg"          1 = no 256x256 tile, 2 = 256x128 3-stage ring, 3 = 2-stage 256x256 kernel
 *   "gemm_nonpersist"   1 = non-persistent 8-phase bf16 GEMM for every shape
 *   "gemm_4phase"       8-wave GEMM K-tile schedule, bit-identical outputs: 0 = two 32-MFMA phases per K-tile (round 6
 *                       default), 1 = four 16-MFMA phases (rounds 1-5)
 *   "gelu_exact"        1 = erf-GELU in the bf16 path's epilogues
 *   "conv0_valu"        1 = VALU conv0 + GroupNorm kernel instead of the matrix-core one
 *   "posconv_gemm"      1 = grouped GEMM for the bf16 positional conv
 *   "no_lnfold"         1 = materialise the LayerNorm outputs (bf16 WavLM-base: per call; bf16 Whisper-small /
 *                       -large: read at sse_model_create, the folded model holds no plain QKV weights past layer 0)
 *   "gemm_mx_staged"    1 = LDS-staged epilogue for every MX-fp8 GEMM
 *   "no_split"          1 = WavLM batches run as one stream (no two-stream half-batch split)
 *   "split_cumask"      two-stream half-batch split on CU-masked streams: 1 = CUs [0, n/2) | [n/2, n),
 *                       2 = even | odd CUs (each half's grids sized to its CUs); 0 = both halves share every CU
 *   "logmel_v1"         1 = the one-frame-per-wave log-mel kernel
 *   "ln_x3_v1", "attn_x3_f32", "ln_rows_v1", "posconv_2cl"   earlier kernels kept for A/B and bit-identity tests
 *   "attn_short"        short-T (<= 160 frames) attention: 0 = head-pipelined, double-buffered, one block per CU
 *                       (production), 1 = one head at a time (bit-identical; the reference of
 *                       tests/test_gpu_attention_pipe.py), 2 = two blocks per CU with single-buffered refills
 *                       (round 6; bit-identical, slower)
 *   "attn_long"         Whisper bf16 / fp8 encoder attention: 0 = the 32x32 swapped-product kernel with two
 *                       32-query blocks per wave (production), 2 = the same with one (identical outputs),
 *                       1 = the 16x16 flash kernel (same bar, not bit-identical)
 *   "fp8_attn_bf16"     1 = the fp8 Whisper path keeps the bf16 QKV output and the bf16 flash attention
 *   "f8_oproj"          1 = the fp8 Whisper path's attention writes MX-fp8 and its out-projection runs on the MX
 *                       GEMM (opt-in: Whisper-large-v2 then misses the fp8 bar, 0.083 vs 0.08 rel-L2)
 * sse_set_option returns the previous value (>= 0), or SSE_ERR_INVALID for an unknown name or a value outside
 * the switch's range (0..1; gemm_cfg 0..3, attn_short 0..2, attn_long 0..2, split_cumask 0..2) -- nothing is changed then. */
int sse_set_option(const char* name, int value);
int sse_get_option(const char* name);

#ifdef __cplusplus
}
#endif
#endif /* SSE_H */
