// Internal helpers shared by the gfx950 kernels and the host orchestration.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef _Float16 f16;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;

// Split-fp16 operands (SSE_DTYPE_FP16X3).  A value v is carried as hi = f16(v) and lo' = f16((v - hi)
// * 2^11): lo' keeps the magnitude of v, so it stays a normal fp16 for every v the fp16 range holds
// (an unscaled lo would fall into fp16 subnormals for |v| < 2^-3).  Activation rows are [hi | lo' | hi]
// and weight rows (pre-scaled by 2^s) [hi | hi * 2^-11 | lo] per K-block, so one f16 MFMA over
// K' = 3K accumulates hi*hi + lo*hi + hi*lo: about 22 significant bits per operand (the dropped
// lo*lo term is ~2^-22 relative).
constexpr float X3_LO_SCALE = 2048.f;
__host__ __device__ inline void x3_split4(const f32x4& v, f16x4& hi, f16x4& lo) {
  #pragma unroll
  for (int e = 0; e < 4; ++e) {
    hi[e] = (f16)v[e];
    lo[e] = (f16)((v[e] - (float)hi[e]) * X3_LO_SCALE);
  }
}

#define SSE_DEV __device__ __forceinline__

// Address-space casts for global_load_lds.
#define GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define LPTR(p) ((__attribute__((address_space(3))) void*)(p))

// erf-GELU, branch-free: gelu(x) = x - x/2 erfc(x/sqrt2) (x >= 0), x/2 erfc(-x/sqrt2) (x < 0), with
// erfc from the Chebyshev fit of Numerical Recipes (erfcc, relative error < 1.2e-7 over the
// whole line).  fp32 evaluation: max |err| 2.4e-7, relative 2.4e-6 wherever |gelu| > 1e-6
// (checked against scipy erf on 2.2M points); the negative tail keeps relative precision.
// One v_rcp, one v_exp and ~14 FMA, no divergent branches (ocml erff branches on |x|).
SSE_DEV float gelu_erf(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, z, 1.0f));
  float p = 0.17087277f;
  p = fmaf(p, t, -0.82215223f);
  p = fmaf(p, t, 1.48851587f);
  p = fmaf(p, t, -1.13520398f);
  p = fmaf(p, t, 0.27886807f);
  p = fmaf(p, t, -0.18628806f);
  p = fmaf(p, t, 0.09678418f);
  p = fmaf(p, t, 0.37409196f);
  p = fmaf(p, t, 1.00002368f);
  p = fmaf(p, t, -1.26551223f);
  const float erfc = t * __expf(fmaf(-z, z, p));
  const float h = 0.5f * x * erfc;
  return x >= 0.f ? x - h : h;
}

// Same evaluation on a channel pair with packed fp32 math (v_pk_fma_f32 / v_pk_mul_f32): the
// polynomial runs at 2 results per instruction, only v_rcp / v_exp stay scalar.  Each lane is
// the identical IEEE fma chain as gelu_erf, so results are bit-identical to the scalar form.
typedef float f32x2 __attribute__((ext_vector_type(2)));
SSE_DEV f32x2 gelu_erf2(f32x2 x) {
  const f32x2 z = __builtin_elementwise_abs(x) * 0.70710678118654752f;
  const f32x2 d = __builtin_elementwise_fma(f32x2{0.5f, 0.5f}, z, f32x2{1.0f, 1.0f});
  const f32x2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 p = {0.17087277f, 0.17087277f};
  p = __builtin_elementwise_fma(p, t, f32x2{-0.82215223f, -0.82215223f});
  p = __builtin_elementwise_fma(p, t, f32x2{1.48851587f, 1.48851587f});
  p = __builtin_elementwise_fma(p, t, f32x2{-1.13520398f, -1.13520398f});
  p = __builtin_elementwise_fma(p, t, f32x2{0.27886807f, 0.27886807f});
  p = __builtin_elementwise_fma(p, t, f32x2{-0.18628806f, -0.18628806f});
  p = __builtin_elementwise_fma(p, t, f32x2{0.09678418f, 0.09678418f});
  p = __builtin_elementwise_fma(p, t, f32x2{0.37409196f, 0.37409196f});
  p = __builtin_elementwise_fma(p, t, f32x2{1.00002368f, 1.00002368f});
  p = __builtin_elementwise_fma(p, t, f32x2{-1.26551223f, -1.26551223f});
  const f32x2 e = __builtin_elementwise_fma(-z, z, p);
  const f32x2 erfc = t * f32x2{__expf(e.x), __expf(e.y)};
  const f32x2 h = 0.5f * x * erfc;
  const f32x2 pos = x - h;
  return f32x2{x.x >= 0.f ? pos.x : h.x, x.y >= 0.f ? pos.y : h.y};
}

// The bf16 path's GELU (ACT_GELU_FAST): x * Phi(x) with Phi(x) - 1/2 = xc R(xc^2), xc = clamp(x, +-4.5),
// R the degree-8 minimax fit (tools/fit_gelu.py; its constant nudged so Phi(4.5) = 1 exactly in fp32 and
// Phi(-4.5) = 3e-8: relu beyond the clamp) -- no transcendental: 2 med3 + 11 packed ops per pair
// (the sigmoid form x / (1 + 2^(x P(x^2))) cost 2 v_exp + 2 v_rcp more; persistent-GEMM A/B ffn1 +3-7 %,
// conv1 +2-4 %).  Max abs error 7.3e-5 vs fp64 erf: 50x below the bf16 output's half-ulp at |y| ~ 1.
// The fp32 path keeps gelu_erf2.
SSE_DEV f32x2 gelu_fast2(f32x2 x) {
  const f32x2 xc = {__builtin_amdgcn_fmed3f(x.x, -4.5f, 4.5f), __builtin_amdgcn_fmed3f(x.y, -4.5f, 4.5f)};
  const f32x2 s = xc * xc;
  f32x2 p = {3.144668553e-11f, 3.144668553e-11f};
  p = __builtin_elementwise_fma(p, s, f32x2{-3.420433270e-09f, -3.420433270e-09f});
  p = __builtin_elementwise_fma(p, s, f32x2{1.634204949e-07f, 1.634204949e-07f});
  p = __builtin_elementwise_fma(p, s, f32x2{-4.547368462e-06f, -4.547368462e-06f});
  p = __builtin_elementwise_fma(p, s, f32x2{8.266720397e-05f, 8.266720397e-05f});
  p = __builtin_elementwise_fma(p, s, f32x2{-1.047152211e-03f, -1.047152211e-03f});
  p = __builtin_elementwise_fma(p, s, f32x2{9.627013467e-03f, 9.627013467e-03f});
  p = __builtin_elementwise_fma(p, s, f32x2{-6.607707590e-02f, -6.607707590e-02f});
  p = __builtin_elementwise_fma(p, s, f32x2{3.987890482e-01f, 3.987890482e-01f});
  return x * __builtin_elementwise_fma(xc, p, f32x2{0.5f, 0.5f});
}

// GELU for a bf16 OUTPUT (round 3): the same clamped odd form at clamp 4.0 and degree 6 in xc^2
// (tools/fit_gelu.py C_CLAMP = 4.0, DEG = 7; constant nudged by whole ulps so Phi(4) = 1 exactly in fp32),
// max abs error 2.2e-4 -- 1/18 of the bf16 half-ulp at |y| = 1 -- for 2 fewer packed fma per pair than
// gelu_fast2, which keeps the fp16 outputs (3 more mantissa bits: 7.3e-5 there is 1/7 of the half-ulp).
SSE_DEV f32x2 gelu_bf2(f32x2 x) {
  const f32x2 xc = {__builtin_amdgcn_fmed3f(x.x, -4.0f, 4.0f), __builtin_amdgcn_fmed3f(x.y, -4.0f, 4.0f)};
  const f32x2 s = xc * xc;
  f32x2 p = {2.368073737e-08f, 2.368073737e-08f};
  p = __builtin_elementwise_fma(p, s, f32x2{-1.652635206e-06f, -1.652635206e-06f});
  p = __builtin_elementwise_fma(p, s, f32x2{4.923747110e-05f, 4.923747110e-05f});
  p = __builtin_elementwise_fma(p, s, f32x2{-8.292031125e-04f, -8.292031125e-04f});
  p = __builtin_elementwise_fma(p, s, f32x2{8.865549229e-03f, 8.865549229e-03f});
  p = __builtin_elementwise_fma(p, s, f32x2{-6.484667212e-02f, -6.484667212e-02f});
  p = __builtin_elementwise_fma(p, s, f32x2{3.981720209e-01f, 3.981720209e-01f});
  return x * __builtin_elementwise_fma(xc, p, f32x2{0.5f, 0.5f});
}
// N independent pairs stage by stage (bit-identical to N calls of gelu_bf2 / gelu_fast2): a lone Horner
// chain is latency-bound (a dependent packed fma every ~8 cycles plus hazard nops); N chains in lockstep
// keep the VALU issuing (the persistent GEMM's epilogue runs 8 at a time).
template <bool H16, int N>
SSE_DEV void gelu_out2_n(f32x2 (&x)[N]) {
  constexpr float C = H16 ? 4.5f : 4.0f;
  constexpr int NC = H16 ? 9 : 7;
  constexpr float cf[9] = {3.144668553e-11f, -3.420433270e-09f, 1.634204949e-07f, -4.547368462e-06f,
                           8.266720397e-05f, -1.047152211e-03f, 9.627013467e-03f, -6.607707590e-02f,
                           3.987890482e-01f};
  constexpr float cb[7] = {2.368073737e-08f, -1.652635206e-06f, 4.923747110e-05f, -8.292031125e-04f,
                           8.865549229e-03f, -6.484667212e-02f, 3.981720209e-01f};
  f32x2 xc[N], s[N], p[N];
  #pragma unroll
  for (int n = 0; n < N; ++n) {
    xc[n] = f32x2{__builtin_amdgcn_fmed3f(x[n].x, -C, C), __builtin_amdgcn_fmed3f(x[n].y, -C, C)};
    s[n] = xc[n] * xc[n];
    const float c0 = H16 ? cf[0] : cb[0];
    p[n] = f32x2{c0, c0};
  }
  #pragma unroll
  for (int k = 1; k < NC; ++k) {
    const float ck = H16 ? cf[k] : cb[k < 7 ? k : 6];
    #pragma unroll
    for (int n = 0; n < N; ++n) p[n] = __builtin_elementwise_fma(p[n], s[n], f32x2{ck, ck});
  }
  #pragma unroll
  for (int n = 0; n < N; ++n) x[n] = x[n] * __builtin_elementwise_fma(xc[n], p[n], f32x2{0.5f, 0.5f});
}

// gelu_fp8out2 (below) over N independent pairs stage by stage (bit-identical to N calls)
template <int N>
SSE_DEV void gelu_fp8out2_n(f32x2 (&x)[N]) {
  constexpr float cf[6] = {-3.503167250e-07f, 2.229058919e-05f, -5.630472442e-04f, 7.574830670e-03f,
                           -6.208017841e-02f, 3.963519037e-01f};
  f32x2 xc[N], s[N], p[N];
  #pragma unroll
  for (int n = 0; n < N; ++n) {
    xc[n] = f32x2{__builtin_amdgcn_fmed3f(x[n].x, -3.5f, 3.5f), __builtin_amdgcn_fmed3f(x[n].y, -3.5f, 3.5f)};
    s[n] = xc[n] * xc[n];
    p[n] = f32x2{cf[0], cf[0]};
  }
  #pragma unroll
  for (int k = 1; k < 6; ++k)
    #pragma unroll
    for (int n = 0; n < N; ++n) p[n] = __builtin_elementwise_fma(p[n], s[n], f32x2{cf[k], cf[k]});
  #pragma unroll
  for (int n = 0; n < N; ++n) x[n] = x[n] * __builtin_elementwise_fma(xc[n], p[n], f32x2{0.5f, 0.5f});
}

// the output's polynomial GELU: bf16 only -> gelu_bf2; fp16, fp32 or an fp32 copy (Cf) -> gelu_fast2
template <bool H16> SSE_DEV f32x2 gelu_out2(f32x2 x) { return H16 ? gelu_fast2(x) : gelu_bf2(x); }
SSE_DEV f32x2 gelu_out2(f32x2 x, bool bf_only) { return bf_only ? gelu_bf2(x) : gelu_fast2(x); }

// GELU for an MX-fp8 output (the fc1 epilogue of the fp8 path, whose result is rounded to e4m3: 3
// mantissa bits, half-step 3 %): the same clamped odd polynomial at degree 5 in xc^2 and clamp 3.5
// (tools/fit_gelu.py C_CLAMP = 3.5, DEG = 6), max abs error 8.2e-4 -- 5 packed fma instead of 8.
SSE_DEV f32x2 gelu_fp8out2(f32x2 x) {
  const f32x2 xc = {__builtin_amdgcn_fmed3f(x.x, -3.5f, 3.5f), __builtin_amdgcn_fmed3f(x.y, -3.5f, 3.5f)};
  const f32x2 s = xc * xc;
  f32x2 p = {-3.503167250e-07f, -3.503167250e-07f};
  p = __builtin_elementwise_fma(p, s, f32x2{2.229058919e-05f, 2.229058919e-05f});
  p = __builtin_elementwise_fma(p, s, f32x2{-5.630472442e-04f, -5.630472442e-04f});
  p = __builtin_elementwise_fma(p, s, f32x2{7.574830670e-03f, 7.574830670e-03f});
  p = __builtin_elementwise_fma(p, s, f32x2{-6.208017841e-02f, -6.208017841e-02f});
  p = __builtin_elementwise_fma(p, s, f32x2{3.963519037e-01f, 3.963519037e-01f});
  return x * __builtin_elementwise_fma(xc, p, f32x2{0.5f, 0.5f});
}


template <typename T> SSE_DEV T from_f32(float v);
template <> SSE_DEV float from_f32<float>(float v) { return v; }
template <> SSE_DEV bf16 from_f32<bf16>(float v) { return (bf16)v; }
template <> SSE_DEV f16 from_f32<f16>(float v) { return (f16)v; }
SSE_DEV float to_f32(float v) { return v; }
SSE_DEV float to_f32(bf16 v) { return (float)v; }
SSE_DEV float to_f32(f16 v) { return (float)v; }

// 16-bit activation formats: bf16 (SSE_DTYPE_BF16 / FP8) and fp16 (SSE_DTYPE_FP16).  Four values of
// either packed into 8 bytes and back; H16 = true selects fp16.
template <bool H16> SSE_DEV uint2 pack_h4(const f32x4& v) {
  if constexpr (H16) {
    const f16x4 x = {(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
    return __builtin_bit_cast(uint2, x);
  } else {
    const bf16x4 x = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
    return __builtin_bit_cast(uint2, x);
  }
}
template <bool H16> SSE_DEV f32x4 unpack_h4(uint2 u) {
  if constexpr (H16) {
    const f16x4 x = __builtin_bit_cast(f16x4, u);
    return f32x4{(float)x[0], (float)x[1], (float)x[2], (float)x[3]};
  } else {
    const bf16x4 x = __builtin_bit_cast(bf16x4, u);
    return f32x4{(float)x[0], (float)x[1], (float)x[2], (float)x[3]};
  }
}
template <bool H16> SSE_DEV float round_h(float v) { return H16 ? (float)(f16)v : (float)(bf16)v; }
// one 16-bit value in a bf16x8 / bf16x4 lane (the 16-bit vectors are bit containers for both formats)
template <bool H16> SSE_DEV bf16 hbits(float v) { return H16 ? __builtin_bit_cast(bf16, (f16)v) : (bf16)v; }
template <bool H16> SSE_DEV float hval(bf16 b) { return H16 ? (float)__builtin_bit_cast(f16, b) : (float)b; }
// 16x16x32 MFMA on bf16 or fp16 operands held in bf16x8 containers
template <bool H16> SSE_DEV f32x4 mfma_h(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  if constexpr (H16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
typedef __attribute__((ext_vector_type(16))) float f32x16;
// 32x32x16 MFMA on bf16 or fp16 operands held in bf16x8 containers
template <bool H16> SSE_DEV f32x16 mfma32_h(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  if constexpr (H16)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// 8 fp32 -> 16 B of bf16 / fp16
template <bool H16> SSE_DEV uint4 pack_h8(const f32x4& a, const f32x4& b) {
  const uint2 x = pack_h4<H16>(a), y = pack_h4<H16>(b);
  return make_uint4(x.x, x.y, y.x, y.y);
}
template <typename T> constexpr bool is_f16_v = __is_same(T, f16);

SSE_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
SSE_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
SSE_DEV double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Epilogue activation codes.
// ACT_GELU_FAST: gelu_fast2, used by the bf16 path only (host picks it, see gelu_act<T>()).
enum { ACT_NONE = 0, ACT_GELU = 1, ACT_GELU_FAST = 2 };

// Kernel-selection switches for A/B equality tests, set only through the C-ABI
// (sse_set_option, include/sse.h); process-wide, 0 = the production choice.  Nothing is read from
// the environment.
enum {
  OPT_GEMM_CFG = 0,     // 1: never 256x256, 2: 256x128 3-stage ring, 3: 2-stage 256x256 kernel
  OPT_GEMM_NONPERSIST,  // 1: the non-persistent LDS-staged 8-phase kernel for every shape
  OPT_GELU_EXACT,       // 1: erf-GELU on the bf16 path too
  OPT_CONV0_VALU,       // 1: packed-fp32 VALU conv0 instead of the matrix-core kernel
  OPT_POSCONV_GEMM,     // 1: grouped GEMM for the bf16 positional conv
  OPT_NO_LNFOLD,        // 1: materialise post-LN LayerNorm outputs (bf16 WavLM-base)
  OPT_GEMM_MX_STAGED,   // 1: LDS-staged epilogue for every MX-fp8 GEMM
  OPT_NO_SPLIT,         // 1: WavLM batches run as one stream (no two-stream half-batch split)
  OPT_LOGMEL_V1,        // 1: the round-2 log-mel kernel (one frame per wave) instead of 4 frames per wave
  OPT_LN_X3_V1,         // 1: the one-row-per-wave split-fp16 LayerNorm (A/B, bit-identity test)
  OPT_ATTN_X3_F32,      // 1: the split-fp16 path's attention on the exact-f32 MFMA (A/B, tests)
  OPT_LN_ROWS_V1,       // 1: 16-bit LayerNorm rows over 512 columns on the one-row-per-wave kernel (A/B, tests)
  OPT_POSCONV_2CL,      // 1: the 16-bit positional conv at 2 clips per block for every shape (A/B, tests)
  OPT_ATTN_SHORT,       // short-T attention: 0 head-pipelined (default), 1 one head at a time (bit-identity tests)
  OPT_ATTN_LONG,        // no-bias (Whisper) flash attention: 0 32x32 swapped form, 2 query blocks per wave (default);
                        // 2 the same with one; 1 the 16x16 flash2 kernel
  OPT_FP8_ATTN_BF16,    // 1: the fp8 (MX) Whisper path keeps the bf16 QKV output and the bf16 flash attention
  OPT_SPLIT_CUMASK,     // two-stream split on CU-masked streams: 1 = CUs [0, n/2) | [n/2, n), 2 = even | odd CUs
  OPT_GEMM_4PHASE,      // 8-wave GEMM K-tile schedule (bit-identical): 0 = two 32-MFMA phases per K-tile (default since
                        // round 6), 1 = four 16-MFMA phases (rounds 1-5)
  OPT_F8_OPROJ,         // 1: the fp8 (MX) Whisper path's out-projection on the MX GEMM (MX-fp8 attention output);
                        // opt-in: large-v2 at B = 128 then misses the 0.08 rel-L2 bar (0.083)
  OPT_COUNT
};
int sse_opt(int id);
// CUs a kernel launched on stream s may use: the registered count of a CU-masked stream (split_forward,
// OPT_SPLIT_CUMASK), else dev_cus.  Launchers that size a grid to the CU count (persistent GEMM, attention
// heads per block, conv0) ask it, so a masked stream's grid matches its CUs.
int sse_stream_cus(hipStream_t s, int dev_cus);
inline bool gelu_exact_env() { return sse_opt(OPT_GELU_EXACT) != 0; }

// ---------------------------------------------------------------------------------------
// GEMM descriptor.  C[m][n] = sum_k A(m, k) * Bt[n][k]  (+bias[n]) (act) (+resid[m][n]).
// A(m, k) addressing:
//   SEG  : A + (m / rows_per_seg) * seg_stride + (m % rows_per_seg) * lda + k
//          (plain GEMM: rows_per_seg = M, lda = K; strided conv without padding:
//           rows_per_seg = T_out, seg_stride = T_in*C, lda = stride*C, K = k*C)
//   CONV : padded (grouped) conv over channels-last input [seg][T_in][ld_in]:
//          j = k / cin, c = k % cin, t_in = (m % T_out) * stride + j - pad,
//          A + ((m / T_out) * T_in + t_in) * ld_in + group * cin + c, zero outside [0, T_in)
// Columns beyond K (k >= K) read as zero on both operands.
// ---------------------------------------------------------------------------------------
struct GemmArgs {
  const void* A;
  const void* B;        // [groups][N][K] row-major (K contiguous)
  int M, N, K;
  int rows_per_seg;     // SEG / CONV (= T_out)
  long long seg_stride; // SEG
  long long lda;        // SEG
  int T_in, stride, pad, cin, ld_in;   // CONV
  const float* bias;    // [groups*N] or null
  const float* resid;   // [M][ldc] fp32 or null (row m % resid_rows when resid_rows > 0)
  int resid_rows;       // 0: resid row = m; >0: periodic residual (Whisper embed_positions)
  float* Cf;            // fp32 out [M][ldc] or null
  void* Ct;             // element-type out [M][ldc] or null
  int ldc;
  int act;
  const void* zero;     // >= 64 zero bytes of device memory
  // resid' = LayerNorm(resid) applied in the epilogue from per-row (mean, rstd) and per-column
  // (w, b): the residual stream then never has to be written normalised in fp32 (post-LN path)
  const float2* rstats;
  const float* rln_w;
  const float* rln_b;
  // MX-fp8 operands (launch_gemm8_mx): A / B are e4m3 bytes, one E8M0 scale per 32 consecutive K
  // elements in the tile layouts of mx_a_scale_off / mx_b_scale_off.  c_scale != null: Ct is e4m3
  // with its scales written in the A layout of a following GEMM whose K is this GEMM's N.
  const unsigned char* a_scale;
  const unsigned char* b_scale;
  unsigned char* c_scale;
  // Folded LayerNorm (post-LN bf16 path, no LayerNorm kernel): A holds bf16 of the UN-normalised
  // rows x and B = W diag(ln_w) (bf16); the epilogue forms LN(x) W^T + b as
  //   rstd_m * (acc - mean_m * acol[n]) + bias[n],   acol[n] = sum_k B[n][k],  bias = b + W ln_b,
  // with (mean_m, rstd_m) combined from the per-256-column partials apart[m][apart_nt] (ln_part_stats).
  const float2* apart;
  int apart_nt;
  const float* acol;
  // residual LayerNorm from partials rpart[m][rpart_nt] (instead of rstats), affine rln_w / rln_b
  const float2* rpart;
  int rpart_nt;
  float ln_eps;
  // partials of the rows this GEMM writes: opart[m][N / 256] = (mean, M2) over each 256-column
  // tile (residual GEMMs of the folded path; of the rounded values when the output is bf16)
  float2* opart;
  // bf16 residual [M][ldc] (instead of resid; folded post-LN path: the residual stream is kept in
  // bf16 and the output is bf16 Ct only)
  const bf16* resid_t;
  // split-fp16 GEMM (SSE_DTYPE_FP16X3): A / B are fp16 planes (x3_split4), the MFMA is the f16 one and
  // the epilogue scales the accumulator by alpha (the weights' power-of-two scale undone).  ct3: Ct is
  // the next GEMM's tripled operand [M][3N] (ldc = 3N), row = [hi | lo' | hi].
  int f16;
  float alpha;
  int ct3;
  // plain fp16 GEMM (SSE_DTYPE_FP16): A, B, Ct and resid_t are fp16 instead of bf16, the f16 MFMA, no
  // scale; otherwise exactly the bf16 path (launch_gemm<f16> sets it)
  int h16;
  // MX-fp8 out with ROW-MAJOR scales (launch_gemm8_mx): c_scale[m * (N / 32) + n / 32] instead of the A tile
  // layout (the fp8 attention's Q / K operand, read per row)
  int c_scale_rm;
  // bf16 out of launch_gemm8_mx: per-segment column amax of the stored values, atomicMax of the float bits of
  // max |bf16(C[m][n])| over the rows m of segment m / vamax_rows into vamax[(m / vamax_rows) * N + n] (the fp8
  // attention's per-(clip, column) V scale; the caller zeroes vamax)
  unsigned* vamax;
  int vamax_rows;
  // the fp8 attention's fused QKV GEMM (launch_gemm8_mx, n_split > 0): columns [0, n_split) are written as the
  // MX-fp8 Ct with row-major c_scale (ldc = n_split), columns [n_split, N) as bf16 into ct2 [M][ldc2] (column
  // n - n_split) with vamax over them (vamax[s][n - n_split])
  void* ct2;
  int n_split, ldc2;
};

// (mean, rstd) of a row of 256 * NT values from its per-tile partials (mean_t, M2_t), Chan's pairwise
// combination: mean = avg mean_t, M2 = sum M2_t + 256 sum (mean_t - mean)^2, rstd = 1 / sqrt(M2 / n + eps).
// Branch-free for a compile-time tile count (the folded path is enabled for H / 256 in {2, 3, 4}).
template <int NT>
SSE_DEV float2 ln_part_combine(const float2 (&v)[NT], float eps) {
  float mean = 0.f;
  #pragma unroll
  for (int t = 0; t < NT; ++t) mean += v[t].x;
  mean *= 1.0f / NT;
  float m2 = 0.f;
  #pragma unroll
  for (int t = 0; t < NT; ++t) {
    const float d = v[t].x - mean;
    m2 += v[t].y + 256.f * d * d;
  }
  // v_rsq_f32 (1 ulp) instead of the correctly rounded 1 / sqrtf (a ~20-instruction refinement sequence): the
  // folded epilogues take this per row and per lane (8 rows per lane per tile)
  return make_float2(mean, __builtin_amdgcn_rsqf(m2 * (1.0f / (256 * NT)) + eps));
}
template <int NT>
SSE_DEV float2 ln_part_stats_n(const float2* __restrict__ part, long long m, float eps) {
  float2 v[NT];
  #pragma unroll
  for (int t = 0; t < NT; ++t) v[t] = part[m * NT + t];
  return ln_part_combine<NT>(v, eps);
}
SSE_DEV float2 ln_part_stats(const float2* __restrict__ part, int nt, long long m, float eps) {
  switch (nt) {
    case 2: return ln_part_stats_n<2>(part, m, eps);
    case 4: return ln_part_stats_n<4>(part, m, eps);
    case 5: return ln_part_stats_n<5>(part, m, eps);
    default: return ln_part_stats_n<3>(part, m, eps);
  }
}

// ---- MX-fp8 scale layouts (both operands: K-tiles of 128, one E8M0 byte per 32-element block) ----
// The 8-phase MX GEMM stages, per 256-row (column) tile and K-tile, one 1 KiB scale block by
// LDS-DMA; inside it the bytes are ordered so that each lane's MFMA scales are one dword:
//   A rows   m = mi*128 + wm*64 + i*16 + r16 : [mi][wm][q][r16][i]   (q = block within the K-tile)
//   B cols   n = ni*128 + wn*32 + j*16 + r16 : [wn][q][r16][ni][j]
__host__ __device__ inline long long mx_a_scale_off(long long m, int blk, int kt) {
  return ((m >> 8) * kt + (blk >> 2)) * 1024 + ((((m >> 6) & 3) * 4 + (blk & 3)) * 16 + (m & 15)) * 4 + ((m >> 4) & 3);
}
__host__ __device__ inline long long mx_b_scale_off(long long n, int blk, int kt) {
  return ((n >> 8) * kt + (blk >> 2)) * 1024 + ((((n >> 5) & 3) * 4 + (blk & 3)) * 16 + (n & 15)) * 4 +
         ((n >> 7) & 1) * 2 + ((n >> 4) & 1);
}
// bytes of a scale tensor for R rows (columns) and K elements
__host__ __device__ inline long long mx_scale_bytes(long long R, int K) { return ((R + 255) / 256) * (K / 128) * 1024; }

// E8M0 exponent of a 32-element block with max |x| = amax: the smallest E with amax <= 448 * 2^E
// (448 = e4m3 max), clamped to [-127, 127]; returns the biased byte E + 127.
// For |amax| (bits u, sign masked off): be - 127 - (mantissa <= 0x600000 ? 8 : 7) biased by 127 is
// ((u + 0x1FFFFF) >> 23) - 8 (the mantissa test folded into the carry), clamped below at 0 (zero / denormal
// blocks: 2^-127); the upper clamp is never reached (be <= 255 gives <= 248).  The sign mask makes -0.0 or a
// negative input give the exponent of its magnitude instead of a byte past 255.  Four integer ops instead of nine.
__host__ __device__ inline int mx_scale_exp(float amax) {
  union { float f; unsigned u; } v;
  v.f = amax;
  const int e = (int)(((v.u & 0x7FFFFFFFu) + 0x1FFFFFu) >> 23) - 8;
  return e > 0 ? e : 0;
}
// max over the 8 lanes (lane & ~7) .. (lane | 7): DPP quad_perm xor 1, xor 2, then row_half_mirror
// (lane i <-> 7 - i within each 8-lane half-row swaps the two quads) -- VALU only, no LDS; IEEE maximum
// (fmaxf's maxnum would first canonicalise the DPP-moved operand: one more v_max per step)
SSE_DEV float max8_dpp(float v) {
  v = __builtin_elementwise_maximum(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true)));
  v = __builtin_elementwise_maximum(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true)));
  v = __builtin_elementwise_maximum(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, true)));
  return v;
}

// sum over the 64 lanes of a wave without LDS: DPP xor 1, xor 2, half-row mirror (8 lanes), row
// mirror (16 lanes), then v_permlane16_swap (32) and v_permlane32_swap (64); every lane gets the total
SSE_DEV float wave_sum_fast(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, true));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, true));
  const auto t16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(t16[0]) + __uint_as_float(t16[1]);
  const auto t32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(t32[0]) + __uint_as_float(t32[1]);
}

// 2^-(b - 127) as float (b in [0, 254]); exact (2^127 .. 2^-127, the last a denormal)
__host__ __device__ inline float mx_inv_scale(int b) {
  union { float f; unsigned u; } v;
  const int e = 127 - (b - 127);               // biased exponent of 2^(127 - b)
  if (e >= 1) { v.u = (unsigned)e << 23; return v.f; }
  v.u = 0x00400000u;                           // 2^-127
  return v.f;
}

// LayerNorm affine of one 4-column group, the exact expression of layernorm_kernel
SSE_DEV f32x4 ln_apply4(f32x4 v, float2 st, const float* w, const float* b, int n) {
  const f32x4 wv = *(const f32x4*)(w + n), bv = *(const f32x4*)(b + n);
  f32x4 o;
  #pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = fmaf((v[e] - st.x) * st.y, wv[e], bv[e]);
  return o;
}

enum { AMODE_SEG = 0, AMODE_CONV = 1 };

// Launchers (kernels_gemm.hip).  groups > 1 only with AMODE_CONV (grid.z = group).
int launch_gemm_bf16(const GemmArgs& a, int amode, int groups, hipStream_t s);
int launch_gemm_f32(const GemmArgs& a, int amode, int groups, hipStream_t s);

int launch_gemm8_bf16(const GemmArgs& a, hipStream_t s);   // kernels_gemm8.hip
int launch_gemm8_mx(const GemmArgs& a, hipStream_t s);     // kernels_gemm8.hip (MX-fp8 operands)
template <typename T> inline int launch_gemm(const GemmArgs& a, int amode, int groups, hipStream_t s);
template <> inline int launch_gemm<bf16>(const GemmArgs& a, int amode, int groups, hipStream_t s) {
  return launch_gemm_bf16(a, amode, groups, s);
}
template <> inline int launch_gemm<float>(const GemmArgs& a, int amode, int groups, hipStream_t s) {
  return launch_gemm_f32(a, amode, groups, s);
}
// fp16 operands: the 8-phase kernels only (N % 256 == 0, K % 64 == 0, SEG addressing); -3 otherwise
template <> inline int launch_gemm<f16>(const GemmArgs& a, int amode, int groups, hipStream_t s) {
  if (amode != AMODE_SEG || groups != 1 || a.f16 || a.ct3) return -3;
  GemmArgs g = a;
  g.h16 = 1;
  g.alpha = 1.f;
  return launch_gemm8_bf16(g, s);
}
