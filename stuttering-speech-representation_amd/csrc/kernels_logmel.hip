// K9: Whisper log-mel front end (HF/models/whisper/feature_extraction_whisper.py:135-168,
// 300-307; HF/audio_utils.py:638-740) on gfx950, one fused pass per 20-frame block:
//
//   lm_stft_mel: the block's 3440 samples (zero-pad / truncate to 480000, reflect-pad 200 each side,
//                computed on the fly from the raw clip) staged in LDS once; per frame (one wave)
//                Hann window, the 400-point real DFT as a 200-point complex FFT of the even/odd
//                samples (Stockham radix 8 x 5 x 5 in LDS, fp32, twiddles from fp64) plus the
//                real-FFT split, |X|^2 (201 bins, LDS) -> Slaney mel over each filter's support ->
//                log10(max(., 1e-10)) -> logv [B][3000][n_mels], per-clip max (atomic)
//   lm_final:    max(x, max_clip - 8), (x + 4) / 4  -> [B][n_mels][3000] (HF layout) and/or
//                channels-last [B][3000][n_mels] in the encoder's element type (conv1 operand)
// HBM traffic per clip: the clip once (1.92 MB) + logv written and read back (0.96 MB each) + the
// output; the spectrum never leaves LDS.  The filter bank is generated on device in fp64.
#include "common.h"
#include "kernels_logmel.h"

namespace {

constexpr int N_FFT = 400, HOP = 160, PAD = 200, NS = 480000, NP = NS + 2 * PAD, NFR = 3000;
constexpr int NF = N_FFT / 2 + 1;   // 201 bins

__device__ double hz_to_mel(double f) {
  return f >= 1000.0 ? 15.0 + log(f / 1000.0) * (27.0 / log(6.4)) : 3.0 * f / 200.0;
}
__device__ double mel_to_hz(double m) {
  return m >= 15.0 ? 1000.0 * exp((log(6.4) / 27.0) * (m - 15.0)) : 200.0 * m / 3.0;
}

// Slaney mel filter bank [201][n_mels] (HF mel_filter_bank, norm="slaney", mel_scale="slaney")
__global__ void lm_filters_kernel(float* __restrict__ fb, int n_mels) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= NF * n_mels) return;
  const int f = i / n_mels, m = i - f * n_mels;
  const double mmin = hz_to_mel(0.0), mmax = hz_to_mel(8000.0);
  const double step = (mmax - mmin) / (n_mels + 1);
  const double f0 = mel_to_hz(mmin + step * m), f1 = mel_to_hz(mmin + step * (m + 1)),
               f2 = mel_to_hz(mmin + step * (m + 2));
  const double ff = 8000.0 * f / (NF - 1);
  const double down = (ff - f0) / (f1 - f0), up = (f2 - ff) / (f2 - f1);
  double v = fmin(down, up);
  v = v > 0.0 ? v : 0.0;
  fb[i] = (float)(v * (2.0 / (f2 - f0)));
}

__device__ __forceinline__ unsigned ord_f32(float v) {
  const unsigned u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord_f32(unsigned u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

constexpr int MAXSUP = 32;   // bins per Slaney filter (80 mels on 201 bins: at most 27)

// support [first, last] of each mel filter's nonzero bins (triangular filters: contiguous) and the
// filter's weights over it packed [n_mels][MAXSUP] (staged in LDS by the STFT kernel).  Block = one
// filter, a thread per bin (one load each, min / max of the nonzero bins in LDS).
__global__ __launch_bounds__(256) void lm_support_kernel(const float* __restrict__ fb, int n_mels,
                                                         int2* __restrict__ sup, float* __restrict__ fbp,
                                                         float* __restrict__ fbt) {
  __shared__ int lh[2];
  const int m = blockIdx.x, f = threadIdx.x;
  if (f == 0) { lh[0] = NF; lh[1] = -1; }
  __syncthreads();
  if (f < NF && fb[f * n_mels + m] != 0.f) {
    atomicMin(&lh[0], f);
    atomicMax(&lh[1], f);
  }
  __syncthreads();
  const int lo = lh[0];
  int hi = lh[1];
  if (hi - lo + 1 > MAXSUP) hi = lo + MAXSUP - 1;   // not reached for n_mels >= 64 (host checks n_mels)
  if (f == 0) sup[m] = make_int2(lo, hi);
  if (f < MAXSUP) {
    const float v = lo + f <= hi ? fb[(lo + f) * n_mels + m] : 0.f;
    fbp[m * MAXSUP + f] = v;
    fbt[f * n_mels + m] = v;   // [i][m]: the 4-frame kernel's LDS image, copied linearly (no strided LDS stores)
  }
}

constexpr int MEL_FR = 20;   // frames per block (3000 = 150 x 20), 5 per wave
static_assert(NFR % MEL_FR == 0, "mel grid must cover every frame");
constexpr int NZ = N_FFT / 2;                       // 200-point complex FFT
constexpr int SPAN = HOP * (MEL_FR - 1) + N_FFT;    // 3440 samples per block

// twiddles W_200^k = exp(-2 pi i k / 200) and the real-split W_400^k, k < 200, from fp64; then the
// Hann window as (w[2n], w[2n+1]) pairs (torch.hann_window(400), periodic, evaluated in float32)
__global__ void lm_twiddle_kernel(float2* __restrict__ tw, unsigned* __restrict__ mx, int B) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  for (int b = k; b < B; b += gridDim.x * blockDim.x) mx[b] = 0u;   // per-clip maxima (ord_f32(-inf) > 0)
  if (k < 2 * NZ) {
    const double a = k < NZ ? -2.0 * (double)k / NZ : -2.0 * (double)(k - NZ) / N_FFT;   // in units of pi
    tw[k] = make_float2((float)cospi(a), (float)sinpi(a));
  } else if (k < 3 * NZ) {
    const int n = k - 2 * NZ;
    tw[k] = make_float2(0.5f - 0.5f * cosf(6.283185307179586f * (float)(2 * n) / (float)N_FFT),
                        0.5f - 0.5f * cosf(6.283185307179586f * (float)(2 * n + 1) / (float)N_FFT));
  }
}

SSE_DEV float2 cmul(float2 a, float2 b) { return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }

// one radix-R Stockham stage over NZ points (span Ns so far): lane j < NZ/R does butterfly j
template <int R>
SSE_DEV void fft_stage(const float2* __restrict__ x, float2* __restrict__ y, int Ns, const float2* __restrict__ tw,
                       int lane) {
  constexpr int NB = NZ / R;
  if (lane < NB) {
    const int j = lane, k = j % Ns;
    float2 v[R];
    #pragma unroll
    for (int r = 0; r < R; ++r) {
      v[r] = x[j + r * NB];
      if (r) v[r] = cmul(v[r], tw[(k * r * (NZ / (Ns * R))) % NZ]);   // W_{Ns R}^{k r}
    }
    float2 o[R];
    if constexpr (R == 8) {   // 8-point DFT as radix 2 x 2 x 2 (constant twiddles)
      const float h = 0.70710678118654752f;
      float2 a[8];
      #pragma unroll
      for (int r = 0; r < 4; ++r) {
        a[r] = make_float2(v[r].x + v[r + 4].x, v[r].y + v[r + 4].y);
        a[r + 4] = make_float2(v[r].x - v[r + 4].x, v[r].y - v[r + 4].y);
      }
      // twiddles W_8^r on the odd half: 1, (1 - i) h, -i, (-1 - i) h
      a[5] = make_float2((a[5].x + a[5].y) * h, (a[5].y - a[5].x) * h);
      a[6] = make_float2(a[6].y, -a[6].x);
      a[7] = make_float2((a[7].y - a[7].x) * h, -(a[7].x + a[7].y) * h);
      float2 c[8];
      #pragma unroll
      for (int g = 0; g < 2; ++g) {
        const int b0 = 4 * g;
        c[b0 + 0] = make_float2(a[b0].x + a[b0 + 2].x, a[b0].y + a[b0 + 2].y);
        c[b0 + 2] = make_float2(a[b0].x - a[b0 + 2].x, a[b0].y - a[b0 + 2].y);
        c[b0 + 1] = make_float2(a[b0 + 1].x + a[b0 + 3].x, a[b0 + 1].y + a[b0 + 3].y);
        const float2 t = make_float2(a[b0 + 1].x - a[b0 + 3].x, a[b0 + 1].y - a[b0 + 3].y);
        c[b0 + 3] = make_float2(t.y, -t.x);   // * W_4^1 = -i
      }
      // last radix-2 level; bit-reversed order -> natural
      o[0] = make_float2(c[0].x + c[1].x, c[0].y + c[1].y);
      o[4] = make_float2(c[0].x - c[1].x, c[0].y - c[1].y);
      o[2] = make_float2(c[2].x + c[3].x, c[2].y + c[3].y);
      o[6] = make_float2(c[2].x - c[3].x, c[2].y - c[3].y);
      o[1] = make_float2(c[4].x + c[5].x, c[4].y + c[5].y);
      o[5] = make_float2(c[4].x - c[5].x, c[4].y - c[5].y);
      o[3] = make_float2(c[6].x + c[7].x, c[6].y + c[7].y);
      o[7] = make_float2(c[6].x - c[7].x, c[6].y - c[7].y);
    } else {
      #pragma unroll
      for (int q = 0; q < R; ++q) {   // R-point DFT, W_R^{q r} = W_200^{q r NZ / R}
        float2 acc = v[0];
        #pragma unroll
        for (int r = 1; r < R; ++r) {
          const float2 w = tw[((q * r) % R) * (NZ / R)];
          acc.x = fmaf(v[r].x, w.x, fmaf(-v[r].y, w.y, acc.x));
          acc.y = fmaf(v[r].x, w.y, fmaf(v[r].y, w.x, acc.y));
        }
        o[q] = acc;
      }
    }
    const int d = (j / Ns) * Ns * R + k;
    #pragma unroll
    for (int q = 0; q < R; ++q) y[d + q * Ns] = o[q];
  }
}

__global__ __launch_bounds__(256) void lm_stft_mel_kernel(const float* __restrict__ wave, int L, int Lv0,
                                                          const int* __restrict__ lens, const float2* __restrict__ twg,
                                                          const float* __restrict__ fbp, const int2* __restrict__ sup,
                                                          int n_mels, float* __restrict__ logv,
                                                          unsigned* __restrict__ mx) {
  __shared__ float xs[SPAN];
  __shared__ float2 tw[3 * NZ];   // W_200^k | W_400^k | Hann pairs
  const float2* win = tw + 2 * NZ;
  __shared__ float2 za[4][NZ], zb[4][NZ];
  __shared__ float P[4][NF + 3];
  __shared__ float fw[LM_MAXMEL * MAXSUP];   // packed filter weights
  __shared__ int2 fs[LM_MAXMEL];
  const int b = blockIdx.y, t0 = blockIdx.x * MEL_FR;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int Lv = lens ? min(max(lens[b], 0), Lv0) : Lv0;   // the clip's samples (clamped to [0, min(L, NS)]), zeros after
  const float* xw = wave + (long long)b * L;
  for (int i = threadIdx.x; i < SPAN; i += 256) {   // padded index HOP t0 + i -> reflect -> zero-pad
    int j = HOP * t0 + i - PAD;
    if (j < 0) j = -j;
    if (j >= NS) j = 2 * (NS - 1) - j;
    xs[i] = j < Lv ? xw[j] : 0.f;
  }
  for (int i = threadIdx.x; i < 3 * NZ; i += 256) tw[i] = twg[i];
  for (int i = threadIdx.x; i < n_mels * MAXSUP; i += 256) fw[i] = fbp[i];
  for (int i = threadIdx.x; i < n_mels; i += 256) fs[i] = sup[i];
  __syncthreads();
  float lmax = -INFINITY;
  // each wave owns its frame buffers: stages are ordered by a wave-local LDS fence, not a block barrier
  auto wsync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  for (int f = 0; f < MEL_FR / 4; ++f) {
    const int fr = wv * (MEL_FR / 4) + f;
    const float* xf = xs + HOP * fr;
    // z[n] = w[2n] x[2n] + i w[2n+1] x[2n+1]  (torch.hann_window(400), periodic, float32)
    for (int n = lane; n < NZ; n += 64) {
      const float2 w = win[n];
      za[wv][n] = make_float2(w.x * xf[2 * n], w.y * xf[2 * n + 1]);
    }
    wsync();
    fft_stage<8>(za[wv], zb[wv], 1, tw, lane);
    wsync();
    fft_stage<5>(zb[wv], za[wv], 8, tw, lane);
    wsync();
    fft_stage<5>(za[wv], zb[wv], 40, tw, lane);
    wsync();
    // real split: X[k] = (Z[k] + conj Z[N-k]) / 2 - i W_400^k (Z[k] - conj Z[N-k]) / 2, k = 0..200
    for (int k = lane; k < NF; k += 64) {
      float px;
      if (k == 0 || k == NZ) {
        const float2 z0 = zb[wv][0];
        const float xr = k == 0 ? z0.x + z0.y : z0.x - z0.y;
        px = xr * xr;
      } else {
        const float2 a = zb[wv][k], c = zb[wv][NZ - k];
        const float2 e = make_float2(0.5f * (a.x + c.x), 0.5f * (a.y - c.y));   // (Z[k] + conj Z[N-k]) / 2
        const float2 o = make_float2(0.5f * (a.x - c.x), 0.5f * (a.y + c.y));   // (Z[k] - conj Z[N-k]) / 2
        const float2 wo = cmul(tw[NZ + k], o);                                  // W_400^k o
        const float xr = e.x + wo.y, xi = e.y - wo.x;                           // e - i wo
        px = xr * xr + xi * xi;
      }
      P[wv][k] = px;
    }
    wsync();
    for (int m = lane; m < n_mels; m += 64) {
      // in-order fma chain over the filter's support: bit-identical to the dense 201-bin chain (the
      // other terms are fma(0, P, acc) = acc)
      // fixed MAXSUP-long chain with zero weights past the support (all LDS reads issued together)
      float acc = 0.f;
      const int lo = fs[m].x;
      #pragma unroll
      for (int i = 0; i < MAXSUP; ++i) {
        const int k = lo + i < NF ? lo + i : NF - 1;
        acc = fmaf(fw[m * MAXSUP + i], P[wv][k], acc);
      }
      const float v = log10f(fmaxf(acc, 1e-10f));
      logv[((long long)b * NFR + t0 + fr) * n_mels + m] = v;
      lmax = fmaxf(lmax, v);
    }
  }
  lmax = wave_max(lmax);
  if (lane == 0) atomicMax(mx + b, ord_f32(lmax));
}

// ---- round 3: four frames per wave, every lane busy -------------------------------------------------
// The one-frame-per-wave kernel above keeps 25 / 40 of 64 lanes busy in the radix-8 / radix-5 stages and
// 201 / 80 in the split / mel loops, so it is VALU-issue bound at ~40 % lane occupancy.  Here a wave
// transforms LM_F = 4 frames together: every stage's (frame, butterfly) tasks are spread over the 64
// lanes (radix 8: 100 tasks, radix 5: 160, split: 804, mel: 4 n_mels), each stage runs in place in one
// [LM_F][200] complex LDS buffer per wave -- all of a stage's inputs are read into registers, a wave
// barrier, then the outputs written (Stockham order, no ping-pong buffer) -- and the radix-5 butterfly
// is the 5-point Winograd form (~36 flops instead of 80).  Block = 5 waves = 20 frames, the same grid.
constexpr int LM_F = 4, LM_W = 5;
static_assert(LM_F * LM_W == MEL_FR, "block = 20 frames");

// 5-point DFT, W = exp(-2 pi i / 5): y_q = sum_r x_r W^(q r)
SSE_DEV void dft5(const float2 (&x)[5], float2 (&y)[5]) {
  const float c1 = 0.30901699437494742f, c2 = -0.80901699437494742f;   // cos 72, cos 144
  const float s1 = 0.95105651629515357f, s2 = 0.58778525229247313f;    // sin 72, sin 144
  const float2 t1 = make_float2(x[1].x + x[4].x, x[1].y + x[4].y), t2 = make_float2(x[2].x + x[3].x, x[2].y + x[3].y);
  const float2 t3 = make_float2(x[1].x - x[4].x, x[1].y - x[4].y), t4 = make_float2(x[2].x - x[3].x, x[2].y - x[3].y);
  y[0] = make_float2(x[0].x + t1.x + t2.x, x[0].y + t1.y + t2.y);
  const float2 a = make_float2(fmaf(c2, t2.x, fmaf(c1, t1.x, x[0].x)), fmaf(c2, t2.y, fmaf(c1, t1.y, x[0].y)));
  const float2 b = make_float2(fmaf(c1, t2.x, fmaf(c2, t1.x, x[0].x)), fmaf(c1, t2.y, fmaf(c2, t1.y, x[0].y)));
  const float2 d = make_float2(fmaf(s2, t4.x, s1 * t3.x), fmaf(s2, t4.y, s1 * t3.y));     // s1 t3 + s2 t4
  const float2 e = make_float2(fmaf(-s1, t4.x, s2 * t3.x), fmaf(-s1, t4.y, s2 * t3.y));   // s2 t3 - s1 t4
  // y1 = a - i d, y4 = a + i d, y2 = b - i e, y3 = b + i e
  y[1] = make_float2(a.x + d.y, a.y - d.x);
  y[4] = make_float2(a.x - d.y, a.y + d.x);
  y[2] = make_float2(b.x + e.y, b.y - e.x);
  y[3] = make_float2(b.x - e.y, b.y + e.x);
}

SSE_DEV void dft8(const float2 (&v)[8], float2 (&o)[8]) {   // radix 2 x 2 x 2 (constant twiddles)
  const float h = 0.70710678118654752f;
  float2 a[8];
  #pragma unroll
  for (int r = 0; r < 4; ++r) {
    a[r] = make_float2(v[r].x + v[r + 4].x, v[r].y + v[r + 4].y);
    a[r + 4] = make_float2(v[r].x - v[r + 4].x, v[r].y - v[r + 4].y);
  }
  a[5] = make_float2((a[5].x + a[5].y) * h, (a[5].y - a[5].x) * h);
  a[6] = make_float2(a[6].y, -a[6].x);
  a[7] = make_float2((a[7].y - a[7].x) * h, -(a[7].x + a[7].y) * h);
  float2 c[8];
  #pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int b0 = 4 * g;
    c[b0 + 0] = make_float2(a[b0].x + a[b0 + 2].x, a[b0].y + a[b0 + 2].y);
    c[b0 + 2] = make_float2(a[b0].x - a[b0 + 2].x, a[b0].y - a[b0 + 2].y);
    c[b0 + 1] = make_float2(a[b0 + 1].x + a[b0 + 3].x, a[b0 + 1].y + a[b0 + 3].y);
    const float2 t = make_float2(a[b0 + 1].x - a[b0 + 3].x, a[b0 + 1].y - a[b0 + 3].y);
    c[b0 + 3] = make_float2(t.y, -t.x);
  }
  o[0] = make_float2(c[0].x + c[1].x, c[0].y + c[1].y);
  o[4] = make_float2(c[0].x - c[1].x, c[0].y - c[1].y);
  o[2] = make_float2(c[2].x + c[3].x, c[2].y + c[3].y);
  o[6] = make_float2(c[2].x - c[3].x, c[2].y - c[3].y);
  o[1] = make_float2(c[4].x + c[5].x, c[4].y + c[5].y);
  o[5] = make_float2(c[4].x - c[5].x, c[4].y - c[5].y);
  o[3] = make_float2(c[6].x + c[7].x, c[6].y + c[7].y);
  o[7] = make_float2(c[6].x - c[7].x, c[6].y - c[7].y);
}

SSE_DEV void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// one radix-R Stockham stage (span Ns so far) over the wave's LM_F frames, in place: task = (frame,
// butterfly j), lane-strided; inputs into registers, wave barrier, outputs
template <int R>
SSE_DEV void fft_stage4(float2* __restrict__ z, int Ns, const float2* __restrict__ tw, int lane) {
  constexpr int NB = NZ / R, NT = LM_F * NB, IT = (NT + 63) / 64;
  float2 v[IT][R];
  #pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int task = lane + 64 * it;
    if (task < NT) {
      const int f = task / NB, j = task - f * NB, k = j % Ns;
      const float2* zf = z + f * NZ;
      #pragma unroll
      for (int r = 0; r < R; ++r) {
        v[it][r] = zf[j + r * NB];
        if (r) v[it][r] = cmul(v[it][r], tw[(k * r * (NZ / (Ns * R))) % NZ]);   // W_{Ns R}^{k r}
      }
    }
  }
  wave_lds_sync();
  #pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int task = lane + 64 * it;
    if (task < NT) {
      const int f = task / NB, j = task - f * NB, k = j % Ns;
      float2 o[R];
      if constexpr (R == 8) dft8(v[it], o);
      else dft5(v[it], o);
      float2* zf = z + f * NZ + (j / Ns) * Ns * R + k;
      #pragma unroll
      for (int q = 0; q < R; ++q) zf[q * Ns] = o[q];
    }
  }
  wave_lds_sync();
}

// Block = one 20-frame chunk (a persistent form walking chunks with the next chunk's samples prefetched
// into registers measured slower: 0.78 vs 0.61 ms for 128 x 30 s -- its per-chunk block barriers
// serialise the waves that separate blocks on a CU keep out of phase).
constexpr int LM_CPC = NFR / MEL_FR;   // chunks per clip
__global__ __launch_bounds__(64 * LM_W) void lm_stft_mel4_kernel(const float* __restrict__ wave, int B, int L, int Lv0,
                                                                 const int* __restrict__ lens,
                                                                 const float2* __restrict__ twg,
                                                                 const float* __restrict__ fbp,
                                                                 const int2* __restrict__ sup, int n_mels,
                                                                 float* __restrict__ logv, unsigned* __restrict__ mx) {
  constexpr int NTH = 64 * LM_W;
  // dynamic LDS (47.7 KB at 80 mels: three blocks per CU): the frame buffers, whose first 13.8 KB also
  // hold the chunk's samples until every wave has read its window (one block barrier) | twiddles |
  // filter weights transposed [i][m] (lanes of consecutive m read consecutive words; the [m][i] image
  // is a 32-word stride, every lane of a pass on one bank) | each filter's first bin and support length
  extern __shared__ __attribute__((aligned(16))) char lsm[];
  float2 (*zbuf)[LM_F * NZ] = (float2 (*)[LM_F * NZ])lsm;
  float* xs = (float*)lsm;
  static_assert(SPAN * 4 <= LM_W * LM_F * NZ * 8, "samples alias the frame buffers");
  float2* tw = (float2*)(lsm + LM_W * LM_F * NZ * 8);   // W_200^k | W_400^k | Hann pairs
  float* fwt = (float*)(tw + 3 * NZ);
  int* fs = (int*)(fwt + MAXSUP * n_mels);
  int* fsn = fs + n_mels;
  static_assert(LM_F == 4, "mel task split m = task >> 2");
  const float2* win = tw + 2 * NZ;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nch = B * LM_CPC;
  constexpr int NX = (SPAN + NTH - 1) / NTH;
  float xr[NX];
  // samples of chunk c (zero-pad / truncate to 480000, reflect-pad 200) into registers
  auto load_chunk = [&](int c) {
    const int b = c / LM_CPC, t0 = (c - b * LM_CPC) * MEL_FR;
    const int Lv = lens ? min(max(lens[b], 0), Lv0) : Lv0;   // clamped to [0, min(L, NS)]
    const float* xw = wave + (long long)b * L;
    #pragma unroll
    for (int u = 0; u < NX; ++u) {
      const int i = threadIdx.x + u * NTH;
      int j = HOP * t0 + i - PAD;
      if (j < 0) j = -j;
      if (j >= NS) j = 2 * (NS - 1) - j;
      xr[u] = (i < SPAN && j < Lv) ? xw[j] : 0.f;
    }
  };
  const int c = blockIdx.x;
  if (c >= nch) return;
  load_chunk(c);
  {   // tables: every global load issued before the first LDS write
    constexpr int NTW = (3 * NZ + NTH - 1) / NTH, NFW = (LM_MAXMEL * MAXSUP + NTH - 1) / NTH;
    float fr[NFW];
    float2 tr[NTW];
    #pragma unroll
    for (int u = 0; u < NTW; ++u) {
      const int i = threadIdx.x + u * NTH;
      tr[u] = i < 3 * NZ ? twg[i] : make_float2(0.f, 0.f);
    }
    #pragma unroll
    for (int u = 0; u < NFW; ++u) {
      const int i = threadIdx.x + u * NTH;
      fr[u] = i < n_mels * MAXSUP ? fbp[i] : 0.f;
    }
    const int2 sv = threadIdx.x < n_mels ? sup[threadIdx.x] : make_int2(0, -1);
    #pragma unroll
    for (int u = 0; u < NTW; ++u) {
      const int i = threadIdx.x + u * NTH;
      if (i < 3 * NZ) tw[i] = tr[u];
    }
    #pragma unroll
    for (int u = 0; u < NFW; ++u) {
      const int i = threadIdx.x + u * NTH;
      if (i < n_mels * MAXSUP) fwt[i] = fr[u];
    }
    if (threadIdx.x < n_mels) {
      fs[threadIdx.x] = sv.x;
      fsn[threadIdx.x] = sv.y - sv.x + 1;   // lm_support_kernel: hi - lo + 1 <= MAXSUP, 0 for an empty filter
    }
  }
  float2* z = zbuf[wv];
  const int fr0 = wv * LM_F;   // the wave's first frame within the chunk
  {
    const int b = c / LM_CPC, t0 = (c - b * LM_CPC) * MEL_FR;
    #pragma unroll
    for (int u = 0; u < NX; ++u) {
      const int i = threadIdx.x + u * NTH;
      if (i < SPAN) xs[i] = xr[u];
    }
    __syncthreads();
    // z_f[n] = w[2n] x[2n] + i w[2n+1] x[2n+1]: windowed into registers, then (every wave done with the
    // samples the frame buffers alias) stored
    constexpr int NWT = (LM_F * NZ + 63) / 64;
    float2 zw[NWT];
    #pragma unroll
    for (int it = 0; it < NWT; ++it) {
      const int task = lane + 64 * it;
      if (task < LM_F * NZ) {
        const int f = task / NZ, n = task - f * NZ;
        const float2 x2 = *(const float2*)(xs + HOP * (fr0 + f) + 2 * n);
        const float2 w = win[n];
        zw[it] = make_float2(w.x * x2.x, w.y * x2.y);
      }
    }
    __syncthreads();
    #pragma unroll
    for (int it = 0; it < NWT; ++it) {
      const int task = lane + 64 * it;
      if (task < LM_F * NZ) z[task] = zw[it];
    }
    wave_lds_sync();
    fft_stage4<8>(z, 1, tw, lane);
    fft_stage4<5>(z, 8, tw, lane);
    fft_stage4<5>(z, 40, tw, lane);
    // real split + |X|^2 (201 bins per frame) into the same buffer, as floats [LM_F][NF + 3]
    constexpr int NSP = LM_F * NF, ISP = (NSP + 63) / 64;
    float pw[ISP];
    #pragma unroll
    for (int it = 0; it < ISP; ++it) {
      const int task = lane + 64 * it;
      pw[it] = 0.f;
      if (task < NSP) {
        const int f = task / NF, k = task - f * NF;
        const float2* zf = z + f * NZ;
        if (k == 0 || k == NZ) {
          const float2 z0 = zf[0];
          const float xr0 = k == 0 ? z0.x + z0.y : z0.x - z0.y;
          pw[it] = xr0 * xr0;
        } else {
          const float2 a = zf[k], cc = zf[NZ - k];
          const float2 e = make_float2(0.5f * (a.x + cc.x), 0.5f * (a.y - cc.y));
          const float2 o = make_float2(0.5f * (a.x - cc.x), 0.5f * (a.y + cc.y));
          const float2 wo = cmul(tw[NZ + k], o);
          const float xre = e.x + wo.y, xim = e.y - wo.x;
          pw[it] = xre * xre + xim * xim;
        }
      }
    }
    wave_lds_sync();
    float* P = (float*)z;
    constexpr int PST = NF + 3;
    #pragma unroll
    for (int it = 0; it < ISP; ++it) {
      const int task = lane + 64 * it;
      if (task < NSP) {
        const int f = task / NF, k = task - f * NF;
        P[f * PST + k] = pw[it];
      }
    }
    wave_lds_sync();
    // mel: task = (mel m, frame f), m-major, so a 64-lane pass holds 16 neighbouring filters of similar
    // width; each lane sums only its filter's support [lo, hi] (in order: the same fp32 chain as the dense
    // 201-bin sum, whose other terms are fma(0, P, acc) = acc), the pass runs as long as its widest filter
    float lmax = -INFINITY;
    for (int task = lane; task < LM_F * n_mels; task += 64) {
      const int m = task >> 2, f = task & (LM_F - 1);
      const float* Pf = P + f * PST + fs[m];
      const int n = fsn[m];
      float acc = 0.f;
      for (int i = 0; i < n; ++i) acc = fmaf(fwt[i * n_mels + m], Pf[i], acc);
      const float v = log10f(fmaxf(acc, 1e-10f));
      logv[((long long)b * NFR + t0 + fr0 + f) * n_mels + m] = v;
      lmax = fmaxf(lmax, v);
    }
    lmax = wave_max(lmax);
    if (lane == 0) atomicMax(mx + b, ord_f32(lmax));
  }
}

// 64 frames x n_mels per block: channels-last output straight through (coalesced), the HF layout
// [B][n_mels][3000] through an LDS transpose so its 64-frame rows are coalesced too
constexpr int FIN_T = 64;
template <typename TO>
__global__ __launch_bounds__(256) void lm_final_kernel(const float* __restrict__ logv, const unsigned* __restrict__ mx,
                                                       int n_mels, float* __restrict__ out_hf, TO* __restrict__ out_cl) {
  __shared__ float tile[LM_MAXMEL][FIN_T + 1];
  const int b = blockIdx.y, t0 = blockIdx.x * FIN_T;
  const int nt = NFR - t0 < FIN_T ? NFR - t0 : FIN_T;
  const float cl = unord_f32(mx[b]) - 8.0f;
  const float* src = logv + ((long long)b * NFR + t0) * n_mels;
  for (int i = threadIdx.x; i < nt * n_mels; i += 256) {
    const int t = i / n_mels, m = i - t * n_mels;
    const float v = (fmaxf(src[i], cl) + 4.0f) / 4.0f;
    if (out_cl) out_cl[((long long)b * NFR + t0) * n_mels + i] = from_f32<TO>(v);
    tile[m][t] = v;
  }
  if (!out_hf) return;
  __syncthreads();
  for (int i = threadIdx.x; i < n_mels * FIN_T; i += 256) {
    const int m = i / FIN_T, t = i - m * FIN_T;
    if (t < nt) out_hf[((long long)b * n_mels + m) * NFR + t0 + t] = tile[m][t];
  }
}

template <typename TO>
__global__ __launch_bounds__(256) void mel_to_cl_kernel(const float* __restrict__ mel, int n_mels, TO* __restrict__ out) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const int b = blockIdx.y;
  if (i >= (long long)NFR * n_mels) return;
  const int t = (int)(i / n_mels), m = (int)(i - (long long)t * n_mels);
  out[(long long)b * NFR * n_mels + i] = from_f32<TO>(mel[((long long)b * n_mels + m) * NFR + t]);
}

__global__ __launch_bounds__(256) void normalize_apply_kernel(const float* __restrict__ x, int L,
                                                              const float* __restrict__ st, float* __restrict__ y) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const int b = blockIdx.y;
  if (i >= L) return;
  y[(long long)b * L + i] = (x[(long long)b * L + i] - st[2 * b]) * st[2 * b + 1];
}

}  // namespace

template <typename TO>
int launch_mel_to_cl(const float* mel_hf, int B, int n_mels, TO* out_cl, hipStream_t s) {
  hipLaunchKernelGGL((mel_to_cl_kernel<TO>), dim3((NFR * n_mels + 255) / 256, B), dim3(256), 0, s, mel_hf, n_mels,
                     out_cl);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
template int launch_mel_to_cl<float>(const float*, int, int, float*, hipStream_t);
template int launch_mel_to_cl<bf16>(const float*, int, int, bf16*, hipStream_t);

int launch_normalize_apply(const float* x, int B, int L, const float* st, float* y, hipStream_t s) {
  hipLaunchKernelGGL(normalize_apply_kernel, dim3((L + 255) / 256, B), dim3(256), 0, s, x, L, st, y);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

size_t logmel_workspace_bytes(int B, int n_mels) {
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  return al((size_t)3 * NZ * 8) + al((size_t)NF * n_mels * 4) + al((size_t)B * NFR * n_mels * 4) + al((size_t)B * 4) +
         al((size_t)n_mels * 8) + 2 * al((size_t)n_mels * MAXSUP * 4);
}

template <typename TO>
int launch_logmel(const float* x, int B, int L, int n_mels, float* out_hf, TO* out_cl, void* ws, size_t ws_bytes,
                  hipStream_t s, const int* lens) {
  if (B <= 0 || L <= 0 || n_mels < 64 || n_mels > LM_MAXMEL) return -1;   // Whisper: 80 or 128 mels
  if (ws_bytes < logmel_workspace_bytes(B, n_mels)) return -4;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  char* p = (char*)ws;
  float2* tw = (float2*)p; p += al((size_t)3 * NZ * 8);
  float* fb = (float*)p; p += al((size_t)NF * n_mels * 4);
  float* logv = (float*)p; p += al((size_t)B * NFR * n_mels * 4);
  unsigned* mx = (unsigned*)p; p += al((size_t)B * 4);
  int2* sup = (int2*)p; p += al((size_t)n_mels * 8);
  float* fbp = (float*)p; p += al((size_t)n_mels * MAXSUP * 4);
  float* fbt = (float*)p;
  hipLaunchKernelGGL(lm_twiddle_kernel, dim3((3 * NZ + 255) / 256), dim3(256), 0, s, tw, mx, B);
  hipLaunchKernelGGL(lm_filters_kernel, dim3((NF * n_mels + 255) / 256), dim3(256), 0, s, fb, n_mels);
  hipLaunchKernelGGL(lm_support_kernel, dim3(n_mels), dim3(256), 0, s, fb, n_mels, sup, fbp, fbt);
  if (sse_opt(OPT_LOGMEL_V1))
    hipLaunchKernelGGL(lm_stft_mel_kernel, dim3(NFR / MEL_FR, B), dim3(256), 0, s, x, L, L < NS ? L : NS, lens, tw, fbp,
                       sup, n_mels, logv, mx);
  else
  {
    const size_t lds = (size_t)LM_W * LM_F * NZ * 8 + 3 * NZ * 8 + (size_t)MAXSUP * n_mels * 4 + (size_t)n_mels * 8;
    hipLaunchKernelGGL(lm_stft_mel4_kernel, dim3(B * LM_CPC), dim3(64 * LM_W), lds, s, x, B, L, L < NS ? L : NS, lens, tw,
                       fbt, sup, n_mels, logv, mx);
  }
  hipLaunchKernelGGL((lm_final_kernel<TO>), dim3((NFR + FIN_T - 1) / FIN_T, B), dim3(256), 0, s, logv, mx, n_mels,
                     out_hf, out_cl);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
template int launch_logmel<float>(const float*, int, int, int, float*, float*, void*, size_t, hipStream_t,
                                  const int*);
template int launch_logmel<bf16>(const float*, int, int, int, float*, bf16*, void*, size_t, hipStream_t, const int*);
