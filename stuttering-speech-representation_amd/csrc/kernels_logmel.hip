// K9: Whisper log-mel front end (HF/models/whisper/feature_extraction_whisper.py:135-168,
// 300-307; HF/audio_utils.py:638-740) on gfx950.
//
//   1. lm_pad:   zero-pad/truncate to 480000 samples, reflect-pad 200 each side  -> xp [B][480400]
//   2. DFT:      frames (row t = xp[160 t : 160 t + 400]) x windowed cos/sin basis [448][400]
//                on the exact-f32 MFMA GEMM (kernels_gemm.hip, SEG mode, rows overlap)  -> S [B*3000][448]
//   3. lm_mel:   |X|^2 -> Slaney mel (201 x n_mels, fp32 filters) -> log10(max(., 1e-10)), per-clip max
//   4. lm_final: max(x, max_clip - 8), (x + 4) / 4  -> [B][n_mels][3000] (HF layout) and/or
//                channels-last [B][3000][n_mels] in the encoder's element type (conv1 operand)
// The basis (Hann window folded in) and the filter bank are generated on device from the
// closed forms in fp64 into the workspace, so the call needs no host state or allocation.
#include "common.h"
#include "kernels_logmel.h"

namespace {

constexpr int N_FFT = 400, HOP = 160, PAD = 200, NS = 480000, NP = NS + 2 * PAD, NFR = 3000;
constexpr int NF = N_FFT / 2 + 1;   // 201 bins

__global__ void lm_pad_kernel(const float* __restrict__ x, int L, int Lv, float* __restrict__ xp,
                              const int* __restrict__ lens) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (i >= NP) return;
  if (lens) Lv = lens[b] < NS ? lens[b] : NS;   // ragged batch: the clip's own samples, zeros after
  int j = (int)i - PAD;
  if (j < 0) j = -j;
  if (j >= NS) j = 2 * (NS - 1) - j;
  xp[(long long)b * NP + i] = j < Lv ? x[(long long)b * L + j] : 0.f;
}

// basis[f][n] = hann(n) cos(2 pi f n / 400), basis[201 + f][n] = hann(n) sin(...), rest 0.
__global__ void lm_basis_kernel(float* __restrict__ basis) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= LM_NB * N_FFT) return;
  const int row = i / N_FFT, n = i - row * N_FFT;
  // torch.hann_window(400) (periodic), float32
  const float w = 0.5f - 0.5f * cosf(6.283185307179586f * (float)n / (float)N_FFT);
  double v = 0.0;
  if (row < NF) {
    v = cospi(2.0 * ((row * n) % N_FFT) / N_FFT);
  } else if (row < 2 * NF) {
    v = sinpi(2.0 * (((row - NF) * n) % N_FFT) / N_FFT);
  }
  basis[i] = (float)((double)w * v);
}

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

// support [first, last] of each mel filter's nonzero bins (triangular filters: contiguous)
__global__ void lm_support_kernel(const float* __restrict__ fb, int n_mels, int2* __restrict__ sup) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n_mels) return;
  int lo = NF, hi = -1;
  for (int f = 0; f < NF; ++f)
    if (fb[f * n_mels + m] != 0.f) {
      lo = f < lo ? f : lo;
      hi = f;
    }
  sup[m] = make_int2(lo, hi);
}

constexpr int MEL_FR = 20;   // frames per block (3000 = 150 x 20)
static_assert(NFR % MEL_FR == 0, "mel grid must cover every frame");

// mel = fb^T . |X|^2 over each filter's support only: the in-order fma chain over the support is
// bit-identical to the dense 201-bin chain (the other terms are fma(0, P, acc) = acc)
__global__ __launch_bounds__(256) void lm_mel_kernel(const float* __restrict__ S, const float* __restrict__ fb,
                                                     const int2* __restrict__ sup, int n_mels,
                                                     float* __restrict__ logv, unsigned* __restrict__ mx) {
  __shared__ float P[MEL_FR][NF + 3];
  const int b = blockIdx.y, t0 = blockIdx.x * MEL_FR;
  for (int i = threadIdx.x; i < MEL_FR * NF; i += 256) {
    const int fr = i / NF, f = i - fr * NF;
    const float* row = S + ((long long)b * NFR + t0 + fr) * LM_NB;
    const float re = row[f], im = row[NF + f];
    P[fr][f] = re * re + im * im;
  }
  __syncthreads();
  float lmax = -INFINITY;
  for (int i = threadIdx.x; i < MEL_FR * n_mels; i += 256) {
    const int fr = i / n_mels, m = i - fr * n_mels;
    float acc = 0.f;
    const int2 r = sup[m];
    for (int f = r.x; f <= r.y; ++f) acc = fmaf(fb[f * n_mels + m], P[fr][f], acc);
    const float v = log10f(fmaxf(acc, 1e-10f));
    logv[((long long)b * NFR + t0 + fr) * n_mels + m] = v;
    lmax = fmaxf(lmax, v);
  }
  lmax = wave_max(lmax);
  if ((threadIdx.x & 63) == 0) atomicMax(mx + b, ord_f32(lmax));
}

template <typename TO>
__global__ __launch_bounds__(256) void lm_final_kernel(const float* __restrict__ logv, const unsigned* __restrict__ mx,
                                                       int n_mels, float* __restrict__ out_hf, TO* __restrict__ out_cl) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const int b = blockIdx.y;
  if (i >= (long long)NFR * n_mels) return;
  const int t = (int)(i / n_mels), m = (int)(i - (long long)t * n_mels);
  const float cl = unord_f32(mx[b]) - 8.0f;
  const float v = (fmaxf(logv[(long long)b * NFR * n_mels + i], cl) + 4.0f) / 4.0f;
  if (out_hf) out_hf[((long long)b * n_mels + m) * NFR + t] = v;
  if (out_cl) out_cl[(long long)b * NFR * n_mels + i] = from_f32<TO>(v);
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
  return al((size_t)LM_NB * N_FFT * 4) + al((size_t)NF * n_mels * 4) + al((size_t)B * NP * 4) +
         al((size_t)B * NFR * LM_NB * 4) + al((size_t)B * NFR * n_mels * 4) + al((size_t)B * 4) + 256 +
         al((size_t)n_mels * 8);
}

template <typename TO>
int launch_logmel(const float* x, int B, int L, int n_mels, float* out_hf, TO* out_cl, void* ws, size_t ws_bytes,
                  hipStream_t s, const int* lens) {
  if (B <= 0 || L <= 0 || n_mels <= 0 || n_mels > 256) return -1;
  if (ws_bytes < logmel_workspace_bytes(B, n_mels)) return -4;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  char* p = (char*)ws;
  float* zero = (float*)p; p += 256;
  float* basis = (float*)p; p += al((size_t)LM_NB * N_FFT * 4);
  float* fb = (float*)p; p += al((size_t)NF * n_mels * 4);
  float* xp = (float*)p; p += al((size_t)B * NP * 4);
  float* S = (float*)p; p += al((size_t)B * NFR * LM_NB * 4);
  float* logv = (float*)p; p += al((size_t)B * NFR * n_mels * 4);
  unsigned* mx = (unsigned*)p; p += al((size_t)B * 4);
  int2* sup = (int2*)p;
  if (hipMemsetAsync(zero, 0, 256, s) != hipSuccess) return -2;
  if (hipMemsetAsync(mx, 0, (size_t)B * 4, s) != hipSuccess) return -2;
  hipLaunchKernelGGL(lm_basis_kernel, dim3((LM_NB * N_FFT + 255) / 256), dim3(256), 0, s, basis);
  hipLaunchKernelGGL(lm_filters_kernel, dim3((NF * n_mels + 255) / 256), dim3(256), 0, s, fb, n_mels);
  hipLaunchKernelGGL(lm_support_kernel, dim3((n_mels + 63) / 64), dim3(64), 0, s, fb, n_mels, sup);
  hipLaunchKernelGGL(lm_pad_kernel, dim3((NP + 255) / 256, B), dim3(256), 0, s, x, L, L < NS ? L : NS, xp, lens);
  if (hipGetLastError() != hipSuccess) return -2;
  GemmArgs g{};
  g.A = xp; g.B = basis; g.M = B * NFR; g.N = LM_NB; g.K = N_FFT;
  g.rows_per_seg = NFR; g.seg_stride = NP; g.lda = HOP;
  g.Cf = S; g.ldc = LM_NB; g.act = ACT_NONE; g.zero = zero;
  int rc = launch_gemm_f32(g, AMODE_SEG, 1, s);
  if (rc) return rc;
  hipLaunchKernelGGL(lm_mel_kernel, dim3(NFR / MEL_FR, B), dim3(256), 0, s, S, fb, sup, n_mels, logv, mx);
  hipLaunchKernelGGL((lm_final_kernel<TO>), dim3((NFR * n_mels + 255) / 256, B), dim3(256), 0, s, logv, mx, n_mels,
                     out_hf, out_cl);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
template int launch_logmel<float>(const float*, int, int, int, float*, float*, void*, size_t, hipStream_t,
                                  const int*);
template int launch_logmel<bf16>(const float*, int, int, int, float*, bf16*, void*, size_t, hipStream_t, const int*);
