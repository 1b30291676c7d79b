// Pitch-shift augmentation of model_training_01's augment_audio (REF/model_training_01.py:172-177,
// SURVEY §8(f) next-4): torchaudio.transforms.PitchShift(sample_rate, n_steps) with its defaults
// (bins_per_octave 12, n_fft 512, win 512 periodic Hann, hop 128).  torchaudio is absent from the
// image; the published algorithm (torchaudio.functional.pitch_shift = _stretch_waveform +
// resample + _fix_waveform_shape, 2.x) is, with rate = 2^(-n_steps/12):
//   X   = stft(x, center, reflect pad)                  [T = 1 + L/128 frames][257 bins]
//   Y   = phase_vocoder(X, rate, linspace(0, pi*128, 257))   [nnew = ceil(T/rate) frames]
//   xs  = istft(Y, length = round(L/rate))
//   out = resample(xs, int(sr/rate) -> sr), truncated / zero padded to L
// Device layout: spectra are [clip][frame][bin] float2 (bins contiguous: the vocoder's lanes walk
// bins, so every frame step is one coalesced 2 KiB row per clip).  One 256-thread block transforms
// one 512-sample frame with a radix-2 FFT in LDS (twiddles from sincospi in fp64); the vocoder
// runs one lane per (clip, bin) down the frames, accumulating the phase in fp64 like torch's CPU
// cumsum; the overlap-add is a gather (4 frames per output sample, no atomics: deterministic);
// the resample back reuses the polyphase-GEMM resampler (kernels_ingest.hip).
// The vocoder's float32 element-wise chain is kept un-contracted (no FMA) and its two tables
// (arange time steps, linspace phase advance) follow ATen's CPU kernels, so the discrete choices
// (frame index, interpolation weight, phase wrap) are those of the reference run on a CPU.
#include <cmath>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int PS_NFFT = 512, PS_HOP = 128, PS_BINS = 257;
constexpr float PS_TWO_PI = 6.283185307179586f;   // python 2 * math.pi as a float32 tensor scalar

SSE_DEV int brev9(int k) { return (int)(__builtin_bitreverse32((unsigned)k) >> 23); }

// torch.hann_window(512) (periodic): arange(513) * float(2pi/512) -> cos -> * -0.5 -> + 0.5, float32
SSE_DEV float hann512(int n) {
#pragma clang fp contract(off)
  const float c = cosf((float)n * (float)(M_PI * 2.0 / 512.0));
  return c * -0.5f + 0.5f;
}

SSE_DEV void twiddles(float2* tw, int tid) {   // tw[k] = exp(-2 pi i k / 512), k < 256
  double s, c;
  sincospi(-(double)tid / 256.0, &s, &c);
  tw[tid] = make_float2((float)c, (float)s);
}

// In-place 512-point DIF FFT over z (256 threads), output in bit-reversed order.
SSE_DEV void fft512(float2* z, const float2* tw, int tid) {
  #pragma unroll
  for (int h = 256; h >= 1; h >>= 1) {
    __syncthreads();
    const int j = tid & (h - 1), a = ((tid - j) << 1) + j, b = a + h;
    const float2 u = z[a], v = z[b], w = tw[j * (256 / h)];
    const float dx = u.x - v.x, dy = u.y - v.y;
    z[a] = make_float2(u.x + v.x, u.y + v.y);
    z[b] = make_float2(dx * w.x - dy * w.y, dx * w.y + dy * w.x);
  }
  __syncthreads();
}

// X[b][t][f] = sum_n hann[n] xpad[t*128 + n] e^{-2 pi i f n / 512}, xpad = reflect-pad(x, 256)
__global__ __launch_bounds__(256) void stft_kernel(const float* __restrict__ x, int L, int T, float2* __restrict__ X) {
  __shared__ float2 z[PS_NFFT];
  __shared__ float2 tw[256];
  const int t = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  twiddles(tw, tid);
  const float* xb = x + (long long)b * L;
  #pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int n = tid + 256 * r;
    int j = t * PS_HOP + n - PS_NFFT / 2;
    j = j < 0 ? -j : (j >= L ? 2 * (L - 1) - j : j);
    z[n] = make_float2(xb[j] * hann512(n), 0.f);
  }
  fft512(z, tw, tid);
  float2* Xo = X + ((long long)b * T + t) * PS_BINS;
  Xo[tid] = z[brev9(tid)];
  if (tid == 0) Xo[256] = z[1];   // brev9(256) = 1
}

// ATen CPU arange / linspace (RangeFactoriesKernel.cpp) over a contiguous float32 output:
// cpu_serial_kernel_vec runs 2 x Vectorized<float> (AVX2: 8 lanes) per step over the first
// floor(n/16)*16 elements, each vector = base + i*step from the chunk's first index, and the
// scalar formula on the tail.
SSE_DEV float arange_ts(int k, int n, double rate) {
  if (k < (n / 16) * 16) {
    const int k0 = k & ~7;
    const float base = (float)(rate * (double)k0);
    return (float)((double)base + (double)(k - k0) * rate);
  }
  return (float)(rate * (double)k);
}
SSE_DEV float linspace_pa(int f) {   // linspace(0, pi * 128, 257), float32
#pragma clang fp contract(off)
  const float end = (float)(M_PI * PS_HOP), step = end / 256.0f;
  if (f >= 256) return end;                        // scalar tail: end - step * 0
  const int f0 = f & ~7;
  const float base = f0 < 128 ? 0.0f + step * (float)f0 : end - step * (float)(PS_BINS - f0 - 1);
  return base + (float)(f - f0) * step;
}

// torchaudio.functional.phase_vocoder: one lane per (clip, bin), serial over the new frames
__global__ __launch_bounds__(64) void vocoder_kernel(const float2* __restrict__ X, int T, int nnew, double rate,
                                                     float2* __restrict__ Y) {
#pragma clang fp contract(off)
  const int f = blockIdx.x * 64 + threadIdx.x, b = blockIdx.y;
  if (f >= PS_BINS) return;
  const float2* Xb = X + (long long)b * T * PS_BINS + f;
  float2* Yb = Y + (long long)b * nnew * PS_BINS + f;
  const float pa = linspace_pa(f);
  const float2 x00 = Xb[0];
  double acc = 0.0;
  float pk = atan2f(x00.y, x00.x);   // cumsum term k: phase_0, then the phase of step k - 1
  for (int k = 0; k < nnew; ++k) {
    const float ts = arange_ts(k, nnew, rate);
    const int i0 = (int)ts;
    const float alpha = ts - floorf(ts);            // torch.remainder(ts, 1.0)
    const float2 z = make_float2(0.f, 0.f);
    const float2 c0 = i0 < T ? Xb[(long long)i0 * PS_BINS] : z;   // frames T, T+1: pad([0, 2])
    const float2 c1 = i0 + 1 < T ? Xb[(long long)(i0 + 1) * PS_BINS] : z;
    acc += (double)pk;
    const float ph = (float)acc;
    const float n0 = hypotf(c0.x, c0.y), n1 = hypotf(c1.x, c1.y);
    const float mag = alpha * n1 + (1.0f - alpha) * n0;
    float s, c;
    sincosf(ph, &s, &c);
    Yb[(long long)k * PS_BINS] = make_float2(mag * c, mag * s);
    float p = atan2f(c1.y, c1.x) - atan2f(c0.y, c0.x) - pa;
    p = p - PS_TWO_PI * rintf(p / PS_TWO_PI);
    pk = p + pa;
  }
}

// frames[b][k][n] = hann[n] * irfft(Y[b][k])[n]  (DC / Nyquist imaginary parts ignored, 1/512)
__global__ __launch_bounds__(256) void istft_frames_kernel(const float2* __restrict__ Y, int nnew,
                                                           float* __restrict__ fr) {
  __shared__ float2 z[PS_NFFT];
  __shared__ float2 tw[256];
  const int k = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  twiddles(tw, tid);
  const float2* Yk = Y + ((long long)b * nnew + k) * PS_BINS;
  // irfft(Y) = Re(ifft(Z)), Z Hermitian; Re(ifft(Z)) = Re(fft(conj Z)) / 512
  const float2 y = Yk[tid];
  z[tid] = make_float2(y.x, tid == 0 ? 0.f : -y.y);
  if (tid == 0) z[256] = make_float2(Yk[256].x, 0.f);
  else z[512 - tid] = y;                             // conj(conj(Y[f]))
  fft512(z, tw, tid);
  float* fo = fr + ((long long)b * nnew + k) * PS_NFFT;
  #pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int n = tid + 256 * r;
    fo[n] = z[brev9(n)].x * (1.0f / 512.0f) * hann512(n);
  }
}

// istft overlap-add + envelope normalisation, center trim (n_fft/2) and length = Ls
__global__ void istft_ola_kernel(const float* __restrict__ fr, int nnew, int Ls, float* __restrict__ y) {
  const int n = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  if (n >= Ls) return;
  const int pn = n + PS_NFFT / 2;
  float v = 0.f;
  if (pn < PS_NFFT + PS_HOP * (nnew - 1)) {          // beyond the last frame: zero padding
    const int thi = min(pn / PS_HOP, nnew - 1), tlo = max(0, (pn - PS_NFFT + PS_HOP) / PS_HOP);
    float s = 0.f, e = 0.f;
    for (int t = tlo; t <= thi; ++t) {
      const int o = pn - t * PS_HOP;
      const float w = hann512(o);
      s += fr[((long long)b * nnew + t) * PS_NFFT + o];
      e += w * w;
    }
    v = s / e;
  }
  y[(long long)b * Ls + n] = v;
}

__global__ void fix_length_kernel(const float* __restrict__ x, int Lx, int L, float* __restrict__ y) {
  const int n = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  if (n >= L) return;
  y[(long long)b * L + n] = n < Lx ? x[(long long)b * Lx + n] : 0.f;
}

struct PsPlan {
  double rate;
  int T, nnew, Ls, orig, Lo;
  size_t X, Y, fr, xs, xr, rs, total;
};

PsPlan ps_plan(int B, int L, int sr, int n_steps) {
  PsPlan p{};
  p.rate = std::pow(2.0, -(double)n_steps / 12.0);
  p.T = 1 + L / PS_HOP;
  p.nnew = (int)std::ceil((double)p.T / p.rate);
  p.Ls = (int)std::nearbyint((double)L / p.rate);   // python round(): half to even
  p.orig = (int)((double)sr / p.rate);
  p.Lo = p.orig == sr ? p.Ls : resample_length(p.Ls, p.orig, sr);
  auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
  p.X = 0;
  p.Y = p.X + al((size_t)B * p.T * PS_BINS * 8);
  p.fr = p.Y + al((size_t)B * p.nnew * PS_BINS * 8);
  p.xs = p.fr + al((size_t)B * p.nnew * PS_NFFT * 4);
  p.xr = p.xs + al((size_t)B * p.Ls * 4);
  p.rs = p.xr + al((size_t)B * p.Lo * 4);
  p.total = p.rs + (p.orig == sr ? 256 : al(resample_workspace_bytes(B, p.Ls, p.orig, sr)));
  return p;
}

}  // namespace

size_t pitch_shift_workspace_bytes(int B, int L, int sr, int n_steps) { return ps_plan(B, L, sr, n_steps).total; }

int launch_pitch_shift(const float* x, int B, int L, int sr, int n_steps, float* y, void* ws, size_t ws_bytes,
                       hipStream_t s) {
  // reflect padding by n_fft/2 needs L > 256 (torch.stft raises otherwise)
  if (B <= 0 || L <= PS_NFFT / 2 || sr <= 0 || n_steps < -48 || n_steps > 48) return -1;
  const PsPlan p = ps_plan(B, L, sr, n_steps);
  if (p.nnew <= 0 || p.Ls <= 0 || p.orig <= 0) return -1;
  if (ws_bytes < p.total) return -4;
  char* w = (char*)ws;
  float2* X = (float2*)(w + p.X);
  float2* Y = (float2*)(w + p.Y);
  float* fr = (float*)(w + p.fr);
  float* xs = (float*)(w + p.xs);
  float* xr = (float*)(w + p.xr);
  hipLaunchKernelGGL(stft_kernel, dim3(p.T, B), dim3(256), 0, s, x, L, p.T, X);
  if (n_steps == 0) {   // phase_vocoder returns its input at rate 1
    if (hipMemcpyAsync(Y, X, (size_t)B * p.T * PS_BINS * 8, hipMemcpyDeviceToDevice, s) != hipSuccess) return -2;
  } else {
    hipLaunchKernelGGL(vocoder_kernel, dim3((PS_BINS + 63) / 64, B), dim3(64), 0, s, X, p.T, p.nnew, p.rate, Y);
  }
  hipLaunchKernelGGL(istft_frames_kernel, dim3(p.nnew, B), dim3(256), 0, s, Y, p.nnew, fr);
  hipLaunchKernelGGL(istft_ola_kernel, dim3((p.Ls + 255) / 256, B), dim3(256), 0, s, fr, p.nnew, p.Ls, xs);
  if (hipGetLastError() != hipSuccess) return -2;
  const float* src = xs;
  if (p.orig != sr) {
    const int rc = launch_resample(xs, B, p.Ls, p.orig, sr, xr, w + p.rs, p.total - p.rs, s);
    if (rc) return rc;
    src = xr;
  }
  hipLaunchKernelGGL(fix_length_kernel, dim3((L + 255) / 256, B), dim3(256), 0, s, src, p.Lo, L, y);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
