// Ingest transforms for non-16 kHz / multi-channel WAVs:
//   mono mix   torch.mean(waveform, dim=0)                      REF/WavLM_embeddings.py:103-105
//   resample   torchaudio.transforms.Resample(sr, 16000)        REF/WavLM_embeddings.py:107-110
// torchaudio's default "sinc_interp_hann" resampler is a polyphase FIR: output sample i*new + p
// is the dot product of filter row p (2*width + orig taps) with the zero-padded input starting
// at i*orig.  Here the filter bank is generated on device in fp64 (cast to fp32 like
// torchaudio), the input blocks are laid out as GEMM rows, and the dot products run on the
// exact-f32 MFMA GEMM (kernels_gemm.hip); a compaction pass interleaves the phases.
#include <cmath>

#include "common.h"
#include "kernels.h"

namespace {

__global__ void rs_table_kernel(int orig, int nw, int width, int Kp, int Np, float* __restrict__ tab) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= Np * Kp) return;
  const int p = i / Kp, k = i - p * Kp;
  const int K = 2 * width + orig;
  float v = 0.f;
  if (p < nw && k < K) {
    const double lw = 6.0, base = (orig < nw ? orig : nw) * 0.99;
    // t = (-p / new  [float32, as torch's int64 / int promotes to the default dtype]) + idx
    const double tp = (double)(-(float)p / (float)nw);
    double t = (tp + (double)(k - width) / orig) * base;
    t = t < -lw ? -lw : (t > lw ? lw : t);
    const double cw = cos(t * M_PI / lw / 2.0);
    const double win = cw * cw;
    const double tt = t * M_PI;
    const double sinc = tt == 0.0 ? 1.0 : sin(tt) / tt;
    v = (float)(sinc * (win * (base / orig)));   // torchaudio: kernels *= window * scale
  }
  tab[i] = v;
}

// frames[b*nblk + i][k] = xpad[b][i*orig + k], xpad = [width zeros | x | zeros]  (1-D grid)
__global__ void rs_frames_kernel(const float* __restrict__ x, int L, int orig, int width, int K, int Kp, int nblk,
                                 long long total, float* __restrict__ fr) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  const long long r = e / Kp;
  const int k = (int)(e - r * Kp);
  const int b = (int)(r / nblk), i = (int)(r - (long long)b * nblk);
  const long long j = (long long)i * orig + k - width;
  fr[e] = (k < K && j >= 0 && j < L) ? x[(long long)b * L + j] : 0.f;
}

__global__ void rs_compact_kernel(const float* __restrict__ g, int nblk, int nw, int Np, int Lo,
                                  float* __restrict__ y) {
  const int b = blockIdx.y;
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= Lo) return;
  const int i = n / nw, p = n - i * nw;
  y[(long long)b * Lo + n] = g[((long long)b * nblk + i) * Np + p];
}

__global__ void mono_kernel(const float* __restrict__ x, int C, int L, float* __restrict__ y) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= L) return;
  const float* xb = x + (long long)b * C * L;
  float s = xb[i];
  for (int c = 1; c < C; ++c) s += xb[(long long)c * L + i];     // torch.mean: sum, then divide
  y[(long long)b * L + i] = s / (float)C;
}

struct RsPlan {
  int orig, nw, width, K, Kp, Np, nblk, Lo;
  size_t tab, fr, g, total;
};

RsPlan rs_plan(int B, int L, int orig_freq, int new_freq) {
  RsPlan p{};
  int a = orig_freq, c = new_freq;
  while (c) { const int t = a % c; a = c; c = t; }
  p.orig = orig_freq / a;
  p.nw = new_freq / a;
  const double base = (p.orig < p.nw ? p.orig : p.nw) * 0.99;
  p.width = (int)std::ceil(6.0 * p.orig / base);
  p.K = 2 * p.width + p.orig;
  p.Kp = (p.K + 3) / 4 * 4;
  p.Np = (p.nw + 63) / 64 * 64;
  p.nblk = L / p.orig + 1;
  p.Lo = (int)(((long long)p.nw * L + p.orig - 1) / p.orig);
  auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
  p.tab = 0;
  p.fr = al((size_t)p.Np * p.Kp * 4);
  p.g = p.fr + al((size_t)B * p.nblk * p.Kp * 4);
  p.total = p.g + al((size_t)B * p.nblk * p.Np * 4) + 256;   // + a zero page for the GEMM
  return p;
}

}  // namespace

int resample_length(int L, int orig_freq, int new_freq) { return rs_plan(1, L, orig_freq, new_freq).Lo; }

size_t resample_workspace_bytes(int B, int L, int orig_freq, int new_freq) {
  return rs_plan(B, L, orig_freq, new_freq).total;
}

int launch_resample(const float* x, int B, int L, int orig_freq, int new_freq, float* y, void* ws, size_t ws_bytes,
                    hipStream_t s) {
  if (B <= 0 || L <= 0 || orig_freq <= 0 || new_freq <= 0) return -1;
  if (orig_freq == new_freq)
    return hipMemcpyAsync(y, x, (size_t)B * L * 4, hipMemcpyDeviceToDevice, s) == hipSuccess ? 0 : -2;
  const RsPlan p = rs_plan(B, L, orig_freq, new_freq);
  if (ws_bytes < p.total) return -4;
  char* w = (char*)ws;
  float* tab = (float*)(w + p.tab);
  float* fr = (float*)(w + p.fr);
  float* g = (float*)(w + p.g);
  void* zero = w + p.total - 256;
  if (hipMemsetAsync(zero, 0, 256, s) != hipSuccess) return -2;
  hipLaunchKernelGGL(rs_table_kernel, dim3((p.Np * p.Kp + 255) / 256), dim3(256), 0, s, p.orig, p.nw, p.width, p.Kp,
                     p.Np, tab);
  const long long nfr = (long long)B * p.nblk * p.Kp;
  hipLaunchKernelGGL(rs_frames_kernel, dim3((unsigned)((nfr + 255) / 256)), dim3(256), 0, s, x, L, p.orig, p.width,
                     p.K, p.Kp, p.nblk, nfr, fr);
  GemmArgs ga{};
  ga.A = fr; ga.B = tab; ga.M = B * p.nblk; ga.N = p.Np; ga.K = p.Kp; ga.rows_per_seg = ga.M; ga.lda = p.Kp;
  ga.Cf = g; ga.ldc = p.Np; ga.zero = zero;
  const int rc = launch_gemm_f32(ga, AMODE_SEG, 1, s);
  if (rc) return rc;
  hipLaunchKernelGGL(rs_compact_kernel, dim3((p.Lo + 255) / 256, B), dim3(256), 0, s, g, p.nblk, p.nw, p.Np, p.Lo, y);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int launch_mono(const float* x, int B, int C, int L, float* y, hipStream_t s) {
  if (B <= 0 || C <= 0 || L <= 0) return -1;
  hipLaunchKernelGGL(mono_kernel, dim3((L + 255) / 256, B), dim3(256), 0, s, x, C, L, y);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ---------------------------------------------------------------------------------------
// Pointwise augmentation of augment_audio (REF/model_training_1.py:167-214): per clip
//   kind 0 none, 1 noise: x + (float)N(0,1) * factor, 2 volume: x * factor, 3 clamp only;
// then torch.clamp(-1, 1).  N(0,1) is the build's counter-hash Gaussian (synth.gaussian: splitmix64
// uniforms, Box-Muller in fp64) on stream 2*s / 2*s+1, so the oracle can restate it exactly.
namespace {
SSE_DEV uint64_t smix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
SSE_DEV uint64_t sbase(uint64_t seed, uint64_t stream) {
  return smix(seed * 0x100000001B3ull + stream * 0x9E3779B1ull + 0x632BE59BD9B4E019ull);
}
SSE_DEV double u01(uint64_t base, uint64_t i) { return (double)(smix(i + base) >> 11) * (1.0 / 9007199254740992.0); }

__global__ void augment_kernel(const float* __restrict__ x, float* __restrict__ y, int L, const int* __restrict__ kind,
                               const float* __restrict__ factor, const long long* __restrict__ stream, uint64_t seed) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= L) return;
  const int k = kind[b];
  float v = x[(long long)b * L + i];
  if (k == 1) {
    const uint64_t s = (uint64_t)stream[b];
    const double g = sqrt(-2.0 * log1p(-u01(sbase(seed, 2 * s), i))) * cos(2.0 * M_PI * u01(sbase(seed, 2 * s + 1), i));
    v = v + (float)g * factor[b];
  } else if (k == 2) {
    v = v * factor[b];
  }
  y[(long long)b * L + i] = fminf(fmaxf(v, -1.0f), 1.0f);
}
}  // namespace

int launch_augment(const float* x, float* y, int B, int L, const int* kind, const float* factor,
                   const long long* stream, uint64_t seed, hipStream_t s) {
  if (B <= 0 || L <= 0) return -1;
  hipLaunchKernelGGL(augment_kernel, dim3((L + 255) / 256, B), dim3(256), 0, s, x, y, L, kind, factor, stream, seed);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
