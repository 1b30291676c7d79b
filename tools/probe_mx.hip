// Probe (diagnostic, not product): operand / scale lane maps of v_mfma_scale_f32_16x16x128_f8f6f4
// and the byte order / rounding of v_cvt_pk_fp8_f32 on gfx950.  Prints mismatch counts of the
// hypotheses the MX-fp8 GEMM relies on.
//   hipcc --offload-arch=gfx950 -O2 tools/probe_mx.hip -o /tmp/probe_mx && /tmp/probe_mx
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdint.h>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// A [16][128] fp8, B [16][128] fp8 (B as [n][k]); lane l holds row/col l&15, k = 32*(l>>4) + j
template <int OA, int OB>
__global__ void mx_probe(const uint8_t* A, const uint8_t* B, const uint32_t* sa, const uint32_t* sb, float* C) {
  const int l = threadIdx.x;
  i32x8 a, b;
  const uint32_t* pa = (const uint32_t*)(A + (l & 15) * 128 + 32 * (l >> 4));
  const uint32_t* pb = (const uint32_t*)(B + (l & 15) * 128 + 32 * (l >> 4));
  for (int j = 0; j < 8; ++j) { a[j] = pa[j]; b[j] = pb[j]; }
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, OA, (int)sa[l], OB, (int)sb[l]);
  for (int r = 0; r < 4; ++r) C[((l >> 4) * 4 + r) * 16 + (l & 15)] = c[r];   // row (l>>4)*4+r, col l&15
}

__global__ void cvt_probe(const float* x, uint32_t* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 < n) out[i] = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(x[2 * i], x[2 * i + 1], 0, false);
}

static float e4m3_to_f(uint8_t v) {
  const int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  float f = e ? ldexpf(1.f + m / 8.f, e - 7) : ldexpf(m / 8.f, -6);
  if (e == 15 && m == 7) f = NAN;
  return s ? -f : f;
}

int main() {
  uint8_t hA[16 * 128], hB[16 * 128];
  // small integers -3..3 encoded in e4m3: value v -> exponent/mantissa
  auto enc = [](int v) -> uint8_t {
    if (v == 0) return 0;
    const int s = v < 0, a = abs(v);
    int e = 0;
    while ((1 << (e + 1)) <= a) ++e;
    const int m = (a - (1 << e)) * 8 / (1 << e);
    return (uint8_t)((s << 7) | ((e + 7) << 3) | m);
  };
  float fA[16][128], fB[16][128];
  for (int r = 0; r < 16; ++r)
    for (int k = 0; k < 128; ++k) {
      const int va = ((r * 7 + k * 3) % 7) - 3, vb = ((r * 5 + k * 11 + 1) % 7) - 3;
      hA[r * 128 + k] = enc(va); hB[r * 128 + k] = enc(vb);
      fA[r][k] = e4m3_to_f(hA[r * 128 + k]); fB[r][k] = e4m3_to_f(hB[r * 128 + k]);
    }
  uint8_t *dA, *dB; uint32_t *dsa, *dsb; float* dC;
  hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dsa, 256); hipMalloc(&dsb, 256); hipMalloc(&dC, 1024);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  for (int sel = 0; sel < 4; ++sel) {
    uint32_t sa[64], sb[64];
    int ea[64], eb[64];
    for (int l = 0; l < 64; ++l) {
      ea[l] = 127 + (l % 3) - 1;        // 0.5, 1, 2
      eb[l] = 127 + ((l / 3) % 3) - 1;
      sa[l] = 0x7F7F7F7Fu; sb[l] = 0x7F7F7F7Fu;
      sa[l] = (sa[l] & ~(0xFFu << (8 * sel))) | ((uint32_t)ea[l] << (8 * sel));
      sb[l] = (sb[l] & ~(0xFFu << (8 * sel))) | ((uint32_t)eb[l] << (8 * sel));
    }
    hipMemcpy(dsa, sa, 256, hipMemcpyHostToDevice);
    hipMemcpy(dsb, sb, 256, hipMemcpyHostToDevice);
    switch (sel) {
      case 0: hipLaunchKernelGGL((mx_probe<0, 0>), 1, 64, 0, 0, dA, dB, dsa, dsb, dC); break;
      case 1: hipLaunchKernelGGL((mx_probe<1, 1>), 1, 64, 0, 0, dA, dB, dsa, dsb, dC); break;
      case 2: hipLaunchKernelGGL((mx_probe<2, 2>), 1, 64, 0, 0, dA, dB, dsa, dsb, dC); break;
      case 3: hipLaunchKernelGGL((mx_probe<3, 3>), 1, 64, 0, 0, dA, dB, dsa, dsb, dC); break;
    }
    float C[256];
    hipMemcpy(C, dC, 1024, hipMemcpyDeviceToHost);
    // hypotheses: lane group g = l>>4, byte j of the lane is hardware k = kmap(g, j); the scale of
    // hardware block b (k in [32b, 32b+32)) of row m comes from lane m + 16*b
    auto kmap = [](int h, int g, int j) {
      if (h == 0) return 32 * g + j;                                  // contiguous 32
      if (h == 1) return j < 16 ? 16 * g + j : 64 + 16 * g + (j - 16); // 16 + 16
      if (h == 2) return 8 * g + (j & 7) + 32 * (j >> 3);             // 8-wide interleave
      return 4 * g + (j & 3) + 16 * (j >> 2);                          // 4-wide interleave
    };
    for (int h = 0; h < 4; ++h) {
      int bad = 0;
      for (int m = 0; m < 16; ++m)
        for (int n = 0; n < 16; ++n) {
          double ref = 0;
          for (int g = 0; g < 4; ++g)
            for (int j = 0; j < 32; ++j) {
              const int blk = kmap(h, g, j) / 32;
              const double s1 = ldexp(1.0, ea[m + 16 * blk] - 127) * ldexp(1.0, eb[n + 16 * blk] - 127);
              ref += s1 * fA[m][32 * g + j] * fB[n][32 * g + j];
            }
          if (fabs(ref - C[m * 16 + n]) > 1e-3) ++bad;
        }
      printf("opsel %d layout hypothesis %d: mismatches %d / 256\n", sel, h, bad);
    }
  }
  // cvt probe
  const int n = 4096;
  float hx[n];
  for (int i = 0; i < n; ++i) {
    const float u = (float)((i * 2654435761u) % 100000u) / 100000.f;
    hx[i] = (i & 1 ? -1.f : 1.f) * ldexpf(1.f + u, (i % 24) - 12);
  }
  hx[0] = 448.f; hx[1] = 464.f; hx[2] = 0.f; hx[3] = -0.f; hx[4] = 1e-6f; hx[5] = 0.0019531f;
  float* dx; uint32_t* dout;
  hipMalloc(&dx, sizeof hx); hipMalloc(&dout, n * 2);
  hipMemcpy(dx, hx, sizeof hx, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(cvt_probe, n / 512, 256, 0, 0, dx, dout, n);
  uint32_t ho[n / 2];
  hipMemcpy(ho, dout, n * 2, hipMemcpyDeviceToHost);
  // reference RNE e4m3fn (saturating not assumed): nearest representable by exhaustive search
  int badc = 0;
  for (int i = 0; i < n; ++i) {
    const uint8_t got = (ho[i / 2] >> (8 * (i & 1))) & 0xFF;
    float best = 0; int bi = 0; double bd = 1e30;
    for (int v = 0; v < 256; ++v) {
      const float f = e4m3_to_f((uint8_t)v);
      if (isnan(f)) continue;
      const double d = fabs((double)f - hx[i]);
      const bool even = (v & 1) == 0;
      if (d < bd || (d == bd && even)) { bd = d; bi = v; best = f; }
    }
    (void)best;
    if (got != bi && !(fabs(hx[i]) > 448.f)) {
      if (badc < 8) printf("cvt mismatch x=%.9g got %02x ref %02x\n", hx[i], got, bi);
      ++badc;
    }
    if (i < 6) printf("cvt x=%.9g -> %02x (%g)\n", hx[i], got, e4m3_to_f(got));
  }
  printf("cvt mismatches (|x| <= 448): %d / %d\n", badc, n);
  return 0;
}
