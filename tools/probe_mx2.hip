// Probe (diagnostic): which lane's scale byte applies to A element (lane ld, byte j) of
// v_mfma_scale_f32_16x16x128_f8f6f4.  Experiment e = ld*32 + j: A one-hot 1.0 at (ld, j), B all
// 1.0 with unit scales, A scale of lane l = 2^(l-32) in byte `sel`; C[ld&15][*] = 2^(l*-32) names l*.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdint.h>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void probe(float* out) {
  const int e = blockIdx.x, ld = e >> 5, j = e & 31, l = threadIdx.x;
  i32x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, b;
  for (int w = 0; w < 8; ++w) b[w] = 0x38383838;   // e4m3 1.0 = 0x38
  if (l == ld) a[j >> 2] = 0x38 << (8 * (j & 3));
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  const int sa = (95 + l) | (0x7F << 8), sb = 0x7F7F7F7F;
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa, 0, sb);
  for (int r = 0; r < 4; ++r) out[e * 256 + ((l >> 4) * 4 + r) * 16 + (l & 15)] = c[r];
}
int main() {
  float* d; hipMalloc(&d, 2048 * 256 * 4);
  hipLaunchKernelGGL(probe, 2048, 64, 0, 0, d);
  static float h[2048 * 256];
  hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  for (int ld = 0; ld < 64; ++ld) {
    printf("lane %2d:", ld);
    for (int j = 0; j < 32; ++j) {
      const float* C = h + (ld * 32 + j) * 256;
      int nz = 0, row = -1; float v = 0;
      for (int i = 0; i < 256; ++i) if (C[i] != 0.f) { ++nz; row = i / 16; v = C[i]; }
      const int sl = nz ? (int)lrintf(log2f(v)) + 32 : -1;
      printf(" %d/%d%s", row, sl, nz == 16 ? "" : "!");
    }
    printf("\n");
  }
  return 0;
}
