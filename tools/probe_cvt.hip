// Probe (diagnostic): semantics of the gfx950 scaled down-conversion v_cvt_scalef32_pk_fp8_bf16 (two bf16 ->
// two e4m3 with an f32 scale): prints the e4m3 results of (1.5, -3.0) and (200, 0.01) for several scales.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
typedef short v2i16 __attribute__((ext_vector_type(2)));
typedef __bf16 v2bf16 __attribute__((ext_vector_type(2)));
__global__ void k(unsigned* o, const float* sc, int n) {
  const int t = threadIdx.x;
  if (t >= n) return;
  v2bf16 x = {(__bf16)1.5f, (__bf16)(-3.0f)}, y = {(__bf16)200.f, (__bf16)0.01f};
  v2i16 r = {0, 0};
  r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, x, sc[t], false);
  r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, y, sc[t], true);
  o[2 * t] = (unsigned)(unsigned short)r[0];
  o[2 * t + 1] = (unsigned)(unsigned short)r[1];
}
// bit-identity of the scaled f32 conversion with the multiply-then-convert form the epilogues used:
// cvt_scalef32_pk_fp8_f32(a, b, 2^E) vs cvt_pk_fp8_f32(a * 2^-E, b * 2^-E) over hashed values of every magnitude
__global__ void cmp(unsigned* bad, int E) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned h = i * 2654435761u ^ (unsigned)E * 40503u;
  h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
  // |x| in [2^(E-12), 2^(E+9)): e4m3 subnormals, normals, ties and the saturation edge of x / 2^E
  const float m = __builtin_bit_cast(float, 0x3F800000u | (h & 0x7FFFFF));
  const float a = ldexpf(m, E - 12 + (int)((h >> 23) % 21)) * ((h >> 31) ? -1.f : 1.f);
  const float b = -a * 0.7f;
  if (fabsf(a) * ldexpf(1.f, -E) > 448.f || fabsf(b) * ldexpf(1.f, -E) > 448.f) return;
  const float sc = ldexpf(1.f, E), inv = ldexpf(1.f, -E);
  v2i16 r = {0, 0};
  r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(r, a, b, sc, false);
  const int ref = __builtin_amdgcn_cvt_pk_fp8_f32(a * inv, b * inv, 0, false);
  if ((__builtin_bit_cast(int, r) & 0xFFFF) != (ref & 0xFFFF)) atomicAdd(bad, 1u);
}
static double dec(unsigned c) {
  const int s = c & 0x80, e = (c >> 3) & 15, m = c & 7;
  double v = e == 0 ? ldexp(m / 8.0, -6) : ldexp(1.0 + m / 8.0, e - 7);
  if (e == 15 && m == 7) v = NAN;
  return s ? -v : v;
}
int main() {
  const float hs[] = {1.f, 2.f, 0.5f, 0.0078125f, 128.f, 3.f};
  const int n = 6;
  float* ds; unsigned* d;
  hipMalloc(&ds, sizeof hs); hipMalloc(&d, 2 * n * 4);
  hipMemcpy(ds, hs, sizeof hs, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, 1, 64, 0, 0, d, ds, n);
  unsigned h[2 * n];
  hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  for (int t = 0; t < n; ++t)
    printf("scale %-10g (1.5, -3, 200, 0.01) -> %g %g %g %g\n", hs[t], dec(h[2 * t] & 255), dec(h[2 * t] >> 8),
           dec(h[2 * t + 1] & 255), dec(h[2 * t + 1] >> 8));
  unsigned* bad;
  hipMalloc(&bad, 4);
  for (int E : {-20, -8, -1, 0, 3, 10}) {
    hipMemset(bad, 0, 4);
    hipLaunchKernelGGL(cmp, 4096, 256, 0, 0, bad, E);
    unsigned hb = 0;
    hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    printf("E = %3d: cvt_scalef32_pk_fp8_f32 vs cvt_pk_fp8_f32(x * 2^-E): %u mismatches of 1048576\n", E, hb);
  }
  return 0;
}
