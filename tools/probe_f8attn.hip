// Probe (diagnostic) for the fp8 Whisper attention: operand / scale / output layouts of
// v_mfma_scale_f32_32x32x64_f8f6f4, the lane map of ds_read_b64_tr_b8, and the issue cost of the
// 32x32x64 fp8 MFMA next to the 32x32x16 bf16 one.
//   E1: A one-hot 1.0 at (lane la, byte ja), B all 1.0, A scale of lane l = 2^(l-32): the nonzero C row
//       names the row of (la, ja), its value the lane whose scale byte applied.
//   E2: the same for B (one-hot at (lb, jb)): the nonzero C column and the B scale lane.
//   E3: A one-hot at (la, ja), B(lane, byte) = 1.0 only where (lane >> 5, byte) == (la >> 5, ja) or all
//       slots distinct powers: prints which B (lane >> 5, byte) slot the A slot multiplies.
//   TR: LDS bytes = their address (low byte) / (high byte) and each lane's ds_read_b64_tr_b8 result at
//       address lane * 8 and lane * stride.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8b __attribute__((ext_vector_type(8)));

// C layout assumed for a 32x32 f32x16: lane l, element e -> row 8 (e / 4) + 4 (l / 32) + e % 4, col l % 32;
// E1/E2 print the raw (lane, element) position too so the assumption is checked.
__global__ void e1(float* out, int which) {
  const int e = blockIdx.x, la = e >> 5, ja = e & 31, l = threadIdx.x;
  i32x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, b;
  for (int w = 0; w < 8; ++w) b[w] = 0x38383838;   // e4m3 1.0
  if (l == la) a[ja >> 2] = 0x38 << (8 * (ja & 3));
  f32x16 c = {};
  const int sv = (95 + l) | (0x7F << 8) | (0x7F << 16) | (0x7F << 24), one = 0x7F7F7F7F;
  if (which == 0)
    c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, sv, 0, one);
  else
    c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(b, a, c, 0, 0, 0, one, 0, sv);
  for (int r = 0; r < 16; ++r) out[e * 1024 + l * 16 + r] = c[r];
}

// E3: A one-hot at (la, ja); B(lane, byte) = 2^-(slot & 7) e4m3 with slot = (lane >> 5) * 32 + byte and
// B scale of lane l = 2^(slot >> 3) in the low byte... kept simple: B(lane, byte) one-hot 1.0 at
// (hb * 32 + n, jb) for every n (a full B row of K-slot (hb, jb)); run over (hb, jb) for each A slot.
__global__ void e3(float* out, int la, int ja) {
  const int e = blockIdx.x, hb = e >> 5, jb = e & 31, l = threadIdx.x;
  i32x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, b = {0, 0, 0, 0, 0, 0, 0, 0};
  if (l == la) a[ja >> 2] = 0x38 << (8 * (ja & 3));
  if ((l >> 5) == hb) b[jb >> 2] = 0x38 << (8 * (jb & 3));
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
  float s = 0.f;
  for (int r = 0; r < 16; ++r) s += c[r];
  for (int o = 32; o; o >>= 1) s += __shfl_xor(s, o, 64);
  if (l == 0) out[e] = s;
}

__global__ void tr(int* out, int mode) {
  __shared__ __attribute__((aligned(16))) unsigned char s[8192];
  for (int i = threadIdx.x; i < 8192; i += 64) s[i] = mode & 1 ? (unsigned char)(i >> 8) : (unsigned char)i;
  __syncthreads();
  const int l = threadIdx.x;
  int addr = mode < 2 ? l * 8 : (mode < 4 ? l * 64 : (l & 7) * 64 + (l >> 3) * 8);
  i32x2 v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) i32x2*)(s + addr));
  out[l * 2] = v.x;
  out[l * 2 + 1] = v.y;
}

template <int KIND>
__global__ void rate(long long* out, float* sink) {
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  i32x8 a;
  bf16x8 x;
  for (int w = 0; w < 8; ++w) a[w] = 0x38383838 + threadIdx.x;
  for (int w = 0; w < 8; ++w) x[w] = (short)(0x3f80 + threadIdx.x);
  const bf16x8b xb = __builtin_bit_cast(bf16x8b, x);
  __syncthreads();
  const long long t0 = clock64();
  for (int it = 0; it < 256; ++it) {
    if constexpr (KIND == 0) {
      c0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, a, c0, 0, 0, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
      c1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, a, c1, 0, 0, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
      c2 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, a, c2, 0, 0, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
      c3 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, a, c3, 0, 0, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
    } else if constexpr (KIND == 2) {   // 16x16x128 scaled: the MX GEMM's instruction (4 accumulators of 4)
      f32x4 d0 = {c0[0], c0[1], c0[2], c0[3]}, d1 = {c1[0], c1[1], c1[2], c1[3]}, d2 = {c2[0], c2[1], c2[2], c2[3]},
            d3 = {c3[0], c3[1], c3[2], c3[3]};
      d0 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, a, d0, 0, 0, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
      d1 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, a, d1, 0, 0, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
      d2 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, a, d2, 0, 0, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
      d3 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, a, d3, 0, 0, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
      c0[0] = d0[0]; c0[1] = d0[1]; c0[2] = d0[2]; c0[3] = d0[3];
      c1[0] = d1[0]; c1[1] = d1[1]; c1[2] = d1[2]; c1[3] = d1[3];
      c2[0] = d2[0]; c2[1] = d2[1]; c2[2] = d2[2]; c2[3] = d2[3];
      c3[0] = d3[0]; c3[1] = d3[1]; c3[2] = d3[2]; c3[3] = d3[3];
    } else if constexpr (KIND == 3) {   // 16x16x32 bf16: the bf16 GEMM's instruction
      f32x4 d0 = {c0[0], c0[1], c0[2], c0[3]}, d1 = {c1[0], c1[1], c1[2], c1[3]}, d2 = {c2[0], c2[1], c2[2], c2[3]},
            d3 = {c3[0], c3[1], c3[2], c3[3]};
      d0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xb, xb, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xb, xb, d1, 0, 0, 0);
      d2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xb, xb, d2, 0, 0, 0);
      d3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xb, xb, d3, 0, 0, 0);
      c0[0] = d0[0]; c0[1] = d0[1]; c0[2] = d0[2]; c0[3] = d0[3];
      c1[0] = d1[0]; c1[1] = d1[1]; c1[2] = d1[2]; c1[3] = d1[3];
      c2[0] = d2[0]; c2[1] = d2[1]; c2[2] = d2[2]; c2[3] = d2[3];
      c3[0] = d3[0]; c3[1] = d3[1]; c3[2] = d3[2]; c3[3] = d3[3];
    } else {
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xb, xb, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xb, xb, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xb, xb, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xb, xb, c3, 0, 0, 0);
    }
  }
  const long long t1 = clock64();
  float s = 0.f;
  for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  sink[threadIdx.x] = s;
  if (threadIdx.x == 0) out[0] = t1 - t0;
}

static int slot_of(float v) { return v > 0.f ? (int)lrintf(log2f(v)) + 32 : -1; }

int main() {
  float* d;
  hipMalloc(&d, 2048 * 1024 * 4);
  static float h[2048 * 1024];
  for (int which = 0; which < 2; ++which) {
    hipLaunchKernelGGL(e1, 2048, 64, 0, 0, d, which);
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    printf("== E%d: %s operand (lane, byte) -> [C lane/elem pattern] %s / scale lane\n", which + 1,
           which ? "B" : "A", which ? "col" : "row");
    for (int ld = 0; ld < 64; ++ld) {
      printf("lane %2d:", ld);
      for (int j = 0; j < 32; ++j) {
        const float* C = h + (ld * 32 + j) * 1024;
        int nz = 0, idx = -1, first = -1;
        float v = 0.f;
        int rows = 0, cols = 0;   // under the assumed C layout
        int rset = -1, cset = -1;
        bool rconst = true, cconst = true;
        for (int i = 0; i < 1024; ++i)
          if (C[i] != 0.f) {
            ++nz;
            idx = i;
            v = C[i];
            const int l = i / 16, e = i % 16;
            const int row = 8 * (e / 4) + 4 * (l / 32) + e % 4, col = l % 32;
            if (first < 0) { first = i; rset = row; cset = col; }
            if (row != rset) rconst = false;
            if (col != cset) cconst = false;
          }
        (void)rows; (void)cols; (void)idx;
        if (which == 0) printf(" %d/%d%s", rconst ? rset : -9, slot_of(v), nz == 32 ? "" : "!");
        else printf(" %d/%d%s", cconst ? cset : -9, slot_of(v), nz == 32 ? "" : "!");
      }
      printf("\n");
    }
  }
  printf("== E3: A slot (lane, byte) -> B slots (lane>>5, byte) it multiplies\n");
  for (int la : {0, 1, 31, 32, 33, 63})
    for (int ja = 0; ja < 32; ja += 1) {
      hipLaunchKernelGGL(e3, 64, 64, 0, 0, d, la, ja);
      static float r[64];
      hipMemcpy(r, d, sizeof r, hipMemcpyDeviceToHost);
      printf("A(%2d,%2d):", la, ja);
      for (int e = 0; e < 64; ++e)
        if (r[e] != 0.f) printf(" B(%d,%d)=%g", e >> 5, e & 31, r[e]);
      printf("\n");
    }
  int* di;
  hipMalloc(&di, 128 * 4);
  static int hi[128];
  for (int mode = 0; mode < 6; ++mode) {
    hipLaunchKernelGGL(tr, 1, 64, 0, 0, di, mode);
    hipMemcpy(hi, di, sizeof hi, hipMemcpyDeviceToHost);
    printf("== TR mode %d (%s byte, addr %s)\n", mode, mode & 1 ? "high" : "low",
           mode < 2 ? "lane*8" : (mode < 4 ? "lane*64" : "(l&7)*64+(l>>3)*8"));
    for (int l = 0; l < 64; ++l) {
      printf("l%2d:", l);
      for (int k = 0; k < 8; ++k) printf(" %3d", (hi[l * 2 + k / 4] >> (8 * (k & 3))) & 0xFF);
      printf(l % 2 ? "\n" : "   ");
    }
  }
  long long* dt;
  float* sink;
  hipMalloc(&dt, 8);
  hipMalloc(&sink, 1024 * 4);
  long long t;
  hipLaunchKernelGGL(rate<0>, 1, 64, 0, 0, dt, sink);
  hipLaunchKernelGGL(rate<0>, 1, 64, 0, 0, dt, sink);
  hipMemcpy(&t, dt, 8, hipMemcpyDeviceToHost);
  printf("== rate: 32x32x64 f8f6f4 (scaled) %.1f cycles per MFMA (clock64)\n", t / 1024.0);
  hipLaunchKernelGGL(rate<1>, 1, 64, 0, 0, dt, sink);
  hipLaunchKernelGGL(rate<1>, 1, 64, 0, 0, dt, sink);
  hipMemcpy(&t, dt, 8, hipMemcpyDeviceToHost);
  printf("== rate: 32x32x16 bf16 %.1f cycles per MFMA (clock64)\n", t / 1024.0);
  hipLaunchKernelGGL(rate<2>, 1, 64, 0, 0, dt, sink);
  hipLaunchKernelGGL(rate<2>, 1, 64, 0, 0, dt, sink);
  hipMemcpy(&t, dt, 8, hipMemcpyDeviceToHost);
  printf("== rate: 16x16x128 f8f6f4 (scaled) %.1f cycles per MFMA (clock64)\n", t / 1024.0);
  hipLaunchKernelGGL(rate<3>, 1, 64, 0, 0, dt, sink);
  hipLaunchKernelGGL(rate<3>, 1, 64, 0, 0, dt, sink);
  hipMemcpy(&t, dt, 8, hipMemcpyDeviceToHost);
  printf("== rate: 16x16x32 bf16 %.1f cycles per MFMA (clock64)\n", t / 1024.0);
  return 0;
}
