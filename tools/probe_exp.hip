// VALU issue rates on gfx950 (probe, not product code): v_exp_f32 alone, v_add_f32 alone, both interleaved,
// v_pk_add_f32, and a degree-2 polynomial exp2 built from packed adds / FMAs, over 8 independent chains per lane.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe_exp.hip -o tools/_build/probe_exp
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int IT = 4096;

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, float seed) {
  float x[8], y[8];
  #pragma unroll
  for (int i = 0; i < 8; ++i) { x[i] = seed * (threadIdx.x + i) * 1e-6f - 1.0f; y[i] = x[i]; }
  for (int it = 0; it < IT; ++it) {
    if constexpr (MODE == 0) {   // 8 exps
      #pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_exp_f32 %0, %0" : "+v"(x[i]));
    } else if constexpr (MODE == 1) {   // 8 adds
      #pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[i]) : "v"(y[i]));
    } else if constexpr (MODE == 2) {   // 8 exps + 8 adds interleaved (independent)
      #pragma unroll
      for (int i = 0; i < 8; ++i) {
        asm volatile("v_exp_f32 %0, %0" : "+v"(x[i]));
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(y[i]) : "v"(x[(i + 4) & 7]));
      }
    } else if constexpr (MODE == 3) {   // 8 packed adds (16 results)
      #pragma unroll
      for (int i = 0; i < 8; i += 2) {
        asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(*(f2*)&x[i]) : "v"(*(f2*)&y[i]));
        asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(*(f2*)&y[i]) : "v"(*(f2*)&x[i]));
      }
    } else if constexpr (MODE == 4) {   // 8 exps + 16 adds
      #pragma unroll
      for (int i = 0; i < 8; ++i) {
        asm volatile("v_exp_f32 %0, %0" : "+v"(x[i]));
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(y[i]) : "v"(x[(i + 4) & 7]));
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(y[i]) : "v"(x[(i + 5) & 7]));
      }
    } else if constexpr (MODE == 5) {   // 8 fmas
      #pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x[i]) : "v"(y[i]));
    } else if constexpr (MODE == 6) {   // 8 cvt_pk_fp8 + 8 exps
      #pragma unroll
      for (int i = 0; i < 8; ++i) {
        asm volatile("v_exp_f32 %0, %0" : "+v"(x[i]));
        asm volatile("v_cvt_pk_fp8_f32 %0, %1, %1" : "+v"(y[i]) : "v"(x[(i + 4) & 7]));
      }
    }
  }
  float s = 0;
  #pragma unroll
  for (int i = 0; i < 8; ++i) s += x[i] + y[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  int cus = 0, clk = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  float* out;
  hipMalloc(&out, (size_t)cus * 8 * 256 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const char* nm[] = {"8 exp", "8 add", "8 exp + 8 add", "8 pk_add", "8 exp + 16 add", "8 fma", "8 exp + 8 cvt_pk_fp8"};
  void (*fn[])(float*, float) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>};
  for (int waves = 1; waves <= 2; ++waves) {
    const int blocks = cus * waves * 4 / 4;   // 256-thread blocks: 4 waves each -> 1 wave per SIMD per block
    for (int m = 0; m < 7; ++m) {
      float best = 1e30f;
      for (int r = 0; r < 4; ++r) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(fn[m], dim3(blocks), dim3(256), 0, 0, out, 1.0f + r);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (r && ms < best) best = ms;
      }
      // cycles per loop iteration per SIMD at the reported clock (waves per SIMD interleaved)
      const double cyc = best * 1e-3 * clk * 1e3 / IT;
      printf("waves/SIMD %d  %-22s %8.3f ms  %7.1f cycles per iteration per SIMD (%.2f per wave-instr of the first kind)\n",
             waves, nm[m], best, cyc, cyc / (8.0 * waves));
    }
  }
  return 0;
}
