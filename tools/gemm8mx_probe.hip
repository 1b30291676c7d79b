// Where the MX-fp8 GEMM's time goes (round-4 probe, not product code).  Times gemm8_kernel<.., MX> on the
// Whisper-large-v2 B = 128 shapes (M = 192,000 frames) in two builds, interleaved in one process:
//   DBG 0 = the library kernel (C^T in registers, bf16 out), 1 = main loop only (no epilogue),
// plus a K sweep at fixed M, N: tile time = nk * T_ktile + F, so the main loop's cost per 128-deep K-tile
// and the per-tile fixed cost F, against the 0.86 us a K-tile's 16.8 MFLOP take at the 5 PF dense peak.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/gemm8mx_probe.hip -o tools/_build/gemm8mx_probe
#include "../stuttering-speech-representation_amd/csrc/kernels_gemm8.hip"

#include <cstdio>
#include <cstdlib>

int sse_opt(int) { return 0; }
int sse_stream_cus(hipStream_t, int dev_cus) { return dev_cus; }

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);        \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

// e4m3 bytes of magnitude <= 2^-1 * 1.875 (no NaN encodings), E8M0 scales = 2^0
__global__ void fill_u8(unsigned char* p, long long n, unsigned seed, int scale_bytes) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    p[i] = scale_bytes ? (unsigned char)127 : (unsigned char)((h & 0x80) | (h & 0x37));
  }
}

typedef void (*kfn)(GemmArgs);

// mode 1: fc1 (GELU, MX-fp8 out); 2: fc2 (bf16 residual); round 5, the fp8 attention's operands: 4: MX-fp8 out with
// row-major scales (MXE 4), 5: bf16 out + per-clip column amax (MXE 5), 6: the fused Q|K (4) | V (5) form (MXE 6)
struct Shape { const char* name; int M, N, K; int mode = 0; };

int main(int argc, char** argv) {
  const bool f8 = argc > 1 && argv[1][0] == 'f';   // "f8": only the fp8-attention QKV forms
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const Shape shapes[] = {
      {"qkv", 192000, 3840, 1280}, {"ffn1", 192000, 5120, 1280}, {"ffn2", 192000, 1280, 5120},
      {"k640", 192000, 1280, 640}, {"k1280", 192000, 1280, 1280}, {"k2560", 192000, 1280, 2560},
      {"fc1_q8", 192000, 5120, 1280, 1}, {"fc2_res", 192000, 1280, 5120, 2},
      {"qkv", 192000, 3840, 1280, 0}, {"qkv_q8", 192000, 3840, 1280, 4}, {"qk_q8", 192000, 2560, 1280, 4},
      {"v_amax", 192000, 1280, 1280, 5}, {"v_bf16", 192000, 1280, 1280, 0}, {"qkv_fus", 192000, 3840, 1280, 6},
  };
  const long long maxA = 192000LL * 5120, maxB = 5120LL * 5120, maxC = 192000LL * 5120;
  unsigned char *a, *b, *sa, *sb, *cs;
  bf16* c;
  float* bias;
  void* zero;
  CK(hipMalloc(&a, maxA)); CK(hipMalloc(&b, maxB)); CK(hipMalloc(&c, maxC * 2));
  CK(hipMalloc(&sa, maxA / 32 + 4096)); CK(hipMalloc(&sb, maxB / 32 + 4096));
  CK(hipMalloc(&zero, 256)); CK(hipMemset(zero, 0, 256));
  CK(hipMalloc(&cs, maxC / 32 + 4096)); CK(hipMalloc(&bias, 5120 * 4)); CK(hipMemset(bias, 0, 5120 * 4));
  unsigned* vam;
  bf16* c2;
  CK(hipMalloc(&vam, 128 * 5120 * 4)); CK(hipMemset(vam, 0, 128 * 5120 * 4));
  CK(hipMalloc(&c2, 192000LL * 1280 * 2));
  hipLaunchKernelGGL(fill_u8, dim3(2048), dim3(256), 0, 0, a, maxA, 17u, 0);
  hipLaunchKernelGGL(fill_u8, dim3(2048), dim3(256), 0, 0, b, maxB, 91u, 0);
  hipLaunchKernelGGL(fill_u8, dim3(2048), dim3(256), 0, 0, sa, maxA / 32 + 4096, 5u, 1);
  hipLaunchKernelGGL(fill_u8, dim3(2048), dim3(256), 0, 0, sb, maxB / 32 + 4096, 7u, 1);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int ROUNDS = 3, IT = 10;
  int si = -1;
  for (const Shape& s : shapes) {
    ++si;
    if (f8 != (si >= 8)) continue;
    GemmArgs g{};
    g.A = a; g.B = b; g.M = s.M; g.N = s.N; g.K = s.K; g.rows_per_seg = s.M; g.lda = s.K;
    g.Ct = c; g.ldc = s.N; g.act = ACT_NONE; g.zero = zero; g.a_scale = sa; g.b_scale = sb; g.bias = bias;
    if (s.mode == 1) { g.act = ACT_GELU_FAST; g.c_scale = cs; g.bias = bias; }
    if (s.mode == 2) { g.resid_t = c; g.bias = bias; }
    if (s.mode == 4) { g.c_scale = cs; g.c_scale_rm = 1; }
    if (s.mode == 5) { g.vamax = vam; g.vamax_rows = 1500; }
    if (s.mode == 6) { g.c_scale = cs; g.c_scale_rm = 1; g.ldc = 2560; g.n_split = 2560; g.ct2 = c2; g.ldc2 = 1280;
                       g.vamax = vam; g.vamax_rows = 1500; }
    const int n_tiles = ((s.M + 255) / 256) * (s.N / 256);
    const double tf = 2.0 * s.M * s.N * s.K / 1e12;
    double best[4] = {1e30, 1e30, 1e30, 1e30};
    const int ND = f8 ? 2 : 4;   // 2: no MFMA, 3: no steady-loop DMA (both without the epilogue)
    for (int r = 0; r < ROUNDS; ++r)
      for (int dbg = 0; dbg < ND; ++dbg) {
        kfn k = dbg == 2 ? gemm8_kernel<4, true, false, true> : dbg == 3 ? gemm8_kernel<5, true, false, true>
              : dbg ? gemm8_kernel<1, true, false, true>
                    : (s.mode == 2 ? gemm8_kernel<0, true, false, true, 2>
                                   : (s.mode == 1 ? gemm8_kernel<0, true, false, true, 1>
                                                  : (s.mode == 4 ? gemm8_kernel<0, true, false, true, 4>
                                                                 : (s.mode == 5 ? gemm8_kernel<0, true, false, true, 5>
                                                                                : (s.mode == 6 ? gemm8_kernel<0, true, false, true, 6>
                                                                                               : gemm8_kernel<0, true, false, true, 3>)))));
        for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k, dim3(n_tiles), dim3(512), 0, 0, g);
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < IT; ++i) hipLaunchKernelGGL(k, dim3(n_tiles), dim3(512), 0, 0, g);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= IT;
        if (ms < best[dbg]) best[dbg] = ms;
      }
    const double rounds = (double)n_tiles / cus;
    printf("%-6s M=%d N=%d K=%d tiles=%d (%.2f rounds of %d CUs)\n", s.name, s.M, s.N, s.K, n_tiles, rounds, cus);
    const char* nm[4] = {"full", "no-epilogue", "no-ep,no-mfma", "no-ep,no-dma"};
    for (int d = 0; d < ND; ++d)
      printf("   %-12s %9.1f us  %7.1f TF/s  per tile-round %.2f us  per K-tile %.3f us\n", nm[d], best[d] * 1e3,
             tf / (best[d] * 1e-3), best[d] * 1e3 / rounds, best[d] * 1e3 / rounds / (s.K / 128));
    fflush(stdout);
  }
  return 0;
}
