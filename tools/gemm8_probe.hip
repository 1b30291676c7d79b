// Where the persistent bf16 GEMM's time goes outside the main loop (round-4 probe, not product code).
// Times gemm8p_kernel in four builds on the WavLM-base B = 256 shapes, interleaved in one process:
//   DBG 0 = the library kernel, 1 = epilogue math without stores, 2 = no epilogue, 3 = stores without math,
//   4 = no epilogue and no MFMA (memory side of the main loop), 5 = no epilogue and no DMA (MFMA / LDS side),
//   6 / 7 = the library kernel with half of every XCD's blocks starting 6 / 12 us late (are the epilogue stores a burst?),
// (round 4 also timed, then removed from the kernel: full-line store patterns, non-temporal stores, stores
// into one L2-resident tile, half the stores, stores spread over the main loop and deferred stores -- the
// measurements and why they were not kept are in DESIGN.md §3 "GEMM epilogue")
// plus a K sweep at fixed M, N (tile time = nk * T_ktile + F: the per-tile fixed cost F).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/gemm8_probe.hip -o tools/_build/gemm8_probe
#include "../stuttering-speech-representation_amd/csrc/kernels_gemm8.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

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

__global__ void fill_bf16(bf16* p, long long n, unsigned seed, float scale) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    p[i] = (bf16)(((float)(h >> 8) * (2.0f / 16777216.0f) - 1.0f) * scale);
  }
}

typedef void (*kfn)(GemmArgs, int);

template <int ACT, int EP>
static kfn pick(int dbg) {
  switch (dbg) {
    case 1: return gemm8p_kernel<ACT, false, false, EP, 1>;
    case 2: return gemm8p_kernel<ACT, false, false, EP, 2>;
    case 3: return gemm8p_kernel<ACT, false, false, EP, 3>;
    case 4: return gemm8p_kernel<ACT, false, false, EP, 4>;
    case 5: return gemm8p_kernel<ACT, false, false, EP, 5>;
    case 6: return gemm8p_kernel<ACT, false, false, EP, 6>;
    case 7: return gemm8p_kernel<ACT, false, false, EP, 7>;
    default: return gemm8p_kernel<ACT, false, false, EP, 0>;
  }
}

typedef void (*kfr)(GemmArgs);
static kfr pick_r(int dbg) {   // the folded post-LN residual GEMM (oproj / ffn2 of WavLM-base bf16)
  switch (dbg) {
    case 2: return gemm8r_kernel<true, true, true, false, 2>;
    case 5: return gemm8r_kernel<true, true, true, false, 5>;
    case 6: return gemm8r_kernel<true, true, true, false, 6>;
    case 7: return gemm8r_kernel<true, true, true, false, 7>;
    default: return gemm8r_kernel<true, true, true, false, 0>;
  }
}

struct Shape { const char* name; int M, N, K, act, ep; int rps = 0; long long seg = 0, lda = 0; };   // rps > 0: conv addressing

// round 6: gemm8h_kernel (two co-resident 256x128 workgroups per CU) against gemm8p_kernel on the K = 768 shapes
typedef void (*kfh)(GemmArgs);
template <int ACT, int EP>
static kfh pick_h(int dbg) {
  switch (dbg) {
    case 2: return gemm8h_kernel<ACT, EP, 2>;
    case 4: return gemm8h_kernel<ACT, EP, 4>;
    case 5: return gemm8h_kernel<ACT, EP, 5>;
    default: return gemm8h_kernel<ACT, EP, 0>;
  }
}

__global__ void count_diff(const unsigned short* a, const unsigned short* b, long long n, unsigned long long* out) {
  unsigned long long c = 0;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    c += a[i] != b[i];
  if (c) atomicAdd(out, c);
}

static int half_tiles(int argc, char** argv);

int main(int argc, char** argv) {
  if (argc > 1 && argv[1][0] == 'h') return half_tiles(argc, argv);
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const Shape shapes[] = {
      {"qkv", 38144, 2560, 768, ACT_NONE, 1},        {"qkv_fold", 38144, 2560, 768, ACT_NONE, 3},
      {"ffn1", 38144, 3072, 768, ACT_GELU_FAST, 1},  {"ffn1_fold", 38144, 3072, 768, ACT_GELU_FAST, 3},
      {"conv1", 1228544, 512, 1536, ACT_GELU_FAST, 0}, {"k1536", 38144, 2560, 1536, ACT_NONE, 1},
      {"k3072", 38144, 2560, 3072, ACT_NONE, 1},
      // conv1 as the library runs it (overlapping k = 3, s = 2 windows over conv0's 256 x 9599 x 512 output:
      // 2.5 GB of A) and the same GEMM with every row tile reading one L2-resident 256-row window -- the
      // bound on what a conv0 -> conv1 fusion could save on conv1's side (its A never leaving the chip)
      {"conv1_real", 1228544, 512, 1536, ACT_GELU_FAST, 0, 4799, 9599LL * 512, 1024},
      {"conv1_l2", 1228544, 512, 1536, ACT_GELU_FAST, 0, 256, 0, 1024},     {"sq4096", 4096, 4096, 4096, ACT_NONE, 0},
  };
  const long long maxA = 1228544LL * 1536, maxB = 4096LL * 4096, maxC = 1228544LL * 512;
  bf16 *a, *b, *c;
  float *bias, *acol;
  float2* apart;
  void* zero;
  CK(hipMalloc(&a, maxA * 2)); CK(hipMalloc(&b, maxB * 2 * 2)); CK(hipMalloc(&c, maxC * 2 * 2));
  CK(hipMalloc(&bias, 4096 * 4)); CK(hipMalloc(&acol, 4096 * 4)); CK(hipMalloc(&apart, 38144LL * 3 * 8));
  CK(hipMalloc(&zero, 256)); CK(hipMemset(zero, 0, 256));
  hipLaunchKernelGGL(fill_bf16, dim3(2048), dim3(256), 0, 0, a, maxA, 17u, 1.0f);
  hipLaunchKernelGGL(fill_bf16, dim3(2048), dim3(256), 0, 0, b, maxB * 2, 91u, 0.036f);
  {
    std::vector<float> h(4096, 0.01f);
    CK(hipMemcpy(bias, h.data(), 4096 * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(acol, h.data(), 4096 * 4, hipMemcpyHostToDevice));
    std::vector<float2> p(38144 * 3, make_float2(0.f, 256.f));
    CK(hipMemcpy(apart, p.data(), p.size() * 8, hipMemcpyHostToDevice));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int ROUNDS = 3, IT = 20;
  {   // residual GEMMs: oproj (K = 768) and ffn2 (K = 3072), N = 768, bf16 stream + LayerNorm partials in / out
    bf16* rs;
    float *lw, *lb;
    float2* op;
    CK(hipMalloc(&rs, 38144LL * 768 * 2)); CK(hipMalloc(&lw, 768 * 4)); CK(hipMalloc(&lb, 768 * 4));
    CK(hipMalloc(&op, 38144LL * 3 * 8));
    hipLaunchKernelGGL(fill_bf16, dim3(2048), dim3(256), 0, 0, rs, 38144LL * 768, 5u, 1.0f);
    CK(hipMemcpy(lw, bias, 768 * 4, hipMemcpyDeviceToDevice)); CK(hipMemcpy(lb, bias, 768 * 4, hipMemcpyDeviceToDevice));
    for (int K : {768, 3072}) {
      GemmArgs g{};
      g.A = a; g.B = b; g.M = 38144; g.N = 768; g.K = K; g.rows_per_seg = g.M; g.lda = K;
      g.bias = bias; g.Ct = c; g.ldc = 768; g.zero = zero; g.resid_t = rs; g.rpart = apart; g.rpart_nt = 3;
      g.rln_w = lw; g.rln_b = lb; g.ln_eps = 1e-5f; g.opart = op;
      const int tiles = 149 * 3;
      double best[8] = {1e30, 1e30, 1e30, 1e30, 1e30, 1e30, 1e30, 1e30};
      for (int r = 0; r < ROUNDS; ++r)
        for (int dbg : {0, 2, 5, 6, 7}) {
          kfr k = pick_r(dbg);
          for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k, dim3(tiles), dim3(512), 0, 0, g);
          CK(hipEventRecord(e0, 0));
          for (int i = 0; i < IT; ++i) hipLaunchKernelGGL(k, dim3(tiles), dim3(512), 0, 0, g);
          CK(hipEventRecord(e1, 0));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          ms /= IT;
          if (ms < best[dbg]) best[dbg] = ms;
        }
      const double tf = 2.0 * 38144 * 768 * K / 1e12;
      printf("%-10s M=38144 N=768 K=%d tiles=%d (gemm8r, one tile per block)\n", K == 768 ? "oproj" : "ffn2", K, tiles);
      const char* nm[8] = {"full", "", "no-epilogue", "", "", "no-stores", "no-opart", "no-math"};
      for (int d : {0, 2, 5, 6, 7})
        printf("   %-14s %8.1f us  %7.1f TF/s\n", nm[d], best[d] * 1e3, tf / (best[d] * 1e-3));
      fflush(stdout);
    }
  }
  for (const Shape& s : shapes) {
    GemmArgs g{};
    g.A = a; g.B = b; g.M = s.M; g.N = s.N; g.K = s.K; g.rows_per_seg = s.M; g.lda = s.K;
    if (s.rps) { g.rows_per_seg = s.rps; g.seg_stride = s.seg; g.lda = s.lda; }
    g.bias = (s.ep & 1) ? bias : nullptr; g.Ct = c; g.ldc = s.N; g.act = s.act; g.zero = zero;
    if (s.ep & 2) { g.apart = apart; g.apart_nt = 3; g.acol = acol; g.ln_eps = 1e-5f; }
    const int n_tiles = ((s.M + 255) / 256) * (s.N / 256);
    const int G = n_tiles < cus ? n_tiles : cus;
    const double tf = 2.0 * s.M * s.N * s.K / 1e12;
    double best[8] = {1e30, 1e30, 1e30, 1e30, 1e30, 1e30, 1e30, 1e30};
    for (int r = 0; r < ROUNDS; ++r)
      for (int dbg = 0; dbg < 8; ++dbg) {
        kfn k;
        if (s.act == ACT_GELU_FAST) k = s.ep == 3 ? pick<ACT_GELU_FAST, 3>(dbg) : (s.ep == 1 ? pick<ACT_GELU_FAST, 1>(dbg) : pick<ACT_GELU_FAST, 0>(dbg));
        else k = s.ep == 3 ? pick<ACT_NONE, 3>(dbg) : (s.ep == 1 ? pick<ACT_NONE, 1>(dbg) : pick<ACT_NONE, 0>(dbg));
        for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k, dim3(G), dim3(512), 0, 0, g, n_tiles);
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < IT; ++i) hipLaunchKernelGGL(k, dim3(G), dim3(512), 0, 0, g, n_tiles);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= IT;
        if (ms < best[dbg]) best[dbg] = ms;
      }
    const double rounds = (double)n_tiles / cus;
    printf("%-10s M=%d N=%d K=%d tiles=%d (%.2f rounds)\n", s.name, s.M, s.N, s.K, n_tiles, rounds);
    const char* nm[8] = {"full", "math,no-store", "no-epilogue", "store,no-math", "no-ep,no-mfma", "no-ep,no-dma",
                         "full,odd+6us", "full,odd+12us"};
    for (int d = 0; d < 8; ++d)
      printf("   %-14s %8.1f us  %7.1f TF/s  per-round %.2f us\n", nm[d], best[d] * 1e3, tf / (best[d] * 1e-3),
             best[d] * 1e3 / __builtin_ceil(rounds));
    fflush(stdout);
  }
  return 0;
}

// h [rounds]: per shape, gemm8p (the library's persistent 256x256 kernel) vs gemm8h (256x128, two workgroups per
// CU) in interleaved rounds: full launch, gemm8h without epilogue / MFMA / DMA; outputs compared bit for bit.
static int half_tiles(int argc, char** argv) {
  const int ROUNDS = argc > 2 ? atoi(argv[2]) : 3, IT = 20;
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, gemm8h_kernel<ACT_NONE, 1, 0>, 256, 0));
  printf("gemm8h: %d workgroups per CU (occupancy API), %d CUs\n", occ, cus);
  struct S { const char* name; int M, N, K, act, ep; };
  const S shapes[] = {{"qkv", 38144, 2560, 768, ACT_NONE, 1},          {"qkv_fold", 38144, 2560, 768, ACT_NONE, 3},
                      {"ffn1", 38144, 3072, 768, ACT_GELU_FAST, 1},    {"ffn1_fold", 38144, 3072, 768, ACT_GELU_FAST, 3},
                      {"proj", 38144, 768, 512, ACT_NONE, 1},          {"k3072", 38144, 2560, 3072, ACT_NONE, 1},
                      {"m4099", 4099, 768, 768, ACT_GELU_FAST, 3}};
  const long long maxA = 38144LL * 3072, maxB = 3072LL * 3072, maxC = 38144LL * 3072;
  bf16 *a, *b, *c0, *c1;
  float *bias, *acol;
  float2* apart;
  void* zero;
  unsigned long long* nd;
  CK(hipMalloc(&a, maxA * 2)); CK(hipMalloc(&b, maxB * 2)); CK(hipMalloc(&c0, maxC * 2)); CK(hipMalloc(&c1, maxC * 2));
  CK(hipMalloc(&bias, 4096 * 4)); CK(hipMalloc(&acol, 4096 * 4)); CK(hipMalloc(&apart, 38144LL * 3 * 8));
  CK(hipMalloc(&zero, 256)); CK(hipMemset(zero, 0, 256)); CK(hipMalloc(&nd, 8));
  hipLaunchKernelGGL(fill_bf16, dim3(2048), dim3(256), 0, 0, a, maxA, 17u, 1.0f);
  hipLaunchKernelGGL(fill_bf16, dim3(2048), dim3(256), 0, 0, b, maxB, 91u, 0.036f);
  {
    std::vector<float> h(4096);
    for (int i = 0; i < 4096; ++i) h[i] = 0.01f * (float)((i * 37) % 101 - 50);
    CK(hipMemcpy(bias, h.data(), 4096 * 4, hipMemcpyHostToDevice));
    for (int i = 0; i < 4096; ++i) h[i] = 0.5f + 0.001f * (float)((i * 53) % 97);
    CK(hipMemcpy(acol, h.data(), 4096 * 4, hipMemcpyHostToDevice));
    std::vector<float2> p(38144 * 3);
    for (size_t i = 0; i < p.size(); ++i) p[i] = make_float2(0.01f * (float)((i * 29) % 61 - 30), 200.f + (float)(i % 113));
    CK(hipMemcpy(apart, p.data(), p.size() * 8, hipMemcpyHostToDevice));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (const S& s : shapes) {
    GemmArgs g{};
    g.A = a; g.B = b; g.M = s.M; g.N = s.N; g.K = s.K; g.rows_per_seg = s.M; g.lda = s.K;
    g.bias = (s.ep & 1) ? bias : nullptr; g.ldc = s.N; g.act = s.act; g.zero = zero;
    if (s.ep & 2) { g.apart = apart; g.apart_nt = 3; g.acol = acol; g.ln_eps = 1e-5f; }
    const int n_tiles = ((s.M + 255) / 256) * (s.N / 256), h_tiles = ((s.M + 255) / 256) * (s.N / 128);
    const int G = n_tiles < cus ? n_tiles : cus;
    kfn kp;
    kfh kh[4];
    const int hd[4] = {0, 2, 4, 5};
    if (s.act == ACT_GELU_FAST) {
      kp = s.ep == 3 ? pick<ACT_GELU_FAST, 3>(0) : pick<ACT_GELU_FAST, 1>(0);
      for (int d = 0; d < 4; ++d) kh[d] = s.ep == 3 ? pick_h<ACT_GELU_FAST, 3>(hd[d]) : pick_h<ACT_GELU_FAST, 1>(hd[d]);
    } else {
      kp = s.ep == 3 ? pick<ACT_NONE, 3>(0) : pick<ACT_NONE, 1>(0);
      for (int d = 0; d < 4; ++d) kh[d] = s.ep == 3 ? pick_h<ACT_NONE, 3>(hd[d]) : pick_h<ACT_NONE, 1>(hd[d]);
    }
    // bit identity of the two library forms
    CK(hipMemset(c0, 0xFF, (size_t)s.M * s.N * 2)); CK(hipMemset(c1, 0xEE, (size_t)s.M * s.N * 2));
    g.Ct = c0;
    hipLaunchKernelGGL(kp, dim3(G), dim3(512), 0, 0, g, n_tiles);
    g.Ct = c1;
    hipLaunchKernelGGL(kh[0], dim3(h_tiles), dim3(256), 0, 0, g);
    CK(hipMemset(nd, 0, 8));
    hipLaunchKernelGGL(count_diff, dim3(1024), dim3(256), 0, 0, (const unsigned short*)c0, (const unsigned short*)c1,
                       (long long)s.M * s.N, nd);
    unsigned long long ndh = 0;
    CK(hipMemcpy(&ndh, nd, 8, hipMemcpyDeviceToHost));
    g.Ct = c1;
    double best[5] = {1e30, 1e30, 1e30, 1e30, 1e30};
    for (int r = 0; r < ROUNDS; ++r)
      for (int v = 0; v < 5; ++v) {
        auto go = [&] {
          if (v == 0) hipLaunchKernelGGL(kp, dim3(G), dim3(512), 0, 0, g, n_tiles);
          else hipLaunchKernelGGL(kh[v - 1], dim3(h_tiles), dim3(256), 0, 0, g);
        };
        for (int w = 0; w < 3; ++w) go();
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < IT; ++i) go();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= IT;
        if (ms < best[v]) best[v] = ms;
      }
    const double tf = 2.0 * s.M * s.N * s.K / 1e12;
    printf("%-10s M=%d N=%d K=%d  256x256 tiles %d (%.2f rounds), 256x128 tiles %d; differing outputs %llu\n", s.name, s.M,
           s.N, s.K, n_tiles, (double)n_tiles / cus, h_tiles, ndh);
    const char* nm[5] = {"gemm8p (lib)", "gemm8h full", "gemm8h no-epi", "gemm8h no-mfma", "gemm8h no-dma"};
    for (int v = 0; v < 5; ++v)
      printf("   %-16s %8.1f us  %7.1f TF/s\n", nm[v], best[v] * 1e3, tf / (best[v] * 1e-3));
    fflush(stdout);
  }
  return 0;
}
