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

namespace {
// ======================================================================================
// Two co-resident 256x128 workgroups per CU (round 6, VERDICT r5 item 1: hide one tile's epilogue under
// the other tile's main loop).  gemm8p_kernel holds a 256x256 fp32 accumulator tile = half of every SIMD's
// 512-entry register file, so the next tile's MFMAs cannot run while a tile drains its epilogue; the per-CU
// store path (~23 B/clk) leaves ~25 % of a K = 768 round exposed.  Here a workgroup is 4 waves
// (one per SIMD) owning a 256-row x 128-column tile (128 accumulator registers per lane), two workgroups per
// CU (launch bounds: <= 256 VGPRs; 80 KiB of LDS each), one tile per workgroup: while one workgroup runs its
// epilogue or its prologue, the other one's MFMAs keep the SIMDs' matrix pipes busy, and the dispatcher
// starts the next tile in the freed slot.  The price is operand traffic: per 64-deep K step 96 KiB per
// 256 x 256 of output instead of 64 (A is read by both column halves).
//   * K-tile = 32 (64 B per row), a 3-stage LDS ring of A 256 x 64 B | B 128 x 64 B (24 KiB per stage): the
//     stage of K-tile t + 2 is issued right after the barrier of K-tile t (its buffer held K-tile t - 1, whose
//     reads finished before that barrier), so every LDS-DMA has two K-tiles of MFMAs to land.
//   * 16-B chunk c of row r holds logical chunk c ^ swz(r), swz = [0, 2, 3, 1][(r >> 2) & 3]: the MFMA
//     fragment reads (lane (q, r16) reads chunk q of row r16) are conflict-free in ds_read_b128's 16-lane groups
//     with 64-B rows (the 128-B-row swizzle of gemm8p does not apply).
//   * wave (wm, wn) of the 2 x 2 grid owns rows wm*128 + [0, 128) and columns wn*64 + [0, 64): per K-tile 8 A
//     and 4 B fragments (12 ds_read_b128), 32 MFMAs 16x16x32 computing C^T blocks (the same products in the
//     same K order as gemm8p_kernel: outputs bit-identical to it, tests/test_gpu_kernels.py).
//   * epilogue parameters (bias, folded-LN column sums, the rows' LayerNorm partials) go to LDS by DMA before
//     the operand prologue and are retired by the first counted wait; the epilogue is g8p_epilogue's
//     arithmetic on this tile's layout, stores through per-16-row-block buffer resources (rows >= M dropped).
// (Probe-only since the measurement: the library keeps gemm8p_kernel)
// LDS: 3 x 24 KiB operands | bias [0, 512) acol [1 K, 1.5 K) partials [2 K, 8 K) = 80 KiB per workgroup.
constexpr int G8H_STAGE = 24 * 1024;
constexpr int G8H_OPS = 3 * G8H_STAGE;
constexpr int G8H_SMEM = G8H_OPS + 8 * 1024;

// chunk swizzle of a 64-B row (see above): [0, 2, 3, 1] by (row >> 2) & 3
SSE_DEV int g8h_swz(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }

// DBG (timing probes only, tools/gemm8_probe.hip; the library launches DBG = 0): 2 = no epilogue
// (accumulators kept live), 4 = no epilogue and no MFMA (the fragment reads kept live), 5 = no epilogue and
// no main-loop LDS-DMA.
template <int ACT, int EP = 1, int DBG = 0, int FNT = 3>
__global__ __launch_bounds__(256, 2) void gemm8h_kernel(GemmArgs g) {
  static_assert(FNT == 3, "the parameter DMA stages 6 KiB of row partials (H = 768)");
  __shared__ __attribute__((aligned(16))) char smem[G8H_SMEM];   // the ONLY shared object
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int q = lane >> 4, r16 = lane & 15;
  const int M = g.M, K = g.K;
  const int n_tiles_n = g.N / 128;
  const int nk = K / 32;
  constexpr bool has_bias = (EP & 1) != 0, fold = (EP & 2) != 0;
  int bid = blockIdx.x;
  {   // XCD-aware bijective remap: XCD x walks a contiguous range of row-major tiles
    const int nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, x = bid % 8;
    bid = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + bid / 8;
  }
  const int m0 = (bid / n_tiles_n) * 256, n0 = (bid % n_tiles_n) * 128;
  char* const ep = smem + G8H_OPS;

  // ---- epilogue parameters into LDS first (2 DMAs per wave, retired by the first counted wait): waves 0-2 the
  // row partials (2 KiB each), wave 3 the bias and the column sums (512 B each, the other half-piece reads zeros)
  {
    const void* zb = g.zero;
    if (wave < 3) {
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(fold ? (const void*)g.apart : zb), (short)0, fold ? M * FNT * 8 : 0, 0x00020000);
      #pragma unroll
      for (int u = 0; u < 2; ++u)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, LPTR(ep + 2048 + (2 * wave + u) * 1024), 16, (unsigned)lane * 16u,
                                                 (unsigned)(m0 * FNT * 8 + (2 * wave + u) * 1024), 0, 0);
    } else {
      const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(has_bias ? (const void*)(g.bias + n0) : zb), (short)0, has_bias ? 512 : 0, 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, LPTR(ep), 16, (unsigned)lane * 16u, 0u, 0, 0);
      const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(fold ? (const void*)(g.acol + n0) : zb), (short)0, fold ? 512 : 0, 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, LPTR(ep + 1024), 16, (unsigned)lane * 16u, 0u, 0, 0);
    }
  }

  // ---- LDS-DMA sources: one descriptor per operand based at the tile's first row, per-lane byte offsets fixed
  // over K, the scalar offset advancing 64 B per K-tile.  Piece p (1 KiB) = rows 16p .. 16p + 15: lane l writes
  // LDS chunk l & 3 of row 16p + (l >> 2), which holds logical chunk (l & 3) ^ swz(row).  A: pieces wave + 4u
  // (u < 4), B: pieces wave + 4u (u < 2).
  constexpr int NREC = 0x7FFFFFF0;
  __amdgpu_buffer_rsrc_t a_rsrc, b_rsrc;
  unsigned a_voff[4], b_voff[2];
  {
    const int mf = m0 < M ? m0 : M - 1;
    const int seg0 = mf / g.rows_per_seg, rr0 = mf - seg0 * g.rows_per_seg;
    const long long a_base = ((long long)seg0 * g.seg_stride + (long long)rr0 * g.lda) * 2;   // bytes
    a_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)g.A + a_base), (short)0, NREC, 0x00020000);
    b_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)g.B + (long long)n0 * K * 2), (short)0, NREC,
                                               0x00020000);
    #pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int row = (wave + 4 * u) * 16 + (lane >> 2);
      const int ch = (lane & 3) ^ g8h_swz(row);
      int m = m0 + row;
      m = m < M ? m : M - 1;
      const int seg = m / g.rows_per_seg, rr = m - seg * g.rows_per_seg;
      const long long el = ((long long)seg * g.seg_stride + (long long)rr * g.lda) * 2 + ch * 16;
      a_voff[u] = (unsigned)(el - a_base);
      if (u < 2) b_voff[u] = (unsigned)((long long)row * K * 2 + ch * 16);
    }
  }
  auto issue = [&](int t, int buf) {   // K-tile t into ring slot buf (6 LDS-DMA per wave)
    char* dst = smem + buf * G8H_STAGE;
    const unsigned soff = (unsigned)t * 64u;
    #pragma unroll
    for (int u = 0; u < 4; ++u)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, LPTR(dst + (wave + 4 * u) * 1024), 16, a_voff[u], soff, 0, 0);
    #pragma unroll
    for (int u = 0; u < 2; ++u)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, LPTR(dst + 16384 + (wave + 4 * u) * 1024), 16, b_voff[u], soff,
                                               0, 0);
  };

  f32x4 acc[2][2][4][2];   // [mi][ni][i][j]: rows wm*128 + mi*64 + i*16 + r16, columns wn*64 + ni*32 + j*16 + 4q
  #pragma unroll
  for (int a = 0; a < 2; ++a)
    #pragma unroll
    for (int c = 0; c < 2; ++c)
      #pragma unroll
      for (int i = 0; i < 4; ++i)
        #pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][c][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // this lane's fragment byte offset inside a 16-row block: row r16, logical chunk q (rows 16k + r16 share it)
  const int frag = r16 * 64 + ((q ^ g8h_swz(r16)) << 4);
  const int a_frag = (wm * 128) * 64 + frag, b_frag = 16384 + (wn * 64) * 64 + frag;
  auto k_tile = [&](int buf) {
    const char* s = smem + buf * G8H_STAGE;
    bf16x8 af[8], bfr[4];
    #pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = *(const bf16x8*)(s + b_frag + j * 1024);
    #pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = *(const bf16x8*)(s + a_frag + i * 1024);
    if constexpr (DBG == 4) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      #pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("" ::"v"(af[i]));
      #pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(bfr[j]));
      return;
    }
    #pragma unroll
    for (int i = 0; i < 8; ++i)
      #pragma unroll
      for (int j = 0; j < 4; ++j) {
        f32x4& c = acc[i >> 2][j >> 1][i & 3][j & 1];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], c, 0, 0, 0);
      }
  };

  // ---- main loop: wait for K-tile t (this wave's 6 DMAs of t + 1 may stay in flight), barrier (every wave's
  // DMAs of t landed; every wave's reads of t - 1 done), issue t + 2 into t - 1's slot, compute t
  if constexpr (DBG != 5) {
    issue(0, 0);
    if (nk > 1) issue(1, 1);
  }
  int buf = 0;   // ring slot of K-tile t
  int t = 0;
  for (; t + 2 < nk; ++t) {
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    g8_barrier();
    if constexpr (DBG != 5) issue(t + 2, buf == 0 ? 2 : buf - 1);
    k_tile(buf);
    buf = buf == 2 ? 0 : buf + 1;
  }
  for (; t < nk; ++t) {
    if (t + 1 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    g8_barrier();
    k_tile(buf);
    buf = buf == 2 ? 0 : buf + 1;
  }
  if constexpr (DBG == 5) {   // (the parameter DMA is still to be waited for)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if constexpr (DBG == 2 || DBG == 4 || DBG == 5) {
    #pragma unroll
    for (int a = 0; a < 2; ++a)
      #pragma unroll
      for (int c = 0; c < 2; ++c)
        #pragma unroll
        for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(acc[a][c][i][0]), "v"(acc[a][c][i][1]));
    return;
  }

  // ---- epilogue (g8p_epilogue's arithmetic): o = act(rstd_m acc + (bias[n] - rstd_m mean_m acol[n])), or
  // act(acc + bias[n]) without the fold; bf16 pairs of lanes (q, q ^ 1) exchanged so each lane stores 8
  // consecutive columns (one 16-B store per (mi, i, ni))
  {   // lane-derived values from an opaque lane id (kept out of the main loop's registers)
    int ln = (int)(threadIdx.x & 63);
    asm volatile("" : "+v"(ln));
    const int qq = ln >> 4, rr = ln & 15;
    f32x4 bv[2][2], ac[2][2];
    #pragma unroll
    for (int ni = 0; ni < 2; ++ni)
      #pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = wn * 64 + ni * 32 + j * 16 + qq * 4;
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        const f32x4 b = *(const f32x4*)(ep + c * 4), a = *(const f32x4*)(ep + 1024 + c * 4);
        bv[ni][j] = has_bias ? b : z;
        ac[ni][j] = fold ? a : z;
      }
    auto finish_half = [&](int mi) {
      asm volatile("" ::: "memory");
      float2 ast[4];
      #pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float2* p = (const float2*)(ep + 2048) + (wm * 128 + mi * 64 + i * 16 + rr) * FNT;
        float2 v[FNT];
        #pragma unroll
        for (int u = 0; u < FNT; ++u) v[u] = p[u];
        const float2 st = ln_part_combine<FNT>(v, g.ln_eps);
        ast[i] = fold ? st : make_float2(0.f, 1.f);
      }
      #pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float rs = ast[i].y, nm = -ast[i].x * ast[i].y;
        #pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          #pragma unroll
          for (int j = 0; j < 2; ++j) {
            f32x4 o;
            #pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = fmaf(acc[mi][ni][i][j][e], rs, fmaf(nm, ac[ni][j][e], bv[ni][j][e]));
            if constexpr (ACT == ACT_GELU) {
              const f32x2 lo = gelu_erf2(f32x2{o[0], o[1]}), hi = gelu_erf2(f32x2{o[2], o[3]});
              o = f32x4{lo.x, lo.y, hi.x, hi.y};
            }
            acc[mi][ni][i][j] = o;
          }
        if constexpr (ACT == ACT_GELU_FAST) {
          f32x2 o2[8];
          #pragma unroll
          for (int u = 0; u < 4; ++u) {
            const f32x4 v = acc[mi][u >> 1][i][u & 1];
            o2[2 * u] = f32x2{v[0], v[1]};
            o2[2 * u + 1] = f32x2{v[2], v[3]};
          }
          gelu_out2_n<false, 8>(o2);
          #pragma unroll
          for (int u = 0; u < 4; ++u) acc[mi][u >> 1][i][u & 1] = f32x4{o2[2 * u].x, o2[2 * u].y, o2[2 * u + 1].x, o2[2 * u + 1].y};
        }
      }
    };
    const unsigned lane_off = (unsigned)((rr * g.ldc + wn * 64 + (qq & 1) * 16 + (qq >> 1) * 8) * 2);
    auto store_half = [&](int mi) {
      #pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long long r0 = (long long)m0 + wm * 128 + mi * 64 + i * 16, rows = (long long)M - r0;
        const long long nrec = rows > 0 ? (rows * g.ldc - n0) * 2 : 0;
        const __amdgpu_buffer_rsrc_t cr = __builtin_amdgcn_make_buffer_rsrc(
            (void*)((bf16*)g.Ct + (rows > 0 ? r0 * g.ldc + n0 : 0)), (short)0, (int)min(nrec, (long long)0x7FFFFFF0),
            0x00020000);
        #pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
          const f32x4 o0 = acc[mi][ni][i][0], o1 = acc[mi][ni][i][1];
          const bf16x4 x0 = {(bf16)o0[0], (bf16)o0[1], (bf16)o0[2], (bf16)o0[3]};
          const bf16x4 x1 = {(bf16)o1[0], (bf16)o1[1], (bf16)o1[2], (bf16)o1[3]};
          const uint2 X = __builtin_bit_cast(uint2, x0), Y = __builtin_bit_cast(uint2, x1);
          const auto s0 = __builtin_amdgcn_permlane16_swap(X.x, Y.x, false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(X.y, Y.y, false, false);
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{s0[0], s1[0], s0[1], s1[1]}, cr, lane_off + (unsigned)(ni * 64), 0u, 0);
        }
      }
    };
    finish_half(0);
    store_half(0);
    finish_half(1);
    store_half(1);
  }
}

}  // namespace

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

static bool g_ph2 = true;   // round 6: the library's two-phase K-tile schedule (argument "4": the four-phase one)
template <int ACT, int EP, bool P2>
static kfn pick2(int dbg) {
  switch (dbg) {
    case 1: return gemm8p_kernel<ACT, false, false, EP, 1, 3, P2>;
    case 2: return gemm8p_kernel<ACT, false, false, EP, 2, 3, P2>;
    case 3: return gemm8p_kernel<ACT, false, false, EP, 3, 3, P2>;
    case 4: return gemm8p_kernel<ACT, false, false, EP, 4, 3, P2>;
    case 5: return gemm8p_kernel<ACT, false, false, EP, 5, 3, P2>;
    case 6: return gemm8p_kernel<ACT, false, false, EP, 6, 3, P2>;
    case 7: return gemm8p_kernel<ACT, false, false, EP, 7, 3, P2>;
    default: return gemm8p_kernel<ACT, false, false, EP, 0, 3, P2>;
  }
}
template <int ACT, int EP>
static kfn pick(int dbg) {
  return g_ph2 ? pick2<ACT, EP, true>(dbg) : pick2<ACT, EP, false>(dbg);
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
  if (argc > 1 && argv[1][0] == '4') g_ph2 = false;
  printf("persistent GEMM schedule: %s phases per K-tile\n", g_ph2 ? "two" : "four");
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
