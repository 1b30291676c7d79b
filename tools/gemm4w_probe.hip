// Round-3 groundwork probe: a 256x256 bf16 GEMM tile on 4 waves (one wave per SIMD, each wave a
// 128x128 sub-tile in 256 accumulator registers) against the library's 8-wave 8-phase kernel
// (sse_gemm, same buffers, same box).  Per 64-deep K-tile the 4-wave form reads 128 KiB of LDS
// fragments instead of 192 KiB and has one barrier instead of eight ("Why the GEMM
// main loop sits at ≈54 %").  Not part of the library; build and run:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gemm4w_probe.hip -o tools/_build/gemm4w_probe -ldl
//   tools/_build/gemm4w_probe            (from the repo root, so libsse.so is found)
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "../stuttering-speech-representation_amd/csrc/common.h"

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef unsigned int u32x2_w4 __attribute__((ext_vector_type(2)));

constexpr int W4_HALF = 256 * 128;     // one operand's K-tile: 256 rows x 128 B (64 bf16)
constexpr int W4_BUF = 2 * W4_HALF;    // A | B
constexpr int W4_SMEM = 2 * W4_BUF;    // two K-tiles in flight: 128 KiB

template <int I, int N, typename F>
SSE_DEV void g8_sfor_w4(F&& f) {   // f(integral_constant<int, I>) for I .. N-1
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    g8_sfor_w4<I + 1, N>(f);
  }
}

SSE_DEV void w4_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// ILV = 1: interleave the next fragment reads / LDS-DMA issues between the MFMAs with
// sched_group_barrier; ILV = 0: leave the order to the compiler.
template <int ILV, bool UNI = false, bool ASM = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm4w_kernel(
    const bf16* __restrict__ A, const bf16* __restrict__ B, bf16* __restrict__ C, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char smem[W4_SMEM];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int q = lane >> 4, r16 = lane & 15;
  const int ntn = N / 256, MT = (M + 255) / 256;
  int bid = blockIdx.x;
  {   // XCD-aware bijective remap, then 8-row-tile groups (row fastest)
    const int nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, x = bid % 8;
    bid = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + bid / 8;
  }
  constexpr int GM = 8;
  const int first = (bid / (GM * ntn)) * GM, gm = MT - first < GM ? MT - first : GM;
  const int rr = bid - first * ntn;
  const int m0 = (first + rr % gm) * 256, n0 = (rr / gm) * 256;
  const int nk = K / 64;

  constexpr int NREC = 0x7FFFFFF0;
  const __amdgpu_buffer_rsrc_t a_rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)(A + (long long)m0 * K), (short)0, NREC, 0x00020000);
  const __amdgpu_buffer_rsrc_t b_rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)(B + (long long)n0 * K), (short)0, NREC, 0x00020000);
  unsigned av[8], bv[8];
  #pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int row = (s * 4 + wave) * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ ((row >> 1) & 7);
    const int m = m0 + row < M ? row : M - 1 - m0;
    av[s] = (unsigned)(m * K * 2 + ch * 16);
    bv[s] = (unsigned)(row * K * 2 + ch * 16);
  }
  auto issue = [&](int t, auto s_c) {   // LDS-DMA piece s of K-tile t (A and B)
    constexpr int s = decltype(s_c)::value;
    char* dst = smem + (t & 1) * W4_BUF + (s * 4 + wave) * 1024;
    const unsigned so = (unsigned)(t < nk ? t : nk - 1) * 128u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, LPTR(dst), 16, av[s], so, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, LPTR(dst + W4_HALF), 16, bv[s], so, 0, 0);
  };
  auto issue_all = [&](int t) {
    issue(t, std::integral_constant<int, 0>{}); issue(t, std::integral_constant<int, 1>{});
    issue(t, std::integral_constant<int, 2>{}); issue(t, std::integral_constant<int, 3>{});
    issue(t, std::integral_constant<int, 4>{}); issue(t, std::integral_constant<int, 5>{});
    issue(t, std::integral_constant<int, 6>{}); issue(t, std::integral_constant<int, 7>{});
  };

  const int swz = (r16 >> 1) & 7;
  bf16x8 a0[8], b0[8], a1[8], b1[8];
  auto load_k = [&](bf16x8 (&ra)[8], bf16x8 (&rb)[8], int t, int ks) {
    const char* ba = smem + (t & 1) * W4_BUF + (wm * 128 + r16) * 128 + (((q + 4 * ks) ^ swz) * 16);
    const char* bb = smem + (t & 1) * W4_BUF + W4_HALF + (wn * 128 + r16) * 128 + (((q + 4 * ks) ^ swz) * 16);
    #pragma unroll
    for (int i = 0; i < 8; ++i) {
      ra[i] = *(const bf16x8*)(ba + i * 16 * 128);
      rb[i] = *(const bf16x8*)(bb + i * 16 * 128);
    }
  };
  f32x4 acc[8][8];
  #pragma unroll
  for (int i = 0; i < 8; ++i)
    #pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const bf16x8 (&ra)[8], const bf16x8 (&rb)[8]) {
    #pragma unroll
    for (int i = 0; i < 8; ++i)
      #pragma unroll
      for (int j = 0; j < 8; ++j) {
        if constexpr (ASM)   // accumulator tied in place ("+a"): no spare AGPR quad, no rotation copies
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(rb[j]), "v"(ra[i]));
        else
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rb[j], ra[i], acc[i][j], 0, 0, 0);
      }
  };

  // s_waitcnt through the builtin so the compiler's own wait insertion sees it (an asm wait is
  // invisible to it and it re-waits on reads issued after it): gfx9 encoding, expcnt 7 = no wait
  constexpr int WAIT_ALL = 0x0070;              // vmcnt(0) lgkmcnt(0)
  constexpr int WAIT_VM16 = 0x4F70;             // vmcnt(16)
  issue_all(0);
  if (nk > 1) {
    issue_all(1);
    __builtin_amdgcn_s_waitcnt(WAIT_VM16);
  } else {
    __builtin_amdgcn_s_waitcnt(WAIT_ALL);
  }
  w4_barrier();
  load_k(a0, b0, 0, 0);
  // one K-tile; ISSUE / LOAD are compile-time so the steady-state body has no branches
  auto step = [&](int t, auto issue_c, auto load_c) {
    load_k(a1, b1, t, 1);
    mma(a0, b0);
    if constexpr (ILV) {
      #pragma unroll
      for (int u = 0; u < 16; ++u) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // one ds_read
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);   // four MFMAs
      }
    }
    __builtin_amdgcn_s_waitcnt(WAIT_ALL);
    w4_barrier();
    if constexpr (decltype(issue_c)::value) issue_all(t + 2);   // into the buffer every wave has finished reading
    if constexpr (decltype(load_c)::value) load_k(a0, b0, t + 1, 0);
    mma(a1, b1);
    if constexpr (ILV) {
      #pragma unroll
      for (int u = 0; u < 16; ++u) {
        if constexpr (decltype(issue_c)::value) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // one LDS-DMA
        if constexpr (decltype(load_c)::value) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);    // one ds_read
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);                                           // four MFMAs
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  // ASM form, interleaved by hand (asm volatile keeps the source order): per row i of the wave's
  // 8x8 blocks, 8 in-place MFMAs then the next fragment pair (2 ds_read) and, after the barrier,
  // one LDS-DMA piece (2 buffer loads) -- 128 MFMA cycles per 2 + 2 memory instructions
  auto load_frag = [&](bf16x8 (&ra)[8], bf16x8 (&rb)[8], int t, int ks, int i) {
    const char* ba = smem + (t & 1) * W4_BUF + (wm * 128 + r16) * 128 + (((q + 4 * ks) ^ swz) * 16);
    const char* bb = smem + (t & 1) * W4_BUF + W4_HALF + (wn * 128 + r16) * 128 + (((q + 4 * ks) ^ swz) * 16);
    ra[i] = *(const bf16x8*)(ba + i * 16 * 128);
    rb[i] = *(const bf16x8*)(bb + i * 16 * 128);
  };
  auto mma_row = [&](const bf16x8 (&ra)[8], const bf16x8 (&rb)[8], int i) {
    #pragma unroll
    for (int j = 0; j < 8; ++j)
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(rb[j]), "v"(ra[i]));
  };
  auto step_asm = [&](int t) {
    g8_sfor_w4<0, 8>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      mma_row(a0, b0, i);
      load_frag(a1, b1, t, 1, i);
    });
    __builtin_amdgcn_s_waitcnt(WAIT_ALL);
    w4_barrier();
    g8_sfor_w4<0, 8>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      issue(t + 2, ic);
      mma_row(a1, b1, i);
      load_frag(a0, b0, t + 1, 0, i);
    });
  };
  using T_ = std::integral_constant<bool, true>;
  using F_ = std::integral_constant<bool, false>;
  if constexpr (ASM) {
    for (int t = 0; t < nk; ++t) step_asm(t);
  } else if constexpr (UNI) {
    // uniform body: the last two iterations re-load tile nk-1 into a buffer nobody reads again
    // and read fragments of a dead buffer, so every iteration is the same straight-line code
    for (int t = 0; t < nk; ++t) step(t, T_{}, T_{});
  } else {
    int t = 0;
    for (; t + 2 < nk; ++t) step(t, T_{}, T_{});
    if (t + 1 < nk) step(t++, F_{}, T_{});
    step(t, F_{}, F_{});
  }
  __builtin_amdgcn_s_waitcnt(WAIT_ALL);   // no LDS-DMA may land after the block releases its LDS
  if constexpr (ASM) {   // MFMA write latency, then pin every accumulator read behind it (see gemm4p_kernel)
    asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
    #pragma unroll
    for (int i = 0; i < 8; ++i)
      asm volatile("" : "+a"(acc[i][0]), "+a"(acc[i][1]), "+a"(acc[i][2]), "+a"(acc[i][3]), "+a"(acc[i][4]),
                   "+a"(acc[i][5]), "+a"(acc[i][6]), "+a"(acc[i][7]));
  }
  // C^T blocks: lane holds C[row r16][cols 4q .. 4q+3] of each 16x16 block
  #pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wm * 128 + i * 16 + r16;
    if (m < M) {
      #pragma unroll
      for (int j = 0; j < 8; ++j) {
        const f32x4 v = acc[i][j];
        *(bf16x4*)(C + (long long)m * N + n0 + wn * 128 + j * 16 + 4 * q) =
            bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
      }
    }
  }
}


// Persistent form of the ASM kernel: a block walks tiles b, b + G, ...; after a tile's last
// fragment reads it issues the next tile's K-tiles 0 and 1 of LDS-DMA, then runs its last 64 MFMAs
// with each row block's C stores (buffer stores, exactly 64 per wave) right behind that block's
// MFMAs; vmcnt retires in issue order, so the next tile's vmcnt(63) waits for both K-tiles but not
// for the stores.  The first K-tile's MFMAs take srcC = 0 (no accumulator reset).
// One block per CU (512 registers, 128 KiB of LDS): no co-resident block hides an exposed epilogue.
template <int GM>   // tile raster: GM row tiles per group, row fastest (GM = 1: row-major)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm4p_kernel(
    const bf16* __restrict__ A, const bf16* __restrict__ B, bf16* __restrict__ C, int M, int N, int K, int n_tiles) {
  __shared__ __attribute__((aligned(16))) char smem[W4_SMEM];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int q = lane >> 4, r16 = lane & 15;
  const int ntn = N / 256, MT = (M + 255) / 256;
  const int nk = K / 64;
  constexpr int WAIT_ALL = 0x0070, WAIT_VM16 = 0x4F70, WAIT_VM63 = 0xCF7F;   // vmcnt 63 = hi 0b11, lo 0xF
  constexpr int NREC = 0x7FFFFFF0;
  const __amdgpu_buffer_rsrc_t c_rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)C, (short)0, (int)((long long)M * N * 2 < NREC ? (long long)M * N * 2 : NREC), 0x00020000);
  auto tile_origin = [&](int tid, int& m0, int& n0) {
    const int q8 = n_tiles / 8, r8 = n_tiles % 8, x = tid % 8;
    int bid = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + tid / 8;
    const int first = (bid / (GM * ntn)) * GM, gm = MT - first < GM ? MT - first : GM;
    const int rr = bid - first * ntn;
    m0 = (first + rr % gm) * 256;
    n0 = (rr / gm) * 256;
  };
  __amdgpu_buffer_rsrc_t a_rsrc, b_rsrc;
  unsigned av[8], bv[8];
  auto setup = [&](int m0, int n0) {
    a_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (long long)m0 * K), (short)0, NREC, 0x00020000);
    b_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)(B + (long long)n0 * K), (short)0, NREC, 0x00020000);
    #pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int row = (s * 4 + wave) * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ ((row >> 1) & 7);
      const int m = m0 + row < M ? row : M - 1 - m0;
      av[s] = (unsigned)(m * K * 2 + ch * 16);
      bv[s] = (unsigned)(row * K * 2 + ch * 16);
    }
  };
  auto issue = [&](int t, auto s_c) {
    constexpr int s = decltype(s_c)::value;
    char* dst = smem + (t & 1) * W4_BUF + (s * 4 + wave) * 1024;
    const unsigned so = (unsigned)(t < nk ? t : nk - 1) * 128u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, LPTR(dst), 16, av[s], so, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, LPTR(dst + W4_HALF), 16, bv[s], so, 0, 0);
  };
  auto issue_all = [&](int t) { g8_sfor_w4<0, 8>([&](auto sc) { issue(t, sc); }); };
  const int swz = (r16 >> 1) & 7;
  bf16x8 a0[8], b0[8], a1[8], b1[8];
  auto load_frag = [&](bf16x8 (&ra)[8], bf16x8 (&rb)[8], int t, int ks, int i) {
    const char* ba = smem + (t & 1) * W4_BUF + (wm * 128 + r16) * 128 + (((q + 4 * ks) ^ swz) * 16);
    const char* bb = smem + (t & 1) * W4_BUF + W4_HALF + (wn * 128 + r16) * 128 + (((q + 4 * ks) ^ swz) * 16);
    ra[i] = *(const bf16x8*)(ba + i * 16 * 128);
    rb[i] = *(const bf16x8*)(bb + i * 16 * 128);
  };
  f32x4 acc[8][8];
  auto mma_row = [&](const bf16x8 (&ra)[8], const bf16x8 (&rb)[8], int i) {
    #pragma unroll
    for (int j = 0; j < 8; ++j)
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(rb[j]), "v"(ra[i]));
  };

  // first K-tile of a tile: srcC = inline constant 0 instead of 256 accumulator writes
  auto mma_row_z = [&](const bf16x8 (&ra)[8], const bf16x8 (&rb)[8], int i) {
    #pragma unroll
    for (int j = 0; j < 8; ++j)
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc[i][j]) : "v"(rb[j]), "v"(ra[i]));
  };
  auto half0 = [&](int t, bool zero) {   // MFMAs on a0/b0 (ks 0 of K-tile t), reads of a1/b1 (ks 1)
    if (zero)
      g8_sfor_w4<0, 8>([&](auto ic) {
        mma_row_z(a0, b0, decltype(ic)::value);
        load_frag(a1, b1, t, 1, decltype(ic)::value);
      });
    else
      g8_sfor_w4<0, 8>([&](auto ic) {
        mma_row(a0, b0, decltype(ic)::value);
        load_frag(a1, b1, t, 1, decltype(ic)::value);
      });
  };
  int m0c = 0, n0c = 0;
  auto store_row = [&](int i) {   // exactly 8 buffer stores per row block; rows >= M are dropped
    const int m = m0c + wm * 128 + i * 16 + r16;
    const unsigned rowoff = (unsigned)(((long long)m * N + n0c + wn * 128 + 4 * q) * 2);
    #pragma unroll
    for (int j = 0; j < 8; ++j) {
      const f32x4 v = acc[i][j];
      const bf16x4 o = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_w4, o), c_rsrc, m < M ? rowoff + j * 32 : 0xFFFFFFF0u,
                                            0, 0);
    }
  };

  int tid = blockIdx.x;
  if (tid >= n_tiles) return;
  int m0, n0;
  tile_origin(tid, m0, n0);
  setup(m0, n0);
  issue_all(0);
  issue_all(1);
  for (;;) {
    // K-tiles 0 and 1 landed; after the first tile the previous tile's 64 stores per wave were issued
    // after them (vmcnt retires in order): vmcnt(63) leaves those stores draining
    if (tid == (int)blockIdx.x) __builtin_amdgcn_s_waitcnt(WAIT_VM16 & ~0x4000);   // vmcnt(0) first tile
    else __builtin_amdgcn_s_waitcnt(WAIT_VM63);
    w4_barrier();
    g8_sfor_w4<0, 8>([&](auto ic) { load_frag(a0, b0, 0, 0, decltype(ic)::value); });
    for (int t = 0; t < nk - 1; ++t) {
      half0(t, t == 0);
      __builtin_amdgcn_s_waitcnt(WAIT_ALL);
      w4_barrier();
      g8_sfor_w4<0, 8>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        issue(t + 2, ic);
        mma_row(a1, b1, i);
        load_frag(a0, b0, t + 1, 0, i);
      });
    }
    // last K-tile: no DMA into the buffers; the next tile's first two K-tiles go out before the
    // stores, and each row block's stores follow its last 8 MFMAs (overlapping the next row's)
    half0(nk - 1, nk == 1);
    __builtin_amdgcn_s_waitcnt(WAIT_ALL);   // also drains the redundant re-loads of tile nk-1
    w4_barrier();                           // every wave's reads of both buffers are done
    m0c = m0;
    n0c = n0;
    const int next = tid + gridDim.x;
    if (next < n_tiles) {
      tile_origin(next, m0, n0);
      setup(m0, n0);
      issue_all(0);
      issue_all(1);
    }
    // the reads of a row block's accumulators are pinned behind an asm that names them (a plain
    // register read is otherwise free to move up to the MFMA asm that produced them, ahead of the
    // hazard distance the compiler cannot see): row i-1 after row i's 8 MFMAs, row 7 after 24 nops
    auto fence_row = [&](int i) {
      asm volatile("" : "+a"(acc[i][0]), "+a"(acc[i][1]), "+a"(acc[i][2]), "+a"(acc[i][3]), "+a"(acc[i][4]),
                   "+a"(acc[i][5]), "+a"(acc[i][6]), "+a"(acc[i][7]));
    };
    g8_sfor_w4<0, 8>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      mma_row(a1, b1, i);
      if constexpr (i > 0) {   // 8 independent MFMAs since row i-1's last one
        fence_row(i - 1);
        store_row(i - 1);
      }
    });
    asm volatile("s_nop 7\n s_nop 7\n s_nop 7" : "+a"(acc[7][0]), "+a"(acc[7][1]), "+a"(acc[7][2]), "+a"(acc[7][3]),
                 "+a"(acc[7][4]), "+a"(acc[7][5]), "+a"(acc[7][6]), "+a"(acc[7][7]));
    store_row(7);
    if (next >= n_tiles) break;
    tid = next;
  }
  __builtin_amdgcn_s_waitcnt(WAIT_ALL);
}

__global__ void ref_kernel(const bf16* A, const bf16* B, float* C, int M, int N, int K) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
  if (n >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += (float)A[(long long)m * K + k] * (float)B[(long long)n * K + k];
  C[(long long)m * N + n] = s;
}

__global__ void fill_kernel(bf16* p, long long n, unsigned seed) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    p[i] = (bf16)((float)(h >> 8) * (2.0f / 16777216.0f) - 1.0f);
  }
}

typedef int (*sse_gemm_t)(int, const void*, const void*, const float*, const float*, float*, void*, int, int, int, int,
                          const void*, void*);

template <typename F>
static float time_ms(F&& f, int iters) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) f();
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) f();
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / iters;
}

static double rel_l2(const std::vector<bf16>& c, const std::vector<float>& r) {
  double num = 0, den = 0;
  for (size_t i = 0; i < r.size(); ++i) {
    const double d = (double)(float)c[i] - r[i];
    num += d * d; den += (double)r[i] * r[i];
  }
  return std::sqrt(num / den);
}

int main() {
  void* h = dlopen("stuttering-speech-representation_amd/libsse.so", RTLD_NOW);
  sse_gemm_t sse_gemm = h ? (sse_gemm_t)dlsym(h, "sse_gemm") : nullptr;
  if (!sse_gemm) printf("libsse.so not loaded (%s): 4-wave kernel only\n", dlerror());
  const int shapes[][4] = {{4096, 4096, 4096, 1}, {8192, 8192, 8192, 0}, {38144, 3072, 768, 1},
                           {38144, 768, 3072, 1}, {38144, 2304, 768, 0}};
  void* zero;
  CK(hipMalloc(&zero, 256));
  CK(hipMemset(zero, 0, 256));
  for (auto& s : shapes) {
    const int M = s[0], N = s[1], K = s[2], check = s[3];
    bf16 *a, *b, *c4, *c8;
    CK(hipMalloc(&a, (size_t)M * K * 2)); CK(hipMalloc(&b, (size_t)N * K * 2));
    CK(hipMalloc(&c4, (size_t)M * N * 2)); CK(hipMalloc(&c8, (size_t)M * N * 2));
    hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, a, (long long)M * K, 17u);
    hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, b, (long long)N * K, 91u);
    const int grid = ((M + 255) / 256) * (N / 256);
    const double tf = 2.0 * M * N * K / 1e12;
    float t8 = -1.f;
    std::vector<bf16> h8;
    if (sse_gemm) {
      auto run8 = [&] {
        const int rc = sse_gemm(1, a, b, nullptr, nullptr, nullptr, c8, M, N, K, 0, zero, nullptr);
        if (rc) { printf("sse_gemm rc %d\n", rc); exit(1); }
      };
      t8 = time_ms(run8, 20);
      CK(hipDeviceSynchronize());
      h8.resize((size_t)M * N);
      CK(hipMemcpy(h8.data(), c8, h8.size() * 2, hipMemcpyDeviceToHost));
    }
    printf("M=%d N=%d K=%d  8-phase: %.1f TF/s (%.1f us)\n", M, N, K, t8 > 0 ? tf / (t8 * 1e-3) : 0.0, t8 * 1e3);
    typedef void (*kfn)(const bf16*, const bf16*, bf16*, int, int, int);
    const kfn variants[6] = {gemm4w_kernel<0, false>, gemm4w_kernel<1, false>, gemm4w_kernel<0, true>,
                             gemm4w_kernel<1, true>, gemm4w_kernel<0, true, true>, gemm4w_kernel<1, true, true>};
    const char* names[6] = {"4w", "4w+ilv", "4w uniform", "4w uniform+ilv", "4w asm", "4w asm+ilv"};
    for (int v = 0; v < 6; ++v) {
      auto run4 = [&] { hipLaunchKernelGGL(variants[v], dim3(grid), dim3(256), 0, 0, a, b, c4, M, N, K); };
      const float t4 = time_ms(run4, 20);
      CK(hipDeviceSynchronize());
      std::vector<bf16> hc((size_t)M * N);
      CK(hipMemcpy(hc.data(), c4, hc.size() * 2, hipMemcpyDeviceToHost));
      double eq = -1;
      if (!h8.empty()) {
        size_t same = 0;
        for (size_t i = 0; i < hc.size(); ++i)
          same += __builtin_bit_cast(unsigned short, hc[i]) == __builtin_bit_cast(unsigned short, h8[i]);
        eq = (double)same / hc.size();
      }
      printf("  %-15s %.1f TF/s (%.1f us), bit-equal to 8-phase: %.4f\n", names[v], tf / (t4 * 1e-3), t4 * 1e3, eq);
      if (check && v == 0) {
        float* cr;
        CK(hipMalloc(&cr, (size_t)M * N * 4));
        hipLaunchKernelGGL(ref_kernel, dim3((N + 255) / 256, M), dim3(256), 0, 0, a, b, cr, M, N, K);
        std::vector<float> hr((size_t)M * N);
        CK(hipMemcpy(hr.data(), cr, hr.size() * 4, hipMemcpyDeviceToHost));
        printf("  %-15s rel-L2 vs fp32 reference %.3e\n", names[v], rel_l2(hc, hr));
        CK(hipFree(cr));
      }
      fflush(stdout);
    }
    {
      int cus = 256;
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
      const int gp = grid < cus ? grid : cus;
      for (int gmv = 0; gmv < 2; ++gmv) {
      auto runp = [&] {
        if (gmv) hipLaunchKernelGGL(gemm4p_kernel<1>, dim3(gp), dim3(256), 0, 0, a, b, c4, M, N, K, grid);
        else hipLaunchKernelGGL(gemm4p_kernel<8>, dim3(gp), dim3(256), 0, 0, a, b, c4, M, N, K, grid);
      };
      const float tp = time_ms(runp, 20);
      CK(hipDeviceSynchronize());
      std::vector<bf16> hc((size_t)M * N);
      CK(hipMemcpy(hc.data(), c4, hc.size() * 2, hipMemcpyDeviceToHost));
      double eq = -1;
      if (!h8.empty()) {
        size_t same = 0;
        for (size_t i = 0; i < hc.size(); ++i)
          same += __builtin_bit_cast(unsigned short, hc[i]) == __builtin_bit_cast(unsigned short, h8[i]);
        eq = (double)same / hc.size();
      }
      printf("  %-15s %.1f TF/s (%.1f us), bit-equal to 8-phase: %.4f\n", gmv ? "4w persistent rm" : "4w persistent",
             tf / (tp * 1e-3), tp * 1e3, eq);
      fflush(stdout);
      }
    }
    CK(hipFree(a)); CK(hipFree(b)); CK(hipFree(c4)); CK(hipFree(c8));
  }
  return 0;
}
