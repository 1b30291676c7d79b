// 256x256 bf16 MFMA GEMM with an 8-phase ping-pong schedule (gfx950).
//
// Same contract as gemm_body<bf16, 256, 256, ...> in kernels_gemm.hip (SEG-mode A rows, B as
// [N][K], fused bias / GELU / fp32 residual epilogue), restricted to K % 64 == 0, N % 256 == 0.
//
// Why: in the 2-stage loop every K-step ends in vmcnt(0) + barrier, so the block waits for the
// tile it just requested and all 8 waves issue their LDS reads at the same moment; PMC on the
// WavLM shapes showed 39-45 % of wave cycles parked (SQ_WAIT_ANY) with the MFMA pipe busy 24-41 %.
//
// Schedule (derivation in DESIGN.md "GEMM 8-phase schedule"):
//  * 8 waves = 2 groups (wm) x 4 (wn).  Wave (wm, wn) owns rows {mi*128 + wm*64 + [0,64)} and
//    columns {ni*128 + wn*32 + [0,32)} for mi, ni in {0,1}, so each 128-row / 128-column HALF of
//    the A / B tile is read by all waves in exactly one phase.
//  * K-tile t (BK = 64) runs 4 phases (mi, ni) = (0,0) (0,1) (1,1) (1,0).  A phase is an
//    L-section (ds_read fragments, issue one half-tile of LDS-DMA, counted vmcnt), a barrier,
//    an M-section (16 MFMA 16x16x32 at raised priority) and a barrier.  Group 1 starts one
//    barrier late, so on every SIMD one wave is in its M-section while the other loads.
//  * B fragments of ni = 0 stay in registers from phase 0 to phase 3, so per K-tile each half
//    is read once: A0 and B0 in phase 0, B1 in phase 1, A1 in phase 2.
//  * Phase k = 4t+p issues: p0 -> B1(t+1), p1 -> A1(t+1), p2 -> A0(t+2), p3 -> B0(t+2) into
//    buffer (tile & 1).  Every half is issued >= 5 phases before its first read and after the
//    barrier that follows the last lgkmcnt of its previous occupant; a uniform vmcnt(8) at the
//    end of each L-section (fewer in the tail) retires what the next phase reads.
//  * Round 6 (the default for all three 8-wave kernels; option gemm_4phase = 1 keeps four phases): the same K-tile in TWO phases of 32 MFMAs -- Q0 reads A0, B0, B1 (A0 B0, A0 B1), Q1 reads A1
//    (A1 B1, A1 B0) -- half the barriers, bit-identical; issue schedule Q0(t) -> A1(t+1), Q1(t) -> A0, B0, B1(t+2)
//    (g8_ops2 / g8_count2 / g8_issue2; DESIGN.md "Two phases per K-tile").
//
// MX = true: MX-fp8 operands (OCP e4m3 + E8M0 per 32 K-elements, v_mfma_scale_f32_16x16x128_f8f6f4,
// 2x the bf16 MFMA rate).  A K-tile is still 128 B per row (128 elements), the LDS image and the
// fragment reads are byte-identical to the bf16 kernel's: the MX instruction takes lane group q's
// K elements from chunks q and q+4 of the row (k in [16q, 16q+16) u [64+16q, 64+16q+16), probed on
// gfx950, tools/probe_mx2.hip) and block b's scale of row r from lane r + 16b.  Per K-tile the
// 256 A-row and 256 B-column scales (2 KiB, layouts mx_a_scale_off / mx_b_scale_off) are one extra
// dword LDS-DMA per wave, issued with A0 (phase p = 2) into a 4-deep ring (tile & 3), so the same
// WAR / RAW argument holds; that phase counts 3 vector-memory ops instead of 2.
#include <string.h>

#include <type_traits>

#include "common.h"


namespace {

constexpr int G8_HALF = 128 * 128;            // one half-tile: 128 rows x 128 B (64 bf16 of K)
constexpr int G8_BUF = 4 * G8_HALF;           // A rows 0-127 | A rows 128-255 | B cols 0-127 | B cols 128-255
constexpr int G8_OPS = 2 * G8_BUF;            // two K-tiles: 128 KiB
constexpr int G8_CLD = 256 + 4;               // epilogue fp32 row stride (floats)
constexpr int G8_EPI = 128 * G8_CLD * 4;      // one 128-row half of the C tile
constexpr int G8_SC = 2048;                   // MX: one K-tile's scales (A 1 KiB | B 1 KiB)
constexpr int G8_OPS_MX = G8_OPS + 4 * G8_SC; // MX: operands + 4-deep scale ring
constexpr int G8_SMEM = G8_OPS > G8_EPI ? G8_OPS : G8_EPI;
constexpr int G8_SMEM_MX = G8_OPS_MX > G8_EPI ? G8_OPS_MX : G8_EPI;

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef short v2i16g8 __attribute__((ext_vector_type(2)));

// phase k = 4t + p (k >= -8) -> the (tile, half) whose LDS-DMA it issues
SSE_DEV void g8_target(int k, int& tile, int& half) {
  const int t = (k + 8) / 4 - 2, p = (k + 8) & 3;
  tile = p < 2 ? t + 1 : t + 2;
  half = p == 0 ? 3 : (p == 1 ? 1 : (p == 2 ? 0 : 2));
}

// vector-memory ops (per wave) issued at phase k: 2 LDS-DMA per half-tile, +1 scale DMA (MX) at
// the phase that issues A0 (p = 2)
template <bool MX>
SSE_DEV int g8_ops(int k, int nk) {
  if (k < -6) return 0;
  int tile, half;
  g8_target(k, tile, half);
  if (tile >= nk) return 0;
  return MX && half == 0 ? 3 : 2;
}

template <bool MX>
SSE_DEV int g8_count(int k, int nk) {   // ops issued at phases k-3 .. k (the wait at the end of L(k))
  return g8_ops<MX>(k, nk) + g8_ops<MX>(k - 1, nk) + g8_ops<MX>(k - 2, nk) + g8_ops<MX>(k - 3, nk);
}

// s_waitcnt vmcnt(n), n in [0, 63] (6-bit field; larger n waits for everything).  The bf16 kernels
// only ever wait for even counts (2 ops per phase, even store counts): a 32-way switch.
template <bool MX>
SSE_DEV void g8_vmcnt_dyn(int n) {
#define G8_VM(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
#define G8_VE(N) case N / 2: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
  if constexpr (MX) {
    switch (n) {
      G8_VM(1) G8_VM(2) G8_VM(3) G8_VM(4) G8_VM(5) G8_VM(6) G8_VM(7) G8_VM(8) G8_VM(9) G8_VM(10) G8_VM(11)
      G8_VM(12) G8_VM(13) G8_VM(14) G8_VM(15) G8_VM(16) G8_VM(17) G8_VM(18) G8_VM(19) G8_VM(20) G8_VM(21)
      G8_VM(22) G8_VM(23) G8_VM(24) G8_VM(25) G8_VM(26) G8_VM(27) G8_VM(28) G8_VM(29) G8_VM(30) G8_VM(31)
      G8_VM(32) G8_VM(33) G8_VM(34) G8_VM(35) G8_VM(36) G8_VM(37) G8_VM(38) G8_VM(39) G8_VM(40) G8_VM(41)
      G8_VM(42) G8_VM(43) G8_VM(44) G8_VM(45) G8_VM(46) G8_VM(47) G8_VM(48) G8_VM(49) G8_VM(50) G8_VM(51)
      G8_VM(52) G8_VM(53) G8_VM(54) G8_VM(55) G8_VM(56) G8_VM(57) G8_VM(58) G8_VM(59) G8_VM(60) G8_VM(61)
      G8_VM(62) G8_VM(63)
      default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
  } else {
    switch (n >> 1) {
      G8_VE(2) G8_VE(4) G8_VE(6) G8_VE(8) G8_VE(10) G8_VE(12) G8_VE(14) G8_VE(16) G8_VE(18) G8_VE(20) G8_VE(22)
      G8_VE(24) G8_VE(26) G8_VE(28) G8_VE(30) G8_VE(32) G8_VE(34) G8_VE(36) G8_VE(38) G8_VE(40) G8_VE(42)
      G8_VE(44) G8_VE(46) G8_VE(48) G8_VE(50) G8_VE(52) G8_VE(54) G8_VE(56) G8_VE(58) G8_VE(60) G8_VE(62)
      default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
  }
#undef G8_VM
#undef G8_VE
}

// retire every op issued at phases <= k-4
template <bool MX>
SSE_DEV void g8_wait(int k, int nk) { g8_vmcnt_dyn<MX>(g8_count<MX>(k, nk)); }

// Two-phase schedule (round 6 default; gemm8p_kernel's template comment): 2-phase index j = 2t + h, Q0(t) issues
// A1(t+1), Q1(t) issues A0, B0, B1(t+2); the prologue is j = -3 .. -1.  ih(tile, half) issues one half-tile (2 ops).
// (MX: Q1's A0 issue carries the K-tile's scale DMA, 7 ops)
template <bool MX = false>
SSE_DEV int g8_ops2(int j, int nk) {
  if (j < -3) return 0;
  const int t = j >> 1;
  return (j & 1) == 0 ? (t + 1 < nk ? 2 : 0) : (t + 2 < nk ? (MX ? 7 : 6) : 0);
}
// ops the wait at the end of L(j) leaves in flight: what was issued at j and j - 1
template <bool MX = false>
SSE_DEV int g8_count2(int j, int nk) { return g8_ops2<MX>(j, nk) + g8_ops2<MX>(j - 1, nk); }
template <typename IH>
SSE_DEV void g8_issue2(int j, int nk, IH&& ih) {
  if (j < -3) return;
  const int t = j >> 1;
  if ((j & 1) == 0) {
    if (t + 1 < nk) ih(t + 1, 1);
  } else if (t + 2 < nk) {
    ih(t + 2, 0);
    ih(t + 2, 2);
    ih(t + 2, 3);
  }
}

// epilogue memory ops; NT = non-temporal (streaming: C tiles and residual rows are touched once
// and should not evict the A / B operand lines from L2)
template <bool NT, typename V> SSE_DEV void g8_st(V* p, V v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
template <bool NT, typename V> SSE_DEV V g8_ld(const V* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

SSE_DEV void g8_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int OA, int OB>
SSE_DEV f32x4 g8_mx(i32x8 a, i32x8 b, f32x4 c, int sa, int sb) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, OA, sa, OB, sb);
}
// 16x16x32 MFMA on bf16 or (split-fp16 path) fp16 operands; the 16-B fragments are the same bytes
template <bool F16>
SSE_DEV f32x4 g8_mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
template <int I, int N, typename F>
SSE_DEV void g8_sfor(F&& f) {   // f(integral_constant<int, I>) for I .. N-1, compile-time indices
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    g8_sfor<I + 1, N>(f);
  }
}

// two 16-B fragments (chunks q and q+4 of the K-tile row) as one 32-byte MX operand
SSE_DEV i32x8 g8_cat(bf16x8 lo, bf16x8 hi) {
  const i32x4 a = __builtin_bit_cast(i32x4, lo), b = __builtin_bit_cast(i32x4, hi);
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

// DBG = 1 (timing experiments only, not launched by the library): no epilogue, a checksum keeps the MFMAs live.
template <bool RES, bool Q8 = false, bool RB = false, int FX = 0, bool RSC = false, bool VAM = false, bool RBL = false>
SSE_DEV void g8_epilogue_direct(const GemmArgs& g, f32x4 (&acc)[2][2][4][2], int m0, int n0, int wm, int wn,
                                int q, int r16, const char* rl0 = nullptr, const char* rl1 = nullptr);

// TR = true: the MFMAs compute C^T blocks (the B fragment is the MFMA's A operand), so every
// lane ends up holding 4 consecutive output columns of one row and the epilogue stores straight
// from registers (see g8_epilogue_direct).  TR = false: C blocks, LDS-staged epilogue.
// MXE (MX, TR): the epilogue fixed at compile time -- 0: runtime selection (tests, any combination); 1: fc1
// (bias, ACT_GELU_FAST, MX-fp8 out); 2: fc2 (bias, the bf16 residual stream in place; a kernel holding both
// it and the fp8-out epilogue spilled 178 VGPRs); 3: qkv (bias, bf16 out); 4: the fp8 attention's Q / K (bias,
// MX-fp8 out, row-major scales); 5: its V (bias, bf16 out, per-clip column amax).  Runtime selects in the
// persistent bf16 kernel's epilogue measured +5-6 %.
// PH2 (MX only; round 6 default, option gemm_4phase = 1 keeps four phases): two 32-MFMA phases per K-tile, the
// schedule of gemm8p_kernel's template comment, the scale DMA issued with A0 in Q1 (7 ops; steady vmcnt(9) as before)
template <int DBG, bool TR, bool NT, bool MX = false, int MXE = 0, bool PH2 = false>
__global__ __launch_bounds__(512) void gemm8_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[MX ? G8_SMEM_MX : G8_SMEM];   // the ONLY shared object
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int q = lane >> 4, r16 = lane & 15;
  const int M = g.M, N = g.N, K = g.K;
  const int n_tiles_n = N / 256;
  int bid = blockIdx.x;
  {   // XCD-aware bijective remap (as gemm_body)
    const int nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, x = bid % 8;
    bid = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + bid / 8;
  }
  int mt = bid / n_tiles_n, nt_ = bid % n_tiles_n;
  if constexpr (MX) {
    // grouped raster (MX): 8 row tiles per group, row fastest, so an XCD's ~32 concurrent tiles span
    // 8 A row-tiles x 4 B column-tiles (3.9 MB at K = 1280, L2-resident) instead of 2 x all columns
    // (the whole weight matrix re-streamed into L2 every 2 row-tiles)
    constexpr int GM = 8;
    const int MT = (M + 255) / 256;
    const int first = (bid / (GM * n_tiles_n)) * GM, gm = MT - first < GM ? MT - first : GM;
    const int r = bid - first * n_tiles_n;
    mt = first + r % gm;
    nt_ = r / gm;
  }
  const int m0 = mt * 256, n0 = nt_ * 256;
  constexpr int ES = MX ? 1 : 2;   // operand element bytes; a K-tile is 128 B per row either way
  const int nk = K / (128 / ES);

  // ---- LDS-DMA sources: buffer descriptors based at the block's first A row / B row; each
  // lane's byte offset is fixed for the whole K loop, the scalar soffset advances by 128 B.
  constexpr int NREC = 0x7FFFFFF0;
  __amdgpu_buffer_rsrc_t a_rsrc, b_rsrc, s_rsrc;
  unsigned a_voff[2][2], b_voff[2][2], s_voff = 0;
  {
    const int mf = m0 < M ? m0 : M - 1;
    const int seg0 = mf / g.rows_per_seg, rr0 = mf - seg0 * g.rows_per_seg;
    const long long a_base = ((long long)seg0 * g.seg_stride + (long long)rr0 * g.lda) * ES;   // bytes
    a_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)g.A + a_base), (short)0, NREC, 0x00020000);
    b_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)g.B + (long long)n0 * K * ES), (short)0, NREC,
                                               0x00020000);
    if constexpr (MX) {   // this tile's scale blocks; waves 0-3 stage A's 1 KiB, waves 4-7 B's
      const unsigned char* sb = wave < 4 ? g.a_scale + (long long)(m0 >> 8) * nk * 1024
                                         : g.b_scale + (long long)(n0 >> 8) * nk * 1024;
      s_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)sb, (short)0, NREC, 0x00020000);
      s_voff = (unsigned)((wave & 3) * 256 + lane * 4);
    }
    #pragma unroll
    for (int h = 0; h < 2; ++h)
      #pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int row = h * 128 + (wave + 8 * s) * 8 + (lane >> 3);
        const int ch = (lane & 7) ^ ((row >> 1) & 7);
        int m = m0 + row;
        m = m < M ? m : M - 1;
        const int seg = m / g.rows_per_seg, rr = m - seg * g.rows_per_seg;
        const long long el = ((long long)seg * g.seg_stride + (long long)rr * g.lda) * ES + ch * 16;
        a_voff[h][s] = (unsigned)(el - a_base);
        b_voff[h][s] = (unsigned)((long long)row * K * ES + ch * 16);
      }
  }
  auto issue_half = [&](int tile, int half) {
    char* dst = smem + (tile & 1) * G8_BUF + half * G8_HALF;
    const unsigned soff = (unsigned)tile * 128u;
    if constexpr (MX) {
      if (half == 0)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(s_rsrc, LPTR(smem + G8_OPS + (tile & 3) * G8_SC + wave * 256), 4,
                                                 s_voff, (unsigned)tile * 1024u, 0, 0);
    }
    if (half < 2) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, LPTR(dst + wave * 1024), 16, a_voff[half][0], soff, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, LPTR(dst + (wave + 8) * 1024), 16, a_voff[half][1], soff, 0, 0);
    } else {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, LPTR(dst + wave * 1024), 16, b_voff[half - 2][0], soff, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, LPTR(dst + (wave + 8) * 1024), 16, b_voff[half - 2][1], soff, 0,
                                               0);
    }
  };
  auto issue = [&](int k) {
    if (k < -6) return;
    int tile, half;
    g8_target(k, tile, half);
    if (tile >= nk) return;
    issue_half(tile, half);
  };

  // fc2 (MXE 2): the bf16 residual rows of the tile go to LDS by DMA -- half 0 during the last K-tile into the
  // buffer K-tile nk - 2 used, half 1 after the main loop into the last K-tile's (gemm8r_kernel<RB>'s scheme):
  // 64 pieces of 1 KiB per half, rows of 512 B, 16-B chunk c at c ^ (row & 15); rows >= M read as zeros
  constexpr bool RBP = MX && TR && MXE == 2 && DBG == 0;
  auto res_dma = [&](int mi, int buf) {
    if constexpr (RBP) {
      const long long r0 = (long long)m0 + mi * 128, rows = (long long)M - r0;
      const long long nrec = rows > 0 ? (rows * g.ldc - n0) * 2 : 0;
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(g.resid_t + (rows > 0 ? r0 * g.ldc + n0 : 0)), (short)0, (int)min(nrec, (long long)0x7FFFFFF0),
          0x00020000);
      #pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int u = wave * 8 + e, row = 2 * u + (lane >> 5), c = (lane & 31) ^ (row & 15);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rr, LPTR(smem + buf * G8_BUF + u * 1024), 16,
                                                 (unsigned)((row * g.ldc + c * 8) * 2), 0u, 0, 0);
      }
    }
  };

  // the steady loop's issue (t + 2 < nk): phase p's (tile, half) known at compile time and no range checks.
  // Branch-free on purpose: with issue()'s checks the K-tile body is several basic blocks, sched_barrier
  // does not hold across them, and the MX build had its phase 0-2 MFMAs sunk to the end of the K-tile
  // (the ping-pong gone: 8 0 0 0 MFMAs per phase in the ISA)
  auto issue_steady = [&](int t, auto p_c) {
    constexpr int P = decltype(p_c)::value;
    constexpr int half = P == 0 ? 3 : (P == 1 ? 1 : (P == 2 ? 0 : 2));
    const int tile = P < 2 ? t + 1 : t + 2;
    char* dst = smem + (tile & 1) * G8_BUF + half * G8_HALF;
    const unsigned soff = (unsigned)tile * 128u;
    if constexpr (MX && half == 0)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(s_rsrc, LPTR(smem + G8_OPS + (tile & 3) * G8_SC + wave * 256), 4, s_voff,
                                               (unsigned)tile * 1024u, 0, 0);
    if constexpr (half < 2) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, LPTR(dst + wave * 1024), 16, a_voff[half][0], soff, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, LPTR(dst + (wave + 8) * 1024), 16, a_voff[half][1], soff, 0, 0);
    } else {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, LPTR(dst + wave * 1024), 16, b_voff[half - 2][0], soff, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, LPTR(dst + (wave + 8) * 1024), 16, b_voff[half - 2][1], soff, 0,
                                               0);
    }
  };

  // PH2 steady issue (t + 2 < nk), branch-free as issue_steady: Q0 -> A1(t+1); Q1 -> scales, A0, B0, B1 (t+2)
  auto issue_steady2 = [&](int t, auto h_c) {
    constexpr int Hh = decltype(h_c)::value;
    if constexpr (Hh == 0) {
      char* dst = smem + ((t + 1) & 1) * G8_BUF + G8_HALF;
      const unsigned soff = (unsigned)(t + 1) * 128u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, LPTR(dst + wave * 1024), 16, a_voff[1][0], soff, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, LPTR(dst + (wave + 8) * 1024), 16, a_voff[1][1], soff, 0, 0);
    } else {
      const int tile = t + 2;
      char* dst = smem + (tile & 1) * G8_BUF;
      const unsigned soff = (unsigned)tile * 128u;
      if constexpr (MX)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(s_rsrc, LPTR(smem + G8_OPS + (tile & 3) * G8_SC + wave * 256), 4, s_voff,
                                                 (unsigned)tile * 1024u, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, LPTR(dst + wave * 1024), 16, a_voff[0][0], soff, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, LPTR(dst + (wave + 8) * 1024), 16, a_voff[0][1], soff, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, LPTR(dst + 2 * G8_HALF + wave * 1024), 16, b_voff[0][0], soff, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, LPTR(dst + 2 * G8_HALF + (wave + 8) * 1024), 16, b_voff[0][1], soff,
                                               0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, LPTR(dst + 3 * G8_HALF + wave * 1024), 16, b_voff[1][0], soff, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, LPTR(dst + 3 * G8_HALF + (wave + 8) * 1024), 16, b_voff[1][1], soff,
                                               0, 0);
    }
  };

  f32x4 acc[2][2][4][2];
  #pragma unroll
  for (int a = 0; a < 2; ++a)
    #pragma unroll
    for (int b = 0; b < 2; ++b)
      #pragma unroll
      for (int i = 0; i < 4; ++i)
        #pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[4][2], b0f[2][2], b1f[2][2];
  int sa = 0, sb = 0;   // MX: this lane's A scales (rows i = 0..3 of the current mi), B scales (ni, j)
  auto read_sa = [&](int t, int mi) {
    if constexpr (MX) sa = *(const int*)(smem + G8_OPS + (t & 3) * G8_SC + (((mi * 2 + wm) * 4 + q) * 16 + r16) * 4);
  };
  auto read_sb = [&](int t) {
    if constexpr (MX) sb = *(const int*)(smem + G8_OPS + (t & 3) * G8_SC + 1024 + ((wn * 4 + q) * 16 + r16) * 4);
  };

  // MX: the same two 16-B reads per fragment, landing in one 8-dword operand tuple
  i32x8 afx[4], b0x[2], b1x[2];
  auto rd32 = [&](const char* hb, int row) {
    const i32x4 lo = *(const i32x4*)(hb + row * 128 + ((q ^ ((row >> 1) & 7)) * 16));
    const i32x4 hi = *(const i32x4*)(hb + row * 128 + (((q + 4) ^ ((row >> 1) & 7)) * 16));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto read_a = [&](const char* hb) {
    #pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + i * 16 + r16;
      if constexpr (MX) {
        afx[i] = rd32(hb, row);
      } else {
        #pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          af[i][ks] = *(const bf16x8*)(hb + row * 128 + (((q + 4 * ks) ^ ((row >> 1) & 7)) * 16));
      }
    }
  };
  auto read_b = [&](const char* hb, bf16x8 (&bf)[2][2], i32x8 (&bx)[2]) {
    #pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = wn * 32 + j * 16 + r16;
      if constexpr (MX) {
        bx[j] = rd32(hb, row);
      } else {
        #pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          bf[j][ks] = *(const bf16x8*)(hb + row * 128 + (((q + 4 * ks) ^ ((row >> 1) & 7)) * 16));
      }
    }
  };
  auto mma = [&](f32x4 (&c)[4][2], const bf16x8 (&bf)[2][2], const i32x8 (&bx)[2], auto ni_c) {
    constexpr int NI = decltype(ni_c)::value;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // (compiler-placed per-operand waits instead: neutral, round 5)
    __builtin_amdgcn_sched_barrier(0);
    // (no raised wave priority around the MFMAs, here or in gemm8p / gemm8r: removing it took fp8 Whisper
    // 184.3 -> 183.1 and WavLM-base 11.71 -> 11.65 ms/step, r5_ab_mx_setprio.txt / r5_ab_bf16_setprio.txt)
    if constexpr (MX && DBG == 4) {   // probe: no MFMA (the fragment and scale reads kept live)
      #pragma unroll
      for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(afx[i]));
      #pragma unroll
      for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(bx[j]));
      asm volatile("" ::"v"(sa), "v"(sb));
    } else if constexpr (MX) {
      g8_sfor<0, 4>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        g8_sfor<0, 2>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          if constexpr (TR) c[i][j] = g8_mx<NI * 2 + j, i>(bx[j], afx[i], c[i][j], sb, sa);
          else c[i][j] = g8_mx<i, NI * 2 + j>(afx[i], bx[j], c[i][j], sa, sb);
        });
      });
    } else {
      #pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        #pragma unroll
        for (int i = 0; i < 4; ++i)
          #pragma unroll
          for (int j = 0; j < 2; ++j)
            c[i][j] = TR ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][ks], af[i][ks], c[i][j], 0, 0, 0)
                         : __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][ks], bf[j][ks], c[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  };

  // ---- prologue: phases -6..-1 stage A0(0) B0(0) B1(0) A1(0) A0(1) B0(1) (PH2: j = -3..-1, tile 0 and A0 B0 B1 (1))
  if constexpr (PH2) {
    for (int j = -3; j < 0; ++j) g8_issue2(j, nk, issue_half);
    g8_vmcnt_dyn<MX>(g8_count2<MX>(-1, nk));
  } else {
    for (int k = -6; k < 0; ++k) issue(k);
    g8_wait<MX>(-1, nk);
  }
  g8_barrier();
  if (wm == 1) g8_barrier();   // group 1 runs one barrier behind

  // PH2: the K-tile in two phases of 32 MFMAs (same accumulation order per accumulator: bit-identical)
  auto run_tile2 = [&](int t, auto mode_c) {
    constexpr int MODE = decltype(mode_c)::value;
    const char* buf = smem + (t & 1) * G8_BUF;
    const int j = 2 * t;
    const int xr = (RBP && MODE == 0 && t == nk - 1) ? 8 : 0;
    if (xr) res_dma(0, nk & 1);
    auto issue_wait = [&](auto h_c) {
      constexpr int Hh = decltype(h_c)::value;
      if constexpr (MODE == 1) {
        if constexpr (DBG != 5) issue_steady2(t, h_c);
        if constexpr (MX) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else {
        g8_issue2(j + Hh, nk, issue_half);
        g8_vmcnt_dyn<MX>(g8_count2<MX>(j + Hh, nk) + xr);
      }
    };
    const std::integral_constant<int, 0> ni0;
    const std::integral_constant<int, 1> ni1;
    // Q0: (mi 0) reads A rows 0-127 and all B columns; A0 B0 then A0 B1
    read_a(buf);
    read_b(buf + 2 * G8_HALF, b0f, b0x);
    read_b(buf + 3 * G8_HALF, b1f, b1x);
    read_sa(t, 0);
    read_sb(t);
    issue_wait(std::integral_constant<int, 0>{});
    g8_barrier();
    mma(acc[0][0], b0f, b0x, ni0);
    mma(acc[0][1], b1f, b1x, ni1);
    g8_barrier();
    // Q1: (mi 1) reads A rows 128-255; A1 B1 then A1 B0
    read_a(buf + G8_HALF);
    read_sa(t, 1);
    issue_wait(std::integral_constant<int, 1>{});
    g8_barrier();
    mma(acc[1][1], b1f, b1x, ni1);
    mma(acc[1][0], b0f, b0x, ni0);
    g8_barrier();
  };

  // steady K-tiles (t + 2 < nk): every phase issues a half and waits vmcnt(8) with no
  // scalar bookkeeping; the last two K-tiles take the counted tail path.
  // MODE 1: steady K-tile (t + 2 < nk), branch-free (issue_steady, a uniform counted wait); 0: the last two
  // K-tiles (range-checked issues and computed waits; there the compiler still sinks the MX MFMAs of phases
  // 1-3 to the K-tile's end -- a compile-time tail kept them in place but spilled the 256-VGPR MX kernel)
  auto run_tile = [&](int t, auto mode_c) {
    constexpr int MODE = decltype(mode_c)::value;
    const char* buf = smem + (t & 1) * G8_BUF;
    const int k = 4 * t;
    // RBP, last K-tile: half 0's residual rows go out before phase 0 (the tail waits leave those 8 in flight)
    const int xr = (RBP && MODE == 0 && t == nk - 1) ? 8 : 0;
    if (xr) res_dma(0, nk & 1);
    auto issue_wait = [&](auto p_c) {
      constexpr int P = decltype(p_c)::value;
      if constexpr (MODE == 1) {
        if constexpr (DBG != 5) issue_steady(t, p_c);   // probe 5: no steady-loop DMA
        if constexpr (MX) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else {
        issue(k + P);
        if constexpr (RBP) g8_vmcnt_dyn<MX>(g8_count<MX>(k + P, nk) + xr);
        else g8_wait<MX>(k + P, nk);
      }
    };
    const std::integral_constant<int, 0> ni0;
    const std::integral_constant<int, 1> ni1;
    // phase 0: (mi 0, ni 0) reads A rows 0-127 and B cols 0-127
    read_a(buf);
    read_b(buf + 2 * G8_HALF, b0f, b0x);
    read_sa(t, 0);
    read_sb(t);
    issue_wait(std::integral_constant<int, 0>{});
    g8_barrier();
    mma(acc[0][0], b0f, b0x, ni0);
    g8_barrier();
    // phase 1: (mi 0, ni 1) reads B cols 128-255
    read_b(buf + 3 * G8_HALF, b1f, b1x);
    issue_wait(std::integral_constant<int, 1>{});
    g8_barrier();
    mma(acc[0][1], b1f, b1x, ni1);
    g8_barrier();
    // phase 2: (mi 1, ni 1) reads A rows 128-255
    read_a(buf + G8_HALF);
    read_sa(t, 1);
    issue_wait(std::integral_constant<int, 2>{});
    g8_barrier();
    mma(acc[1][1], b1f, b1x, ni1);
    g8_barrier();
    // phase 3: (mi 1, ni 0) no reads
    issue_wait(std::integral_constant<int, 3>{});
    g8_barrier();
    mma(acc[1][0], b0f, b0x, ni0);
    g8_barrier();
  };
  int t = 0;
  if constexpr (PH2) {
    for (; t + 2 < nk; ++t) run_tile2(t, std::integral_constant<int, 1>{});
    for (; t < nk; ++t) run_tile2(t, std::integral_constant<int, 0>{});
  } else {
    for (; t + 2 < nk; ++t) run_tile(t, std::integral_constant<int, 1>{});
    for (; t < nk; ++t) run_tile(t, std::integral_constant<int, 0>{});
  }
  if (wm == 0) g8_barrier();   // balance group 1's extra barrier: every wave's LDS reads are done
  if constexpr (RBP) {
    res_dma(1, (nk - 1) & 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // half 0 landed; half 1's 8 pieces in flight
    __syncthreads();
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if constexpr (DBG == 1 || DBG == 4 || DBG == 5) {   // (probes: no epilogue)
    float cs = 0.f;
    #pragma unroll
    for (int a = 0; a < 2; ++a)
      #pragma unroll
      for (int b = 0; b < 2; ++b)
        #pragma unroll
        for (int i = 0; i < 4; ++i)
          #pragma unroll
          for (int j = 0; j < 2; ++j) cs += acc[a][b][i][j][0] + acc[a][b][i][j][1] + acc[a][b][i][j][2] + acc[a][b][i][j][3];
    if (cs == 1234.5678f && g.Cf) g.Cf[0] = cs;
    return;
  }

  if constexpr (TR) {
    if constexpr (MX) {   // fp8 (Q8) or bf16 / fp32 out; the bf16 residual stream in place (fc2, RB)
      if constexpr (MXE == 1) g8_epilogue_direct<false, true, false, 1>(g, acc, m0, n0, wm, wn, q, r16);
      else if constexpr (MXE == 2)
        g8_epilogue_direct<true, false, true, 2, false, false, true>(g, acc, m0, n0, wm, wn, q, r16,
                                                                      smem + (nk & 1) * G8_BUF, smem + ((nk - 1) & 1) * G8_BUF);
      else if constexpr (MXE == 3) g8_epilogue_direct<false, false, false, 2>(g, acc, m0, n0, wm, wn, q, r16);
      else if constexpr (MXE == 4) g8_epilogue_direct<false, true, false, 2, true>(g, acc, m0, n0, wm, wn, q, r16);
      else if constexpr (MXE == 5) g8_epilogue_direct<false, false, false, 2, false, true>(g, acc, m0, n0, wm, wn, q, r16);
      else if constexpr (MXE == 6) {   // fused Q|K (MX-fp8, row-major scales) | V (bf16 + vamax): uniform per tile
        if (n0 < g.n_split) {
          GemmArgs g1 = g;
          g1.N = g.n_split;
          g1.ldc = g.n_split;
          g8_epilogue_direct<false, true, false, 2, true>(g1, acc, m0, n0, wm, wn, q, r16);
        } else {   // the V frame: column n - n_split of ct2 / vamax, bias from column n_split on
          GemmArgs g2 = g;
          g2.Ct = g.ct2;
          g2.ldc = g.ldc2;
          g2.N = g.N - g.n_split;
          g2.bias = g.bias + g.n_split;
          g8_epilogue_direct<false, false, false, 2, false, true>(g2, acc, m0, n0 - g.n_split, wm, wn, q, r16);
        }
      }
      else if (g.c_scale) g8_epilogue_direct<false, true>(g, acc, m0, n0, wm, wn, q, r16);
      else g8_epilogue_direct<false>(g, acc, m0, n0, wm, wn, q, r16);
    } else {
      if (g.resid) g8_epilogue_direct<true>(g, acc, m0, n0, wm, wn, q, r16);
      else g8_epilogue_direct<false>(g, acc, m0, n0, wm, wn, q, r16);
    }
    return;
  }

  // ---- epilogue: per 128-row half, stage fp32 through LDS, then coalesced 16-B passes -----
  float* Cs = (float*)smem;
  constexpr int CH = 128 * 256 / 4;
  constexpr int UNR = 4;
  // residual: fp32 (resid) or the bf16 residual stream (resid_t)
  const bool has_bias = g.bias != nullptr, has_res = g.resid != nullptr || g.resid_t != nullptr;
  const bool gelu = g.act == ACT_GELU, gelu_fast = g.act == ACT_GELU_FAST;
  // compile-time mi / it (g8_sfor): acc[mi] and the MX scale words must stay in registers
  g8_sfor<0, 2>([&](auto mic) {
    constexpr int mi = decltype(mic)::value;
    __syncthreads();
    #pragma unroll
    for (int ni = 0; ni < 2; ++ni)
      #pragma unroll
      for (int i = 0; i < 4; ++i)
        #pragma unroll
        for (int j = 0; j < 2; ++j)
          #pragma unroll
          for (int r = 0; r < 4; ++r)
            Cs[(wm * 64 + i * 16 + q * 4 + r) * G8_CLD + ni * 128 + wn * 32 + j * 16 + r16] = acc[mi][ni][i][j][r];
    __syncthreads();
    // chunk c = base + u*512 has column group (c & 63), fixed per thread: the column operands
    // (bias, LayerNorm w/b of the residual) are loaded once, only rows vary
    const int cc = (threadIdx.x & 63) * 4, n = n0 + cc;
    const f32x4 bv = has_bias ? *(const f32x4*)(g.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
    const bool rln = g.rstats || g.rpart, fold = g.apart != nullptr;
    f32x4 lw = f32x4{1.f, 1.f, 1.f, 1.f}, lb = f32x4{0.f, 0.f, 0.f, 0.f}, ac = f32x4{0.f, 0.f, 0.f, 0.f};
    if (rln) {
      lw = *(const f32x4*)(g.rln_w + n);
      lb = *(const f32x4*)(g.rln_b + n);
    }
    if (fold) ac = *(const f32x4*)(g.acol + n);
    // MX-fp8 out: E8M0 bytes of this thread's 16 rows (w + 8k, k = 0..15: r16 = w + 8(k&1), i = (k>>1)&3,
    // wm = k>>3) gathered into the 4 scale dwords of the A layout, stored after the half
    unsigned scw[2][2] = {{0u, 0u}, {0u, 0u}};
    g8_sfor<0, CH / (512 * UNR)>([&](auto itc) {
      constexpr int it = decltype(itc)::value;
      const int base = threadIdx.x + it * 512 * UNR;
      f32x4 v[UNR], rv[UNR];
      float2 st[UNR], ast[UNR];
      long long off[UNR];
      int mrow[UNR];
      bool ok[UNR];
      #pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int row = (base + u * 512) >> 6;   // uniform over the wave: one wave = one 256-column row
        const int m = m0 + mi * 128 + row;
        ok[u] = m < M;
        const int mc = ok[u] ? m : 0;
        mrow[u] = mc;
        off[u] = (long long)mc * g.ldc + n;
        v[u] = *(const f32x4*)(Cs + row * G8_CLD + cc);
        rv[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        st[u] = make_float2(0.f, 1.f);
        ast[u] = make_float2(0.f, 1.f);
        if (has_res) {
          const long long ro = g.resid_rows ? (long long)(mc % g.resid_rows) * g.ldc + n : off[u];
          if (g.resid_t) {
            const bf16x4 rb = *(const bf16x4*)(g.resid_t + ro);
            rv[u] = f32x4{(float)rb[0], (float)rb[1], (float)rb[2], (float)rb[3]};
          } else {
            rv[u] = g8_ld<NT>((const f32x4*)(g.resid + ro));
          }
          if (g.rstats) st[u] = g.rstats[mc];
          else if (g.rpart) st[u] = ln_part_stats_n<3>(g.rpart, mc, g.ln_eps);
        }
        if (fold) ast[u] = ln_part_stats(g.apart, g.apart_nt, mc, g.ln_eps);
      }
      #pragma unroll
      for (int u = 0; u < UNR; ++u) {
        f32x4 o;
        if (fold) {   // LN(x) W^T + b = rstd (acc - mean acol) + b
          const float nm = -ast[u].x * ast[u].y;
          #pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = fmaf(v[u][e], ast[u].y, fmaf(nm, ac[e], bv[e]));
        } else {
          o = v[u] + bv;
        }
        if (gelu) {
          const f32x2 lo = gelu_erf2(f32x2{o[0], o[1]}), hi = gelu_erf2(f32x2{o[2], o[3]});
          o = f32x4{lo.x, lo.y, hi.x, hi.y};
        }
        if (gelu_fast) {
          const bool bfo = !g.Cf;   // bf16-only output: the degree-6 form
          const f32x2 lo = gelu_out2(f32x2{o[0], o[1]}, bfo), hi = gelu_out2(f32x2{o[2], o[3]}, bfo);
          o = f32x4{lo.x, lo.y, hi.x, hi.y};
        }
        f32x4 r = rv[u];
        if (rln) {   // LayerNorm of the residual, the exact expression of layernorm_kernel
          #pragma unroll
          for (int e = 0; e < 4; ++e) r[e] = fmaf((r[e] - st[u].x) * st[u].y, lw[e], lb[e]);
        }
        o += r;
        if (g.opart) {   // (mean, M2) of this row's 256 columns, two-pass over the wave's registers
          const float mt = wave_sum_fast(o[0] + o[1] + o[2] + o[3]) * (1.0f / 256.0f);
          const f32x4 d = o - mt;
          const float m2 = wave_sum_fast(d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3]);
          if (ok[u] && (threadIdx.x & 63) == 0)
            g.opart[(long long)mrow[u] * (g.N >> 8) + (n0 >> 8)] = make_float2(mt, m2);
        }
        if (MX && g.c_scale) {
          // MX-fp8 out: the wave holds one row's 256 columns, 8 lanes = one 32-column block
          const float a = max8_dpp(__builtin_elementwise_maximum(__builtin_elementwise_maximum(fabsf(o[0]), fabsf(o[1])),
                                                               __builtin_elementwise_maximum(fabsf(o[2]), fabsf(o[3]))));
          const int e = mx_scale_exp(a);
          const float inv = mx_inv_scale(e);
          int x = __builtin_amdgcn_cvt_pk_fp8_f32(o[0] * inv, o[1] * inv, 0, false);
          x = __builtin_amdgcn_cvt_pk_fp8_f32(o[2] * inv, o[3] * inv, x, true);
          if (ok[u]) *(int*)((unsigned char*)g.Ct + off[u]) = x;
          const int k = it * UNR + u;   // compile-time after unrolling
          scw[k & 1][(k >> 3) & 1] |= (unsigned)e << (8 * ((k >> 1) & 3));
          continue;
        }
        if (ok[u]) {
          if (g.Cf) g8_st<NT>((f32x4*)(g.Cf + off[u]), o);
          if (g.Ct) {
            const bf16x4 ob = {(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
            g8_st<NT>((bf16x4*)((bf16*)g.Ct + off[u]), ob);
          }
        }
      }
    });
    if (MX && g.c_scale && (threadIdx.x & 7) == 0) {
      const int w = threadIdx.x >> 6;
      #pragma unroll
      for (int h8 = 0; h8 < 2; ++h8)
        #pragma unroll
        for (int wq = 0; wq < 2; ++wq)
          *(unsigned*)(g.c_scale + mx_a_scale_off(m0 + mi * 128 + wq * 64 + w + 8 * h8, n >> 5, g.N >> 7)) = scw[h8][wq];
    }
  });
}


// ======================================================================================
// Persistent variant (default).  One block per CU walks tiles r*G + remap(b) (round r, the
// same XCD-aware remap per round).  After a tile's last MFMA the block first issues the NEXT
// tile's six prologue half-tiles, then runs this tile's direct epilogue: the epilogue math
// overlaps the prologue's HBM/L2 latency, and the epilogue's stores are left in flight -- the
// next tile's first K-tile waits vmcnt(2n + S) (S = store instructions issued after its
// prologue), so it needs only the prologue loads (older than the stores; vector-memory ops
// retire in issue order) and the stores drain under the first K-tile's MFMAs.  From K-tile 1
// on, waits target loads issued after the stores and the plain counts apply.
// ======================================================================================
// tile of block b in round r (-1: idle), XCD-aware bijective remap within the round
SSE_DEV int g8p_tile(int b, int r, int G, int n_tiles) {
  const int base = r * G;
  const int nwg = min(G, n_tiles - base);
  if (b >= nwg) return -1;
  const int q8 = nwg / 8, r8 = nwg % 8, x = b % 8;
  return base + (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + b / 8;
}

// Direct epilogue of one tile (acc holds C^T blocks, see gemm8_kernel<TR = true>): lane holds
// C[m][n .. n+3], m = m0 + mi*128 + wm*64 + i*16 + r16, n = n0 + ni*128 + wn*32 + j*16 + q*4.
// Vector-memory ops retire in issue order, so a load issued after a store cannot be waited for
// without waiting for the store too: every load (bias, LayerNorm columns, row statistics, the
// residual rows of both 128-row halves) is issued before the first store.  The half mi = 0 is
// finished in place in acc, then the residual of mi = 1 is loaded into the same registers, THEN
// the mi = 0 stores go out.
// RES = false compiles the residual out (the caller guarantees g.resid == nullptr).
// Q8 = true: Ct is MX-fp8 (e4m3 + g.c_scale, see store_half_q8).
// RB = true (with RES): the residual is the bf16 stream g.resid_t (MX fc2, in place: resid_t == Ct), read in the
// store layout (one 16-B load per (i, ni)) and redistributed with the inverse v_permlane16_swap when it is used;
// the same fp32 expression as the LDS-staged epilogue (o = acc + bias; o += r), so the results are bit-identical.
// FX: 0 = bias / activation read from g at run time; 1 = bias + ACT_GELU_FAST, 2 = bias, no activation (fixed at
// compile time: the caller guarantees g agrees)
// RSC (with Q8): the scales row-major, c_scale[m * (N / 32) + n / 32] (GemmArgs::c_scale_rm).
// VAM (bf16 out): the per-segment column amax of GemmArgs::vamax (see vamax_half below).
// RBL (with RB): the residual rows are in LDS (gemm8_kernel<MXE = 2> DMAs half 0 to rl0 during the last K-tile and
// half 1 to rl1 after the main loop; rows of 512 B, 16-B chunk c at c ^ (row & 15)); the caller has waited for half 0
template <bool RES, bool Q8, bool RB, int FX, bool RSC, bool VAM, bool RBL>
SSE_DEV void g8_epilogue_direct(const GemmArgs& g, f32x4 (&acc)[2][2][4][2], int m0, int n0, int wm, int wn,
                                int q, int r16, const char* rl0, const char* rl1) {
  const bool has_bias = FX ? true : g.bias != nullptr;
  const bool has_res = RES && (FX ? true : (RB ? g.resid_t != nullptr : g.resid != nullptr));
  const bool ln = RES && !FX && (g.rstats != nullptr || g.rpart != nullptr);
  const bool gelu = !FX && g.act == ACT_GELU, gelu_fast = FX == 1 || (!FX && g.act == ACT_GELU_FAST);
  f32x4 bv[2][2], lw[2][2], lb[2][2];
  #pragma unroll
  for (int ni = 0; ni < 2; ++ni)
    #pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + ni * 128 + wn * 32 + j * 16 + q * 4;
      bv[ni][j] = has_bias ? *(const f32x4*)(g.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
      lw[ni][j] = ln ? *(const f32x4*)(g.rln_w + n) : f32x4{1.f, 1.f, 1.f, 1.f};
      lb[ni][j] = ln ? *(const f32x4*)(g.rln_b + n) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  f32x4 rv[4][2][2];
  uint4 rvb[4][2];   // RB: the raw 16-B store-layout rows, unpacked where they are used
  float2 st[4];
  auto load_half = [&](int mi) {
    if (!has_res) return;
    if constexpr (RBL) {
      if (mi) {   // half 1's residual DMA (the only memory op still in flight) landed for every wave
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    }
    #pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + mi * 128 + wm * 64 + i * 16 + r16;
      const int mc = m < g.M ? m : 0;
      const long long rrow = g.resid_rows ? (long long)(mc % g.resid_rows) * g.ldc : (long long)mc * g.ldc;
      #pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        if constexpr (RB && RBL) {
          const int row = wm * 64 + i * 16 + r16, c = ni * 16 + wn * 4 + (q & 1) * 2 + (q >> 1);
          rvb[i][ni] = *(const uint4*)((mi ? rl1 : rl0) + row * 512 + ((c ^ r16) << 4));
        } else if constexpr (RB) {
          rvb[i][ni] = *(const uint4*)(g.resid_t + rrow + n0 + ni * 128 + wn * 32 + (q & 1) * 16 + (q >> 1) * 8);
        } else {
          #pragma unroll
          for (int j = 0; j < 2; ++j)
            rv[i][ni][j] = *(const f32x4*)(g.resid + rrow + n0 + ni * 128 + wn * 32 + j * 16 + q * 4);
        }
      }
      st[i] = !ln ? make_float2(0.f, 1.f) : (g.rstats ? g.rstats[mc] : ln_part_stats_n<3>(g.rpart, mc, g.ln_eps));
    }
  };
  auto finish_half = [&](int mi) {   // acc[mi] <- bias, activation, (LayerNorm'd) residual
    if constexpr (Q8 && !RES) {   // MX-fp8 out (fc1): the row block's 8 pairs through one lockstep GELU
      if (gelu_fast) {
        #pragma unroll
        for (int i = 0; i < 4; ++i) {
          f32x2 o2[8];
          #pragma unroll
          for (int u = 0; u < 4; ++u) {
            const f32x4 o = acc[mi][u >> 1][i][u & 1] + bv[u >> 1][u & 1];
            o2[2 * u] = f32x2{o[0], o[1]};
            o2[2 * u + 1] = f32x2{o[2], o[3]};
          }
          gelu_fp8out2_n<8>(o2);
          #pragma unroll
          for (int u = 0; u < 4; ++u) acc[mi][u >> 1][i][u & 1] = f32x4{o2[2 * u].x, o2[2 * u].y, o2[2 * u + 1].x, o2[2 * u + 1].y};
        }
        return;
      }
    }
    #pragma unroll
    for (int i = 0; i < 4; ++i)
      #pragma unroll
      for (int ni = 0; ni < 2; ++ni)
        #pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x4 o = acc[mi][ni][i][j] + bv[ni][j];
          if (gelu) {
            const f32x2 lo = gelu_erf2(f32x2{o[0], o[1]}), hi = gelu_erf2(f32x2{o[2], o[3]});
            o = f32x4{lo.x, lo.y, hi.x, hi.y};
          }
          if (gelu_fast) {   // fp8 out (Q8): the lower-degree form, its error far below e4m3 rounding
            const f32x2 lo = Q8 ? gelu_fp8out2(f32x2{o[0], o[1]}) : gelu_out2(f32x2{o[0], o[1]}, !g.Cf);
            const f32x2 hi = Q8 ? gelu_fp8out2(f32x2{o[2], o[3]}) : gelu_out2(f32x2{o[2], o[3]}, !g.Cf);
            o = f32x4{lo.x, lo.y, hi.x, hi.y};
          }
          if (has_res) {
            f32x4 r;
            if constexpr (RB) {
              const uint4 v = rvb[i][ni];
              const auto x = __builtin_amdgcn_permlane16_swap(v.x, v.z, false, false);
              const auto y = __builtin_amdgcn_permlane16_swap(v.y, v.w, false, false);
              r = unpack_h4<false>(j ? make_uint2(x[1], y[1]) : make_uint2(x[0], y[0]));
            } else {
              r = rv[i][ni][j];
            }
            if (ln) {   // LayerNorm of the residual, the exact expression of layernorm_kernel
              #pragma unroll
              for (int e = 0; e < 4; ++e) r[e] = fmaf((r[e] - st[i].x) * st[i].y, lw[ni][j][e], lb[ni][j][e]);
            }
            o += r;
          }
          acc[mi][ni][i][j] = o;
        }
  };
  // fp32 out: one 16-B store per (i, ni, j).  bf16 out: the two j blocks of a lane pair
  // (rows q, q^1 of 16 lanes) are exchanged with v_permlane16_swap so every lane holds 8
  // consecutive columns, n = n0 + ni*128 + wn*32 + (q&1)*16 + (q>>1)*8: one 16-B store per
  // (i, ni) instead of two 8-B stores (the per-CU store path is bound by instruction count).
  // Ct stores go through one buffer resource per 16-row block, based at (row m0 + mi*128 + 16 i, column n0),
  // num_records ending at row M (the range check sees the VGPR offset only, so the row block rides in the
  // base, not in the SGPR offset); es = Ct element bytes (2 bf16, 1 MX-fp8)
  auto ct_rsrc_of = [&](int mi, int i, int es) {
    const long long r0 = (long long)m0 + mi * 128 + i * 16;
    const long long rows = (long long)g.M - r0;
    const long long nrec = rows > 0 ? (rows * g.ldc - n0) * es : 0;
    return __builtin_amdgcn_make_buffer_rsrc((void*)((unsigned char*)g.Ct + (r0 * g.ldc + n0) * es), (short)0,
                                             (int)min(nrec, (long long)0x7FFFFFF0), 0x00020000);
  };
  const unsigned lane_col = (unsigned)(wn * 32 + (q & 1) * 16 + (q >> 1) * 8);
  const unsigned lane_off2 = (unsigned)(((wm * 64 + r16) * g.ldc + lane_col) * 2);
  auto store_half = [&](int mi) {
    #pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + mi * 128 + wm * 64 + i * 16 + r16;
      const bool ok = m < g.M;
      const long long row = (long long)(ok ? m : 0) * g.ldc;
      #pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        if (g.Cf && ok) {
          #pragma unroll
          for (int j = 0; j < 2; ++j)
            *(f32x4*)(g.Cf + row + n0 + ni * 128 + wn * 32 + j * 16 + q * 4) = acc[mi][ni][i][j];
        }
        if (g.Ct) {
          const f32x4 o0 = acc[mi][ni][i][0], o1 = acc[mi][ni][i][1];
          const bf16x4 x0 = {(bf16)o0[0], (bf16)o0[1], (bf16)o0[2], (bf16)o0[3]};
          const bf16x4 x1 = {(bf16)o1[0], (bf16)o1[1], (bf16)o1[2], (bf16)o1[3]};
          const uint2 X = __builtin_bit_cast(uint2, x0), Y = __builtin_bit_cast(uint2, x1);
          const auto s0 = __builtin_amdgcn_permlane16_swap(X.x, Y.x, false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(X.y, Y.y, false, false);
          // the row block's buffer resource (rows >= M out of range): no 64-bit address math, no branch
          const u32x4 v = {s0[0], s1[0], s0[1], s1[1]};
          __builtin_amdgcn_raw_buffer_store_b128(v, ct_rsrc_of(mi, i, 2), lane_off2 + (unsigned)(ni * 256), 0u, 0);
        }
      }
    }
  };
  // MX-fp8 out (the next GEMM's A operand): the 32 columns n0 + ni*128 + wn*32 + [0, 32) of a row
  // are one MX block, held by the row's four q lanes (j = 0, 1 each).  amax over the 8 values and
  // across q (xor 16, 32), E8M0 exponent mx_scale_exp, e4m3 = RNE(x * 2^-E) (v_cvt_pk_fp8_f32),
  // the same lane-pair exchange as the bf16 path (8 consecutive bytes per lane).  The four lanes of
  // a row hold the same exponents; lane q stores the scale dword (i = 0..3) of (mi, ni) = (q>>1, q&1).
  unsigned scw[2][2] = {{0u, 0u}, {0u, 0u}};
  // Round 6: the two 128-column halves' 8-byte pieces of a row block are paired by one more lane-group swap
  // (v_permlane32_swap: lanes q < 2 take half 0's 16 consecutive bytes, q >= 2 half 1's), so a row block goes out as
  // ONE 16-B store per lane instead of two 8-B ones -- the per-CU store path costs per instruction, not per byte
  //  -- and the row-major scales (RSC) as one byte store per half with every lane active (lane q
  // stores row block i = q's exponent) instead of one per row block with a quarter of the lanes.
  const unsigned lane_off16 = (unsigned)((wm * 64 + r16) * g.ldc + wn * 32 + (q & 1) * 16 + (q >> 1) * 128);
  auto store_half_q8 = [&](int mi) {
    int esel[2] = {0, 0};   // RSC: the exponents of row block i = q
    #pragma unroll
    for (int i = 0; i < 4; ++i) {
      u32x2 d[2];
      #pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const f32x4 o0 = acc[mi][ni][i][0], o1 = acc[mi][ni][i][1];
        // (IEEE maximum: the MFMA outputs go in as they are -- fmaxf's maxnum would canonicalise every operand first)
        float a = __builtin_elementwise_maximum(
            __builtin_elementwise_maximum(__builtin_elementwise_maximum(fabsf(o0[0]), fabsf(o0[1])),
                                          __builtin_elementwise_maximum(fabsf(o0[2]), fabsf(o0[3]))),
            __builtin_elementwise_maximum(__builtin_elementwise_maximum(fabsf(o1[0]), fabsf(o1[1])),
                                          __builtin_elementwise_maximum(fabsf(o1[2]), fabsf(o1[3]))));
        {   // the row's four q lanes: max over q ^ 1 then q ^ 2 by lane-group swaps (VALU, no LDS round trip)
          const auto t16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(a), false, false);
          a = __builtin_elementwise_maximum(__uint_as_float(t16[0]), __uint_as_float(t16[1]));
          const auto t32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(a), false, false);
          a = __builtin_elementwise_maximum(__uint_as_float(t32[0]), __uint_as_float(t32[1]));
        }
        const int e = mx_scale_exp(a);
        // e4m3 = RNE(x / 2^(e - 127)) by the scaled conversion (the scale's exponent field only: tools/probe_cvt.hip
        // checks it against cvt_pk_fp8_f32(x * 2^-E) bit for bit); a block of zeros / denormals (e = 0) divides by
        // 2^-126 instead of 2^-127
        const float sc = __builtin_bit_cast(float, (unsigned)(e > 0 ? e : 1) << 23);
        v2i16g8 w0 = {0, 0}, w1 = {0, 0};
        w0 = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(w0, o0[0], o0[1], sc, false);
        w0 = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(w0, o0[2], o0[3], sc, true);
        w1 = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(w1, o1[0], o1[1], sc, false);
        w1 = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(w1, o1[2], o1[3], sc, true);
        const int x0 = __builtin_bit_cast(int, w0), x1 = __builtin_bit_cast(int, w1);
        const auto sw = __builtin_amdgcn_permlane16_swap((unsigned)x0, (unsigned)x1, false, false);
        d[ni] = u32x2{sw[0], sw[1]};   // 8 consecutive bytes: columns (q & 1) * 16 + (q >> 1) * 8 of block (ni, wn)
        if constexpr (RSC) {   // the row's four q lanes hold the same exponent: lane q keeps row block i = q's
          esel[ni] = q == i ? e : esel[ni];
        } else {
          scw[mi][ni] |= (unsigned)e << (8 * i);
        }
      }
      // v_permlane32_swap swaps lanes 32-63 of its first operand with lanes 0-31 of its second: lanes 0-31 (q < 2) end
      // with their own half-0 piece | lane + 32's half-0 piece, lanes 32-63 with lane - 32's half-1 piece | their own
      const auto t0 = __builtin_amdgcn_permlane32_swap(d[0][0], d[1][0], false, false);
      const auto t1 = __builtin_amdgcn_permlane32_swap(d[0][1], d[1][1], false, false);
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{t0[0], t1[0], t0[1], t1[1]}, ct_rsrc_of(mi, i, 1), lane_off16, 0u, 0);
    }
    if constexpr (RSC) {
      const int m = m0 + mi * 128 + wm * 64 + q * 16 + r16;
      if (m < g.M) {
        #pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          g.c_scale[(long long)m * (g.N >> 5) + ((n0 + ni * 128 + wn * 32) >> 5)] = (unsigned char)esel[ni];
      }
    }
  };
  // VAM: max |C| over this wave's 64 rows of half mi (m = mb + 16 i + r16) per column and row segment
  // (m / vamax_rows: at most two segments, vamax_rows >= 64), rows >= M excluded.  Per lane the 16 columns
  // (ni, j, e) are first reduced over its 4 rows, then over the 16 r16 lanes by a halving butterfly (DPP
  // row_mirror, row_half_mirror, quad xor 2, xor 1: each step keeps half the columns, so lane r16 ends with
  // column k = r16 = 8 ni + 4 j + e) and rounded to bf16 (RNE is monotone: bf16(max |x|) = max |bf16(x)|).
  // The atomicMax of the float bits (one per lane and segment) is issued after the last store (vam_flush): an
  // atomic stays in vmcnt for thousands of cycles under contention, and any later wait would take it along.
  float vres[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
  int vseg[2][2] = {{-1, -1}, {-1, -1}};
  auto vamax_half = [&](int mi) {
    const int R = g.vamax_rows;
    const int mb = m0 + mi * 128 + wm * 64;
    if (mb >= g.M) return;
    const int c0 = mb / R, c1 = min(mb + 63, g.M - 1) / R;
    #pragma unroll
    for (int part = 0; part < 2; ++part) {
      const int cs = c0 + part;
      if (cs > c1) break;
      const int lo = cs * R, hi = min(lo + R, g.M);
      float v[16];
      if (lo <= mb && hi >= mb + 64) {   // every row of the block in this segment (wave-uniform)
        #pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          #pragma unroll
          for (int j = 0; j < 2; ++j)
            #pragma unroll
            for (int e = 0; e < 4; ++e)
              v[ni * 8 + j * 4 + e] = __builtin_elementwise_maximum(
                  __builtin_elementwise_maximum(fabsf(acc[mi][ni][0][j][e]), fabsf(acc[mi][ni][1][j][e])),
                  __builtin_elementwise_maximum(fabsf(acc[mi][ni][2][j][e]), fabsf(acc[mi][ni][3][j][e])));
      } else {
        bool ok[4];
        #pragma unroll
        for (int i = 0; i < 4; ++i) ok[i] = mb + i * 16 + r16 >= lo && mb + i * 16 + r16 < hi;
        #pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          #pragma unroll
          for (int j = 0; j < 2; ++j)
            #pragma unroll
            for (int e = 0; e < 4; ++e) {
              float t = 0.f;
              #pragma unroll
              for (int i = 0; i < 4; ++i) t = __builtin_elementwise_maximum(t, ok[i] ? fabsf(acc[mi][ni][i][j][e]) : 0.f);
              v[ni * 8 + j * 4 + e] = t;
            }
      }
      auto step = [&](auto hc, int bit, auto ctl) {
        constexpr int h = decltype(hc)::value;
        const bool up = (r16 >> bit) & 1;
        #pragma unroll
        for (int k = 0; k < h; ++k) {
          const float snd = up ? v[k] : v[k + h];
          const float kp = up ? v[k + h] : v[k];
          const float rc = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(snd), decltype(ctl)::value, 0xF, 0xF, false));
          v[k] = __builtin_elementwise_maximum(kp, rc);
        }
      };
      step(std::integral_constant<int, 8>{}, 3, std::integral_constant<int, 0x140>{});   // row_mirror
      step(std::integral_constant<int, 4>{}, 2, std::integral_constant<int, 0x141>{});   // row_half_mirror
      step(std::integral_constant<int, 2>{}, 1, std::integral_constant<int, 0x4E>{});    // quad [2,3,0,1]
      step(std::integral_constant<int, 1>{}, 0, std::integral_constant<int, 0xB1>{});    // quad [1,0,3,2]
      vres[mi][part] = (float)(bf16)v[0];
      vseg[mi][part] = cs;
    }
  };
  auto vam_flush = [&]() {
    const int k = r16;
    const int n = n0 + (k >> 3) * 128 + wn * 32 + ((k >> 2) & 1) * 16 + q * 4 + (k & 3);
    #pragma unroll
    for (int mi = 0; mi < 2; ++mi)
      #pragma unroll
      for (int part = 0; part < 2; ++part)
        if (vseg[mi][part] >= 0)
          __hip_atomic_fetch_max(g.vamax + (long long)vseg[mi][part] * g.N + n, __float_as_uint(vres[mi][part]),
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  load_half(0);
  finish_half(0);
  if constexpr (VAM) vamax_half(0);
  load_half(1);
  if constexpr (Q8) store_half_q8(0); else store_half(0);
  finish_half(1);
  if constexpr (VAM) vamax_half(1);
  if constexpr (VAM) {
    store_half(1);
    vam_flush();
  } else if constexpr (Q8 && RSC) {
    store_half_q8(1);
  } else if constexpr (Q8) {
    store_half_q8(1);
    const int mi = q >> 1, ni = q & 1;
    const unsigned v = mi ? (ni ? scw[1][1] : scw[1][0]) : (ni ? scw[0][1] : scw[0][0]);
    const long long m = m0 + mi * 128 + wm * 64 + r16;
    *(unsigned*)(g.c_scale + mx_a_scale_off(m, (n0 + ni * 128 + wn * 32) >> 5, g.N >> 7)) = v;
  } else {
    store_half(1);
  }
}

// Epilogue parameters of one tile of the persistent kernel, staged in LDS (one slot per tile,
// two slots): bias[256] fp32 | acol[256] fp32 (folded LayerNorm column sums) | row partials
// [256][3] (mean_t, M2_t) float2.  Each wave issues ONE LDS-DMA of 1 KiB per tile (waves 0-5 the
// partials, 6 the bias, 7 acol) BEFORE that tile's prologue, so the epilogue issues no global
// load at all: it never waits for the next tile's prologue (a global load issued after it could
// only be waited for behind it: vector-memory ops retire in issue order).
constexpr int G8P_EP = 2048 + 256 * 5 * 8;   // 12 KiB per slot: row partials of up to 5 column tiles (H <= 1280)
constexpr int G8P_SMEM = G8_OPS + 2 * G8P_EP;

// Direct epilogue of one tile (acc holds C^T blocks, see gemm8_kernel<TR = true>): lane holds
// C[m][n .. n+3], m = m0 + mi*128 + wm*64 + i*16 + r16, n = n0 + ni*128 + wn*32 + j*16 + q*4.
//   o = act(rstd_m * acc + (bias[n] - rstd_m mean_m acol[n]))   (folded LayerNorm of A, GemmArgs.apart)
//   o = act(acc + bias[n])                                        (otherwise: rstd = 1 and the acol term
//                                                                  is not formed, bit-identical to a plain add)
// DBG (timing probes only, tools/gemm8_probe.hip; the library launches DBG = 0): 1 = math without the
// stores (results kept live by an empty asm), 3 = stores of the raw accumulators without the math.
// FNT: 256-column tiles per row of the folded LayerNorm's input (apart_nt: 3 for H = 768 .. 5 for 1280)
template <int ACT, bool CT3, bool F16, bool has_bias, bool fold, int DBG = 0, int FNT = 3>
SSE_DEV void g8p_epilogue(const GemmArgs& g, f32x4 (&acc)[2][2][4][2], int m0, int n0, int wm, int wn, int q,
                          int r16, const char* ep) {
  {   // lane-derived values recomputed here from an opaque lane id: the compiler hoisted them out of the tile
      // loop, where they held ~12 VGPRs through the main loop (246 -> 234 VGPRs, round 5)
    int ln = (int)(threadIdx.x & 63);
    asm volatile("" : "+v"(ln));
    q = ln >> 4;
    r16 = ln & 15;
  }
  const float alpha = F16 ? g.alpha : 1.f;   // split-fp16: the weights' 2^s undone (exact)
  f32x4 bv[2][2], ac[2][2];
  #pragma unroll
  for (int ni = 0; ni < 2; ++ni)
    #pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = ni * 128 + wn * 32 + j * 16 + q * 4;
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      const f32x4 b = *(const f32x4*)(ep + c * 4), a = *(const f32x4*)(ep + 1024 + c * 4);
      bv[ni][j] = has_bias ? b : z;   // compile-time: absent terms fold away
      ac[ni][j] = fold ? a : z;
    }
  auto finish_half = [&](int mi) {
    if constexpr (DBG == 3) return;
    // this half's row statistics, read from LDS here (a memory barrier keeps the compiler from hoisting
    // the second half's reads: held for the whole tile they cost 8 more registers at the peak)
    asm volatile("" ::: "memory");
    float2 ast[4];
    #pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float2* p = (const float2*)(ep + 2048) + (mi * 128 + wm * 64 + i * 16 + r16) * FNT;
      float2 st;
      if constexpr (FNT == 3) {
        const float2 v[3] = {p[0], p[1], p[2]};
        st = ln_part_combine<3>(v, g.ln_eps);
      } else {
        float2 v[FNT];
        #pragma unroll
        for (int t = 0; t < FNT; ++t) v[t] = p[t];
        st = ln_part_combine<FNT>(v, g.ln_eps);
      }
      ast[i] = fold ? st : make_float2(0.f, alpha);
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
      // the row block's 8 pairs through one lockstep polynomial (gelu_out2_n: 8 independent chains keep the
      // VALU issuing; one chain at a time is latency-bound with a hazard nop per dependent packed fma), with
      // or without the fold: since the row statistics are read per half, the folded GELU_FAST kernel
      // (gemm8p_kernel<ACT_GELU_FAST, false, false, 3, 0, 3>, WavLM-base ffn1) holds 256 VGPRs, 0 spilled
      // (hipcc -Rpass-analysis=kernel-resource-usage, round 5); FNT = 4 / 5 spill 8 / 15 and are not launched
      // with GELU (the Whisper-large-v2 fc1 keeps its LayerNorm kernel).
      if constexpr (ACT == ACT_GELU_FAST) {
        f32x2 o2[8];
        #pragma unroll
        for (int u = 0; u < 4; ++u) {
          const f32x4 v = acc[mi][u >> 1][i][u & 1];
          o2[2 * u] = f32x2{v[0], v[1]};
          o2[2 * u + 1] = f32x2{v[2], v[3]};
        }
        gelu_out2_n<F16 || CT3, 8>(o2);
        #pragma unroll
        for (int u = 0; u < 4; ++u) acc[mi][u >> 1][i][u & 1] = f32x4{o2[2 * u].x, o2[2 * u].y, o2[2 * u + 1].x, o2[2 * u + 1].y};
      }
    }
  };
  // fp32 out: one 16-B store per (i, ni, j).  bf16 out: the two j blocks of a lane pair are exchanged
  // with v_permlane16_swap so every lane holds 8 consecutive columns: one 16-B store per (i, ni), through
  // a buffer resource based at the tile's first row (no 64-bit address math, no exec-mask branch per
  // store: rows >= M fall outside its num_records)
  // One resource per 16-row block i, based at element (m0 + 16 i, n0): its num_records ends at row M's
  // column n0, so every column of rows < M is in range (n0 + 256 (+ 2N, CT3) <= ldc) and every row >= M out.
  // (The row block cannot ride in the SGPR offset of one tile-wide resource: the range check sees only the
  // VGPR offset + immediate, so rows >= M of a partial tile would be written.)
  auto ct_rsrc_of = [&](int i) {
    const long long rows = (long long)g.M - m0 - 16 * i;
    const long long nrec = rows > 0 ? rows * g.ldc * 2 - (long long)n0 * 2 : 0;
    return __builtin_amdgcn_make_buffer_rsrc((void*)((bf16*)g.Ct + (long long)(m0 + 16 * i) * g.ldc + n0), (short)0,
                                             (int)min(nrec, (long long)0x7FFFFFF0), 0x00020000);
  };
  const unsigned lane_off = (unsigned)(((wm * 64 + r16) * g.ldc + wn * 32 + (q & 1) * 16 + (q >> 1) * 8) * 2);
  auto store_half = [&](int mi) {
    #pragma unroll
    for (int i = 0; i < 4; ++i) {
      const __amdgpu_buffer_rsrc_t ct_rsrc = ct_rsrc_of(i);
      const int m = m0 + mi * 128 + wm * 64 + i * 16 + r16;
      const bool ok = m < g.M;
      const long long row = (long long)(ok ? m : 0) * g.ldc;
      #pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        if (g.Cf && ok) {
          #pragma unroll
          for (int j = 0; j < 2; ++j)
            *(f32x4*)(g.Cf + row + n0 + ni * 128 + wn * 32 + j * 16 + q * 4) = acc[mi][ni][i][j];
        }
        if (g.Ct) {
          const f32x4 o0 = acc[mi][ni][i][0], o1 = acc[mi][ni][i][1];
          uint2 X, Y, LX, LY;   // hi (and, CT3, the lo' plane) of the two j blocks
          if constexpr (F16) {
            f16x4 h0, h1, l0, l1;
            x3_split4(o0, h0, l0);
            x3_split4(o1, h1, l1);
            X = __builtin_bit_cast(uint2, h0);
            Y = __builtin_bit_cast(uint2, h1);
            LX = __builtin_bit_cast(uint2, l0);
            LY = __builtin_bit_cast(uint2, l1);
          } else {
            const bf16x4 x0 = {(bf16)o0[0], (bf16)o0[1], (bf16)o0[2], (bf16)o0[3]};
            const bf16x4 x1 = {(bf16)o1[0], (bf16)o1[1], (bf16)o1[2], (bf16)o1[3]};
            X = __builtin_bit_cast(uint2, x0);
            Y = __builtin_bit_cast(uint2, x1);
            LX = LY = make_uint2(0u, 0u);
          }
          const auto s0 = __builtin_amdgcn_permlane16_swap(X.x, Y.x, false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(X.y, Y.y, false, false);
          const long long c = n0 + ni * 128 + wn * 32 + (q & 1) * 16 + (q >> 1) * 8;
          if constexpr (DBG == 1) {
            asm volatile("" ::"v"(s0[0]), "v"(s0[1]), "v"(s1[0]), "v"(s1[1]));
            continue;
          }
          // the row block's buffer resource: lane offset (one VGPR per half) + the column block as an
          // immediate; rows >= M are dropped by the range check
          const unsigned soff = 0u;
          const unsigned voff = lane_off + (unsigned)(mi * 128 * g.ldc * 2) + (unsigned)(ni * 256);
          const u32x4 v = {s0[0], s1[0], s0[1], s1[1]};
          __builtin_amdgcn_raw_buffer_store_b128(v, ct_rsrc, voff, soff, 0);
          if constexpr (CT3) {   // [hi | lo' | hi]: the second hi plane and the lo' plane
            __builtin_amdgcn_raw_buffer_store_b128(v, ct_rsrc, voff + (unsigned)(4 * g.N), soff, 0);
            const auto t0 = __builtin_amdgcn_permlane16_swap(LX.x, LY.x, false, false);
            const auto t1 = __builtin_amdgcn_permlane16_swap(LX.y, LY.y, false, false);
            const u32x4 lv = {t0[0], t1[0], t0[1], t1[1]};
            __builtin_amdgcn_raw_buffer_store_b128(lv, ct_rsrc, voff + (unsigned)(2 * g.N), soff, 0);
          }
        }
      }
    }
  };
  finish_half(0);
  store_half(0);
  finish_half(1);
  store_half(1);
}

// ======================================================================================
// Persistent variant (default for bf16 GEMMs without a residual).  One block per CU walks tiles
// r*G + remap(b) (round r, the same XCD-aware remap per round).  After a tile's last MFMA the block
// issues the NEXT tile's epilogue-parameter DMA and six prologue half-tiles, then runs this tile's
// epilogue from LDS: its math overlaps the prologue's HBM/L2 latency, and its stores are left in
// flight -- the next tile's first K-tile waits vmcnt(2n + S) (S = store instructions issued after
// its prologue), so it needs only the prologue loads and the stores drain under its MFMAs.
// ======================================================================================
// EP: bit 0 = bias present, bit 1 = folded LayerNorm (apart/acol) -- compile-time, so an absent term
// costs no epilogue instruction (runtime selects measured +5-6 % on conv1 / ffn1 when removed).
// DBG (timing probes only): see g8p_epilogue; 2 = no epilogue at all (accumulators kept live); 4 = no epilogue and
// no MFMA (the LDS fragment reads kept live); 5 = no epilogue and no main-loop LDS-DMA.
// PH2 (round 6, the default; option gemm_4phase = 1 keeps four): two phases per K-tile instead of four -- Q0 reads A0, B0, B1 and runs A0 B0 and
// A0 B1 (32 MFMAs), Q1 reads A1 and runs A1 B1, A1 B0 -- so half the barriers per K-tile and 32-MFMA sections.  Issue
// schedule (2-phase index j = 2t + h): Q0(t) -> A1(t+1), Q1(t) -> A0, B0, B1(t+2) (their slots' previous occupants
// were read in Q0(t)); the prologue is j = -3 .. -1 (all of tile 0, then A0, B0, B1 of tile 1).  Every half is
// issued two phases before its first read and the wait at the end of L(j) leaves ops(j) + ops(j - 1) in flight
// (8 in steady state, as the 4-phase schedule).
template <int ACT, bool CT3 = false, bool F16 = false, int EP = 1, int DBG = 0, int FNT = 3, bool PH2 = false>
__global__ __launch_bounds__(512) void gemm8p_kernel(GemmArgs g, int n_tiles) {
  __shared__ __attribute__((aligned(16))) char smem[G8P_SMEM];   // operands | 2 epilogue slots: the ONLY shared object
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int q = lane >> 4, r16 = lane & 15;
  const int M = g.M, K = g.K;
  const int n_tiles_n = g.N / 256;
  const int nk = K / 64;
  const int G = gridDim.x, b = blockIdx.x;
  // stores per wave of one full tile (the count the next tile's first K-tile may leave in
  // flight); under-counting is safe, so it is capped to keep 2n + S within vmcnt's 6 bits
  const int s_full = min(32 * (g.Cf ? 1 : 0) + (CT3 ? 48 : 16) * (g.Ct ? 1 : 0), 54);   // 54 + 9 <= 63
  constexpr bool has_bias = (EP & 1) != 0, fold = (EP & 2) != 0;

  int round = 0;
  int tile = g8p_tile(b, 0, G, n_tiles);
  if (tile < 0) return;
  if constexpr (DBG >= 6) {   // probe: half of each XCD's blocks start (DBG - 5) x 6 us late (desynchronised epilogues)
    if ((b >> 3) & 1) {
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__builtin_amdgcn_s_memrealtime() - t0 < 600ull * (DBG - 5)) __builtin_amdgcn_s_sleep(8);
    }
  }

  constexpr int NREC = 0x7FFFFFF0;
  __amdgpu_buffer_rsrc_t a_rsrc, b_rsrc;
  unsigned a_voff[2][2], b_voff[2][2];
  auto setup = [&](int tl) {
    const int m0 = (tl / n_tiles_n) * 256, n0 = (tl % n_tiles_n) * 256;
    const int mf = m0 < M ? m0 : M - 1;
    const int seg0 = mf / g.rows_per_seg, rr0 = mf - seg0 * g.rows_per_seg;
    const long long a_base = ((long long)seg0 * g.seg_stride + (long long)rr0 * g.lda) * 2;   // bytes
    a_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)g.A + a_base), (short)0, NREC, 0x00020000);
    b_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)g.B + (long long)n0 * K * 2), (short)0, NREC,
                                               0x00020000);
    #pragma unroll
    for (int h = 0; h < 2; ++h)
      #pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int row = h * 128 + (wave + 8 * s) * 8 + (lane >> 3);
        const int ch = (lane & 7) ^ ((row >> 1) & 7);
        int m = m0 + row;
        m = m < M ? m : M - 1;
        const int seg = m / g.rows_per_seg, rr = m - seg * g.rows_per_seg;
        const long long el = ((long long)seg * g.seg_stride + (long long)rr * g.lda) * 2 + ch * 16;
        a_voff[h][s] = (unsigned)(el - a_base);
        b_voff[h][s] = (unsigned)((long long)row * K * 2 + ch * 16);
      }
  };
  auto issue_half = [&](int tl, int half) {
    char* dst = smem + (tl & 1) * G8_BUF + half * G8_HALF;
    const unsigned soff = (unsigned)tl * 128u;
    if (half < 2) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, LPTR(dst + wave * 1024), 16, a_voff[half][0], soff, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, LPTR(dst + (wave + 8) * 1024), 16, a_voff[half][1], soff, 0, 0);
    } else {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, LPTR(dst + wave * 1024), 16, b_voff[half - 2][0], soff, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, LPTR(dst + (wave + 8) * 1024), 16, b_voff[half - 2][1], soff, 0,
                                               0);
    }
  };
  auto issue = [&](int k) {
    if (k < -6) return;
    int tl, half;
    g8_target(k, tl, half);
    if (tl >= nk) return;
    issue_half(tl, half);
  };
  // PH2 schedule (see the template comment)
  auto issue2 = [&](int j) { g8_issue2(j, nk, issue_half); };
  auto count2 = [&](int j) { return g8_count2(j, nk); };
  auto prologue = [&]() {
    if constexpr (PH2) {
      for (int j = -3; j < 0; ++j) issue2(j);
    } else {
      for (int k = -6; k < 0; ++k) issue(k);
    }
  };
  // epilogue-parameter DMA of tile tl into slot: 1 KiB pieces -- the row partials (2 FNT pieces), the bias,
  // the folded column sums -- wave w issuing pieces w and w + 8 (FNT = 3: one per wave); absent operands read
  // as an empty buffer (num_records 0, nothing is fetched; the epilogue ignores the slot bytes).  These DMAs
  // precede the tile's prologue, so the counted waits retire them with it however many a wave issued.
  const void* zb = g.zero;
  auto ep_issue = [&](int tl, int slot) {
    const int m0 = (tl / n_tiles_n) * 256, n0 = (tl % n_tiles_n) * 256;
    char* dst = smem + G8_OPS + slot * G8P_EP;
    if constexpr (FNT == 3) {   // one piece per wave: waves 0-5 the partials, 6 the bias, 7 the column sums
      __amdgpu_buffer_rsrc_t r;
      unsigned soff;
      int off;
      if (wave < 6) {
        r = __builtin_amdgcn_make_buffer_rsrc((void*)(fold ? (const void*)g.apart : zb), (short)0, fold ? M * 24 : 0,
                                              0x00020000);
        soff = (unsigned)(m0 * 24 + wave * 1024);
        off = 2048 + wave * 1024;
      } else if (wave == 6) {
        r = __builtin_amdgcn_make_buffer_rsrc((void*)(has_bias ? (const void*)g.bias : zb), (short)0,
                                              has_bias ? g.N * 4 : 0, 0x00020000);
        soff = (unsigned)(n0 * 4);
        off = 0;
      } else {
        r = __builtin_amdgcn_make_buffer_rsrc((void*)(fold ? (const void*)g.acol : zb), (short)0, fold ? g.N * 4 : 0,
                                              0x00020000);
        soff = (unsigned)(n0 * 4);
        off = 1024;
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, LPTR(dst + off), 16, (unsigned)lane * 16u, soff, 0, 0);
      return;
    }
    constexpr int NP = 2 * FNT + 2;
    #pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int pc = wave + 8 * k;
      if (pc >= NP) break;
      __amdgpu_buffer_rsrc_t r;
      unsigned soff;
      int off;
      if (pc < 2 * FNT) {
        r = __builtin_amdgcn_make_buffer_rsrc((void*)(fold ? (const void*)g.apart : zb), (short)0,
                                              fold ? M * FNT * 8 : 0, 0x00020000);
        soff = (unsigned)(m0 * FNT * 8 + pc * 1024);
        off = 2048 + pc * 1024;
      } else if (pc == 2 * FNT) {
        r = __builtin_amdgcn_make_buffer_rsrc((void*)(has_bias ? (const void*)g.bias : zb), (short)0,
                                              has_bias ? g.N * 4 : 0, 0x00020000);
        soff = (unsigned)(n0 * 4);
        off = 0;
      } else {
        r = __builtin_amdgcn_make_buffer_rsrc((void*)(fold ? (const void*)g.acol : zb), (short)0, fold ? g.N * 4 : 0,
                                              0x00020000);
        soff = (unsigned)(n0 * 4);
        off = 1024;
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, LPTR(dst + off), 16, (unsigned)lane * 16u, soff, 0, 0);
    }
  };

  f32x4 acc[2][2][4][2];
  bf16x8 af[4][2], b0f[2][2], b1f[2][2];
  auto read_a = [&](const char* hb) {
    #pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + i * 16 + r16;
      #pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        af[i][ks] = *(const bf16x8*)(hb + row * 128 + (((q + 4 * ks) ^ ((row >> 1) & 7)) * 16));
    }
  };
  auto read_b = [&](const char* hb, bf16x8 (&bf)[2][2]) {
    #pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = wn * 32 + j * 16 + r16;
      #pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        bf[j][ks] = *(const bf16x8*)(hb + row * 128 + (((q + 4 * ks) ^ ((row >> 1) & 7)) * 16));
    }
  };
  auto mma = [&](f32x4 (&c)[4][2], const bf16x8 (&bf)[2][2]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (DBG == 4) {   // probe: no MFMA (the fragment reads kept live)
      #pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        #pragma unroll
        for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(af[i][ks]));
        #pragma unroll
        for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(bf[j][ks]));
      }
    } else {
      #pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        #pragma unroll
        for (int i = 0; i < 4; ++i)
          #pragma unroll
          for (int j = 0; j < 2; ++j) c[i][j] = g8_mfma<F16>(bf[j][ks], af[i][ks], c[i][j]);
    }
    __builtin_amdgcn_sched_barrier(0);
  };

  int slot = 0;
  ep_issue(tile, 0);
  setup(tile);
  prologue();
  int S = 0;   // store instructions issued after the current tile's prologue
  while (true) {
    const int m0 = (tile / n_tiles_n) * 256, n0 = (tile % n_tiles_n) * 256;
    #pragma unroll
    for (int a = 0; a < 2; ++a)
      #pragma unroll
      for (int c = 0; c < 2; ++c)
        #pragma unroll
        for (int i = 0; i < 4; ++i)
          #pragma unroll
          for (int j = 0; j < 2; ++j) acc[a][c][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the epilogue-parameter DMA precedes the prologue: retired by the same counted waits
    g8_vmcnt_dyn<false>((PH2 ? count2(-1) : g8_count<false>(-1, nk)) + S);
    g8_barrier();
    if (wm == 1) g8_barrier();   // group 1 runs one barrier behind

    // FIRST: 0 = steady, 1 = first K-tile (waits leave the previous tile's S stores in flight)
    auto run_tile = [&](int t, auto steady, auto first) {
      constexpr bool ST = decltype(steady)::value;
      constexpr bool FI = decltype(first)::value;
      const char* buf = smem + (t & 1) * G8_BUF;
      const int k = 4 * t;
      auto issue_wait = [&](int kk) {
        if constexpr (DBG != 5) issue(kk);   // probe 5: no main-loop DMA
        if constexpr (FI) {
          g8_vmcnt_dyn<false>(g8_count<false>(kk, nk) + S);
        } else if constexpr (ST) {
          asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
          g8_wait<false>(kk, nk);
        }
      };
      read_a(buf);
      read_b(buf + 2 * G8_HALF, b0f);
      issue_wait(k);
      g8_barrier();
      mma(acc[0][0], b0f);
      g8_barrier();
      read_b(buf + 3 * G8_HALF, b1f);
      issue_wait(k + 1);
      g8_barrier();
      mma(acc[0][1], b1f);
      g8_barrier();
      read_a(buf + G8_HALF);
      issue_wait(k + 2);
      g8_barrier();
      mma(acc[1][1], b1f);
      g8_barrier();
      issue_wait(k + 3);
      g8_barrier();
      mma(acc[1][0], b0f);
      g8_barrier();
    };
    // PH2: the same K-tile in two phases of 32 MFMAs
    auto run_tile2 = [&](int t, auto steady, auto first) {
      constexpr bool ST = decltype(steady)::value;
      constexpr bool FI = decltype(first)::value;
      const char* buf = smem + (t & 1) * G8_BUF;
      const int j = 2 * t;
      auto issue_wait = [&](int jj) {
        if constexpr (DBG != 5) issue2(jj);
        if constexpr (FI) {
          g8_vmcnt_dyn<false>(count2(jj) + S);
        } else if constexpr (ST) {
          asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
          g8_vmcnt_dyn<false>(count2(jj));
        }
      };
      read_a(buf);
      read_b(buf + 2 * G8_HALF, b0f);
      read_b(buf + 3 * G8_HALF, b1f);
      issue_wait(j);
      g8_barrier();
      mma(acc[0][0], b0f);
      mma(acc[0][1], b1f);
      g8_barrier();
      read_a(buf + G8_HALF);
      issue_wait(j + 1);
      g8_barrier();
      mma(acc[1][1], b1f);
      mma(acc[1][0], b0f);
      g8_barrier();
    };
    using F_ = std::integral_constant<bool, false>;
    using T_ = std::integral_constant<bool, true>;
    int t = 1;
    if constexpr (PH2) {
      run_tile2(0, F_{}, T_{});
      for (; t + 2 < nk; ++t) run_tile2(t, T_{}, F_{});
      for (; t < nk; ++t) run_tile2(t, F_{}, F_{});
    } else {
      run_tile(0, F_{}, T_{});
      for (; t + 2 < nk; ++t) run_tile(t, T_{}, F_{});
      for (; t < nk; ++t) run_tile(t, F_{}, F_{});
    }
    if (wm == 0) g8_barrier();   // balance group 1's extra barrier: every wave's LDS reads are done

    ++round;
    const int next = g8p_tile(b, round, G, n_tiles);
    if (next >= 0) {
      ep_issue(next, slot ^ 1);
      setup(next);
      prologue();
    }
    if constexpr (DBG == 2 || DBG == 4 || DBG == 5) {   // (DBG 6, 7: the library epilogue)
      #pragma unroll
      for (int a = 0; a < 2; ++a)
        #pragma unroll
        for (int c = 0; c < 2; ++c)
          #pragma unroll
          for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(acc[a][c][i][0]), "v"(acc[a][c][i][1]));
    } else {
      g8p_epilogue<ACT, CT3, F16, has_bias, fold, DBG, FNT>(g, acc, m0, n0, wm, wn, q, r16,
                                                           smem + G8_OPS + slot * G8P_EP);
    }
    if (next < 0) break;
    slot ^= 1;
    S = DBG == 1 || DBG == 2 || DBG == 4 || DBG == 5 ? 0 : (m0 + 256 <= M ? s_full : 0);
    tile = next;
  }
}

// ======================================================================================
// Residual GEMMs (C = A B^T + bias + LN?(resid), fp32 out, optional bf16 copy and LayerNorm
// partials of the output rows): one tile per block, the persistent kernel's 8-phase main loop,
// then a register-direct epilogue (acc holds C^T blocks) whose loads all precede its first store:
//   1. LDS-DMA of the epilogue parameters into the (now free) operand LDS: bias, rln_w, rln_b
//      (1 KiB each) and the residual rows' LayerNorm partials [256][3] (6 KiB);
//   2. the residual rows of half 0 (16 x 16 B per lane) -- in flight together with the DMA;
//   3. half 0 finished in registers, THEN half 1's residual loads, THEN half 0's stores: the wait
//      for half 1 never includes a store (vector-memory ops retire in issue order).
// LayerNorm partials of the written rows (OPART, the folded post-LN path): per row, each wave
// reduces its 64 columns (16 in-lane values, lanes q = 0..3) to (mean_c, M2_c), the 4 waves' chunks
// meet in LDS and one thread per row combines them (Chan) into the 256-column (mean_t, M2_t).
// LDS of gemm8r_kernel<RB = true>: operands (2 x 64 KiB) | epilogue parameters | row-chunk statistics
constexpr int G8R_PAR = G8_OPS;                  // [0, 1K) bias | [1K, 2K) rln_w | [2K, 3K) rln_b | [3K, 9K) partials
constexpr int G8R_CST = G8_OPS + 9 * 1024;       // [2 halves][128 rows][4 waves] float2
constexpr int G8R_SMEM_RB = G8R_CST + 8 * 1024;

// Epilogue of gemm8r_kernel<RB = true> (below): o = acc + bias + LN?(resid) rounded to the 16-bit stream type, the
// out-partials of the written rows (OPART), stores through per-16-row-block buffer resources.  The residual rows and
// the parameters are in LDS (see gemm8r_kernel); half 1's residual DMA is in flight on entry.
// DBG (probes only): 5 = no stores (results kept live), 6 = no out-partials, 7 = no math (raw accumulators stored)
template <bool LN, bool OPART_, bool F16, int DBG, typename ResDma>
SSE_DEV void g8r_epilogue_rb(const GemmArgs& g, f32x4 (&acc)[2][2][4][2], char* smem, int m0, int n0, int wm, int wn,
                             int q, int r16, int nk, bool has_bias, ResDma&& res_dma) {
  constexpr bool OPART = OPART_ && DBG != 6;
  const int M = g.M;
  res_dma(1, (nk - 1) & 1);                         // every read of that buffer is done (the barrier before)
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // parameters and half 0 landed; half 1's 8 pieces in flight
  __syncthreads();
  float2* cst = (float2*)(smem + G8R_CST);
  const char* par = smem + G8R_PAR;
  // 16-B store-layout chunk of (i, ni): columns ni*128 + wn*32 + (q&1)*16 + (q>>1)*8 .. +7 = logical chunk c
  const int cl = wn * 4 + (q & 1) * 2 + (q >> 1);
  auto finish_half = [&](int mi) {
    if constexpr (DBG == 7) return;
    // compiler memory barrier: the column parameters are re-read from LDS per half
    asm volatile("" ::: "memory");
    const char* rb = smem + (mi ? (nk - 1) & 1 : nk & 1) * G8_BUF;
    f32x4 rv[4][2][2];
    #pragma unroll
    for (int i = 0; i < 4; ++i)
      #pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const int row = wm * 64 + i * 16 + r16;   // row & 15 == r16
        const uint4 v = *(const uint4*)(rb + row * 512 + ((ni * 16 + (cl ^ r16)) << 4));
        const auto x = __builtin_amdgcn_permlane16_swap(v.x, v.z, false, false);
        const auto y = __builtin_amdgcn_permlane16_swap(v.y, v.w, false, false);
        rv[i][ni][0] = unpack_h4<F16>(make_uint2(x[0], y[0]));   // bf16, or fp16 (h16 path)
        rv[i][ni][1] = unpack_h4<F16>(make_uint2(x[1], y[1]));
      }
    // the four row blocks' statistics side by side: four independent chains through every step (one row block
    // at a time, the sum -> two lane-group swaps -> mean -> 16-long dependent M2 fma chain -> two swaps was
    // latency-bound: 8.3 of the oproj launch's 25 us of epilogue, round-5 probe)
    float sum[4];
    #pragma unroll
    for (int i = 0; i < 4; ++i) {
      float2 st = make_float2(0.f, 1.f);
      if constexpr (LN) {
        const float2* p = (const float2*)(par + 3072) + (mi * 128 + wm * 64 + i * 16 + r16) * 3;
        const float2 v[3] = {p[0], p[1], p[2]};
        st = ln_part_combine<3>(v, g.ln_eps);
      }
      float sp[4];
      #pragma unroll
      for (int ni = 0; ni < 2; ++ni)
        #pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int c = ni * 128 + wn * 32 + j * 16 + q * 4;
          f32x4 r = rv[i][ni][j];
          if constexpr (LN) {   // LayerNorm of the residual, the exact expression of layernorm_kernel
            const f32x4 lw = *(const f32x4*)(par + 1024 + c * 4), lb = *(const f32x4*)(par + 2048 + c * 4);
            #pragma unroll
            for (int e = 0; e < 4; ++e) r[e] = fmaf((r[e] - st.x) * st.y, lw[e], lb[e]);
          }
          const f32x4 bvv = *(const f32x4*)(par + c * 4);
          const f32x4 bv = has_bias ? bvv : f32x4{0.f, 0.f, 0.f, 0.f};
          f32x4 o = (acc[mi][ni][i][j] + bv) + r;
          #pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = round_h<F16>(o[e]);   // the statistics describe the rounded values
          acc[mi][ni][i][j] = o;
          sp[ni * 2 + j] = (o[0] + o[1]) + (o[2] + o[3]);
        }
      sum[i] = (sp[0] + sp[1]) + (sp[2] + sp[3]);
    }
    if constexpr (OPART) {   // this wave's 64 columns of each row: lanes r16 + 16q (sums over q by lane-group swaps)
      auto qsum4 = [](float (&v)[4]) {
        #pragma unroll
        for (int i = 0; i < 4; ++i) {
          const auto t = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[i]), __float_as_uint(v[i]), false, false);
          v[i] = __uint_as_float(t[0]) + __uint_as_float(t[1]);
        }
        #pragma unroll
        for (int i = 0; i < 4; ++i) {
          const auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[i]), __float_as_uint(v[i]), false, false);
          v[i] = __uint_as_float(t[0]) + __uint_as_float(t[1]);
        }
      };
      qsum4(sum);
      float m2[4];
      #pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float mc = sum[i] * (1.0f / 64.0f);
        float p[4];
        #pragma unroll
        for (int u = 0; u < 4; ++u) {
          const f32x4 d = acc[mi][u >> 1][i][u & 1] - mc;
          p[u] = fmaf(d[3], d[3], fmaf(d[2], d[2], fmaf(d[1], d[1], d[0] * d[0])));
        }
        m2[i] = (p[0] + p[1]) + (p[2] + p[3]);
        sum[i] = mc;
      }
      qsum4(m2);
      if (q == 0) {
        #pragma unroll
        for (int i = 0; i < 4; ++i) cst[(mi * 128 + wm * 64 + i * 16 + r16) * 4 + wn] = make_float2(sum[i], m2[i]);
      }
    }
  };
  // one resource per 16-row block based at (m0 + mi*128 + 16 i, n0), num_records ending at row M: rows >= M dropped
  const unsigned lane_off = (unsigned)(((wm * 64 + r16) * g.ldc + wn * 32 + (q & 1) * 16 + (q >> 1) * 8) * 2);
  auto store_half = [&](int mi) {
    #pragma unroll
    for (int i = 0; i < 4; ++i) {
      const long long r0 = (long long)m0 + mi * 128 + 16 * i, rows = (long long)M - r0;
      const long long nrec = rows > 0 ? (rows * g.ldc - n0) * 2 : 0;
      const __amdgpu_buffer_rsrc_t cr = __builtin_amdgcn_make_buffer_rsrc(
          (void*)((bf16*)g.Ct + (rows > 0 ? r0 * g.ldc + n0 : 0)), (short)0, (int)min(nrec, (long long)0x7FFFFFF0),
          0x00020000);
      #pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const uint2 X = pack_h4<F16>(acc[mi][ni][i][0]), Y = pack_h4<F16>(acc[mi][ni][i][1]);
        const auto s0 = __builtin_amdgcn_permlane16_swap(X.x, Y.x, false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(X.y, Y.y, false, false);
        if constexpr (DBG == 5) {
          asm volatile("" ::"v"(s0[0]), "v"(s0[1]), "v"(s1[0]), "v"(s1[1]));
          continue;
        }
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{s0[0], s1[0], s0[1], s1[1]}, cr, lane_off + (unsigned)(ni * 256), 0u, 0);
      }
    }
  };
  finish_half(0);
  __builtin_amdgcn_sched_barrier(0);
  store_half(0);
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (DBG == 5) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // half 1's residual landed (younger: half 0's 8 stores)
  __syncthreads();
  finish_half(1);
  __builtin_amdgcn_sched_barrier(0);
  store_half(1);
  if constexpr (OPART) {
    __syncthreads();
    if (threadIdx.x < 256) {
      const int r = threadIdx.x, m = m0 + r;
      const float2* c = cst + r * 4;
      const float2 c0 = c[0], c1 = c[1], c2 = c[2], c3 = c[3];
      const float mean = 0.25f * ((c0.x + c1.x) + (c2.x + c3.x));
      const float d0 = c0.x - mean, d1 = c1.x - mean, d2 = c2.x - mean, d3 = c3.x - mean;
      const float m2 = ((c0.y + c1.y) + (c2.y + c3.y)) + 64.f * ((d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3));
      if (m < M) g.opart[(long long)m * (g.N >> 8) + (n0 >> 8)] = make_float2(mean, m2);
    }
  }
}

// RB (the 16-bit residual stream, round 5): the epilogue no longer waits on global memory after the main loop --
//   1. its parameters (bias, rln_w, rln_b: 1 KiB each; the residual rows' LayerNorm partials [256][3]: 6 KiB) go
//      into LDS by DMA at kernel START, before the operand prologue (retired by the first counted wait);
//   2. the residual rows of half 0 (128 x 256 16-bit = 64 KiB, 8 DMA pieces per wave) are DMA'd during the LAST
//      K-tile into the operand buffer K-tile nk - 2 used (free: its last reads precede that K-tile's phase-2
//      barrier), half 1 into the other buffer right after the main loop; both images are swizzled on the source
//      side (16-B chunk c of row r at chunk c ^ (r & 15)) so the store-layout ds_read_b128 of 16 rows is
//      conflict-free;
//   3. the row-block stores go through a buffer resource per 16-row block (rows >= M dropped by its range check),
//      the cross-lane sums of the out-partials through v_permlane16/32_swap instead of ds_bpermute.
// Probe (tools/gemm8_probe.hip, oproj 38144 x 768 x 768, round 5 before the change): 65.9 us per launch against
// 37.3 with no epilogue; 7.8 of the 28.6 us were the residual loads, 2.6 the parameter wait.
// DBG (timing probes only, tools/gemm8_probe.hip; the library launches DBG = 0): 2 = no epilogue (accumulators
// kept live).
// PH2: the two-phase K-tile schedule (gemm8p_kernel's template comment; the default, option gemm_4phase = 1 keeps four)
template <bool LN, bool OPART, bool RB, bool F16 = false, int DBG = 0, bool PH2 = false>
__global__ __launch_bounds__(512) void gemm8r_kernel(GemmArgs g) {
  // RB: operands | epilogue parameters (9 KiB, staged at kernel start) | row-chunk statistics (8 KiB)
  __shared__ __attribute__((aligned(16))) char smem[RB ? G8R_SMEM_RB : G8_OPS];   // the ONLY shared object
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int q = lane >> 4, r16 = lane & 15;
  const int M = g.M, K = g.K;
  const int n_tiles_n = g.N / 256;
  const int nk = K / 64;
  int bid = blockIdx.x;
  {   // XCD-aware bijective remap (as gemm8_kernel)
    const int nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, x = bid % 8;
    bid = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + bid / 8;
  }
  const int m0 = (bid / n_tiles_n) * 256, n0 = (bid % n_tiles_n) * 256;

  constexpr int NREC = 0x7FFFFFF0;
  __amdgpu_buffer_rsrc_t a_rsrc, b_rsrc;
  unsigned a_voff[2][2], b_voff[2][2];
  {
    const int mf = m0 < M ? m0 : M - 1;
    const int seg0 = mf / g.rows_per_seg, rr0 = mf - seg0 * g.rows_per_seg;
    const long long a_base = ((long long)seg0 * g.seg_stride + (long long)rr0 * g.lda) * 2;
    a_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)g.A + a_base), (short)0, NREC, 0x00020000);
    b_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)g.B + (long long)n0 * K * 2), (short)0, NREC,
                                               0x00020000);
    #pragma unroll
    for (int h = 0; h < 2; ++h)
      #pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int row = h * 128 + (wave + 8 * s) * 8 + (lane >> 3);
        const int ch = (lane & 7) ^ ((row >> 1) & 7);
        int m = m0 + row;
        m = m < M ? m : M - 1;
        const int seg = m / g.rows_per_seg, rr = m - seg * g.rows_per_seg;
        const long long el = ((long long)seg * g.seg_stride + (long long)rr * g.lda) * 2 + ch * 16;
        a_voff[h][s] = (unsigned)(el - a_base);
        b_voff[h][s] = (unsigned)((long long)row * K * 2 + ch * 16);
      }
  }
  auto issue_half = [&](int tl, int half) {
    char* dst = smem + (tl & 1) * G8_BUF + half * G8_HALF;
    const unsigned soff = (unsigned)tl * 128u;
    if (half < 2) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, LPTR(dst + wave * 1024), 16, a_voff[half][0], soff, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, LPTR(dst + (wave + 8) * 1024), 16, a_voff[half][1], soff, 0, 0);
    } else {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, LPTR(dst + wave * 1024), 16, b_voff[half - 2][0], soff, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, LPTR(dst + (wave + 8) * 1024), 16, b_voff[half - 2][1], soff, 0,
                                               0);
    }
  };
  auto issue = [&](int k) {
    if (k < -6) return;
    int tl, half;
    g8_target(k, tl, half);
    if (tl >= nk) return;
    issue_half(tl, half);
  };
  f32x4 acc[2][2][4][2];
  #pragma unroll
  for (int a = 0; a < 2; ++a)
    #pragma unroll
    for (int c = 0; c < 2; ++c)
      #pragma unroll
      for (int i = 0; i < 4; ++i)
        #pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][c][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[4][2], b0f[2][2], b1f[2][2];
  auto read_a = [&](const char* hb) {
    #pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + i * 16 + r16;
      #pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        af[i][ks] = *(const bf16x8*)(hb + row * 128 + (((q + 4 * ks) ^ ((row >> 1) & 7)) * 16));
    }
  };
  auto read_b = [&](const char* hb, bf16x8 (&bf)[2][2]) {
    #pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = wn * 32 + j * 16 + r16;
      #pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        bf[j][ks] = *(const bf16x8*)(hb + row * 128 + (((q + 4 * ks) ^ ((row >> 1) & 7)) * 16));
    }
  };
  auto mma = [&](f32x4 (&c)[4][2], const bf16x8 (&bf)[2][2]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    #pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      #pragma unroll
      for (int i = 0; i < 4; ++i)
        #pragma unroll
        for (int j = 0; j < 2; ++j) c[i][j] = g8_mfma<F16>(bf[j][ks], af[i][ks], c[i][j]);
    __builtin_amdgcn_sched_barrier(0);
  };
  const bool has_bias = g.bias != nullptr;
  // RB: epilogue parameters into LDS before the prologue (wave w < 6: partials piece w; 6: bias; 7: rln_w, rln_b)
  if constexpr (RB) {
    __amdgpu_buffer_rsrc_t r;
    unsigned soff = 0;
    int off = 0;
    bool go = true;
    if (wave < 6) {
      go = LN;
      r = __builtin_amdgcn_make_buffer_rsrc((void*)(LN ? (const void*)g.rpart : g.zero), (short)0, LN ? M * 24 : 0,
                                            0x00020000);
      soff = (unsigned)(m0 * 24 + wave * 1024);
      off = 3072 + wave * 1024;
    } else if (wave == 6) {
      go = has_bias;
      r = __builtin_amdgcn_make_buffer_rsrc((void*)(has_bias ? (const void*)g.bias : g.zero), (short)0,
                                            has_bias ? g.N * 4 : 0, 0x00020000);
      soff = (unsigned)(n0 * 4);
    } else {
      go = LN;
      r = __builtin_amdgcn_make_buffer_rsrc((void*)(LN ? (const void*)g.rln_w : g.zero), (short)0, LN ? g.N * 4 : 0,
                                            0x00020000);
      soff = (unsigned)(n0 * 4);
      off = 1024;
    }
    if (go) __builtin_amdgcn_raw_ptr_buffer_load_lds(r, LPTR(smem + G8R_PAR + off), 16, (unsigned)lane * 16u, soff, 0, 0);
    if (LN && wave == 7) {
      r = __builtin_amdgcn_make_buffer_rsrc((void*)g.rln_b, (short)0, g.N * 4, 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, LPTR(smem + G8R_PAR + 2048), 16, (unsigned)lane * 16u, soff, 0, 0);
    }
  }
  // RB: residual rows of half mi (128 x 256 16-bit values, 512 B per row) into the 64 KiB operand buffer `dst`:
  // wave w's piece e (1 KiB) holds rows 2u, 2u + 1 (u = 8w + e); lane l writes 16-B chunk l & 31 of row
  // 2u + (l >> 5), which holds logical chunk (l & 31) ^ (row & 15).  Rows >= M read as zeros (never stored).
  auto res_dma = [&](int mi, int buf) {
    if constexpr (RB) {
      const long long r0 = (long long)m0 + mi * 128, rows = (long long)M - r0;
      const long long nrec = rows > 0 ? (rows * g.ldc - n0) * 2 : 0;
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(g.resid_t + (rows > 0 ? r0 * g.ldc + n0 : 0)), (short)0, (int)min(nrec, (long long)0x7FFFFFF0),
          0x00020000);
      #pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int u = wave * 8 + e, row = 2 * u + (lane >> 5), c = (lane & 31) ^ (row & 15);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rr, LPTR(smem + buf * G8_BUF + u * 1024), 16,
                                                 (unsigned)((row * g.ldc + c * 8) * 2), 0u, 0, 0);
      }
    }
  };
  if constexpr (PH2) {
    for (int j = -3; j < 0; ++j) g8_issue2(j, nk, issue_half);
    g8_vmcnt_dyn<false>(g8_count2(-1, nk));
  } else {
    for (int k = -6; k < 0; ++k) issue(k);
    g8_wait<false>(-1, nk);
  }
  g8_barrier();
  if (wm == 1) g8_barrier();   // group 1 runs one barrier behind
  // PH2: the K-tile in two phases of 32 MFMAs (same accumulation order per accumulator: bit-identical)
  auto run_tile2 = [&](int t, auto steady) {
    constexpr bool ST = decltype(steady)::value;
    const char* buf = smem + (t & 1) * G8_BUF;
    const int j = 2 * t;
    const int xr = (RB && !ST && t == nk - 1) ? 8 : 0;
    if (xr) res_dma(0, nk & 1);
    auto issue_wait = [&](int jj) {
      g8_issue2(jj, nk, issue_half);
      if constexpr (ST) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else g8_vmcnt_dyn<false>(g8_count2(jj, nk) + xr);
    };
    read_a(buf);
    read_b(buf + 2 * G8_HALF, b0f);
    read_b(buf + 3 * G8_HALF, b1f);
    issue_wait(j);
    g8_barrier();
    mma(acc[0][0], b0f);
    mma(acc[0][1], b1f);
    g8_barrier();
    read_a(buf + G8_HALF);
    issue_wait(j + 1);
    g8_barrier();
    mma(acc[1][1], b1f);
    mma(acc[1][0], b0f);
    g8_barrier();
  };
  auto run_tile = [&](int t, auto steady) {
    constexpr bool ST = decltype(steady)::value;
    const char* buf = smem + (t & 1) * G8_BUF;
    const int k = 4 * t;
    // RB, last K-tile: half 0's residual rows go out in phase 0 (the tail waits leave those 8 in flight)
    const int xr = (RB && !ST && t == nk - 1) ? 8 : 0;
    if (xr) res_dma(0, nk & 1);
    auto issue_wait = [&](int kk) {
      issue(kk);
      if constexpr (ST) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else g8_vmcnt_dyn<false>(g8_count<false>(kk, nk) + xr);
    };
    read_a(buf);
    read_b(buf + 2 * G8_HALF, b0f);
    issue_wait(k);
    g8_barrier();
    mma(acc[0][0], b0f);
    g8_barrier();
    read_b(buf + 3 * G8_HALF, b1f);
    issue_wait(k + 1);
    g8_barrier();
    mma(acc[0][1], b1f);
    g8_barrier();
    read_a(buf + G8_HALF);
    issue_wait(k + 2);
    g8_barrier();
    mma(acc[1][1], b1f);
    g8_barrier();
    issue_wait(k + 3);
    g8_barrier();
    mma(acc[1][0], b0f);
    g8_barrier();
  };
  int t = 0;
  if constexpr (PH2) {
    for (; t + 2 < nk; ++t) run_tile2(t, std::integral_constant<bool, true>{});
    for (; t < nk; ++t) run_tile2(t, std::integral_constant<bool, false>{});
  } else {
    for (; t + 2 < nk; ++t) run_tile(t, std::integral_constant<bool, true>{});
    for (; t < nk; ++t) run_tile(t, std::integral_constant<bool, false>{});
  }
  if (wm == 0) g8_barrier();   // balance group 1's extra barrier: every wave's LDS reads are done
  if constexpr (RB) {
    if constexpr (DBG == 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      #pragma unroll
      for (int a = 0; a < 2; ++a)
        #pragma unroll
        for (int c = 0; c < 2; ++c)
          #pragma unroll
          for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(acc[a][c][i][0]), "v"(acc[a][c][i][1]));
      return;
    }
    g8r_epilogue_rb<LN, OPART, F16, DBG>(g, acc, smem, m0, n0, wm, wn, q, r16, nk, has_bias, res_dma);
    return;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (DBG == 2) {
    #pragma unroll
    for (int a = 0; a < 2; ++a)
      #pragma unroll
      for (int c = 0; c < 2; ++c)
        #pragma unroll
        for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(acc[a][c][i][0]), "v"(acc[a][c][i][1]));
    return;
  }

  // ---- epilogue ----
  // LDS (operand area, free now): [0, 1K) bias | [1K, 2K) rln_w | [2K, 3K) rln_b | [3K, 9K) partials
  // [256][3] | [16K, 24K) chunk statistics [2 halves][128 rows][4 waves] float2
  {
    __amdgpu_buffer_rsrc_t r;
    unsigned soff = 0;
    int off = 0;
    bool go = true;
    if (wave < 6) {
      go = LN;
      r = __builtin_amdgcn_make_buffer_rsrc((void*)(LN ? (const void*)g.rpart : g.zero), (short)0, LN ? M * 24 : 0,
                                            0x00020000);
      soff = (unsigned)(m0 * 24 + wave * 1024);
      off = 3072 + wave * 1024;
    } else if (wave == 6) {
      go = has_bias;
      r = __builtin_amdgcn_make_buffer_rsrc((void*)(has_bias ? (const void*)g.bias : g.zero), (short)0,
                                            has_bias ? g.N * 4 : 0, 0x00020000);
      soff = (unsigned)(n0 * 4);
    } else {
      go = LN;
      r = __builtin_amdgcn_make_buffer_rsrc((void*)(LN ? (const void*)g.rln_w : g.zero), (short)0, LN ? g.N * 4 : 0,
                                            0x00020000);
      soff = (unsigned)(n0 * 4);
      off = 1024;
    }
    if (go) __builtin_amdgcn_raw_ptr_buffer_load_lds(r, LPTR(smem + off), 16, (unsigned)lane * 16u, soff, 0, 0);
    if (LN && wave == 7) {
      r = __builtin_amdgcn_make_buffer_rsrc((void*)g.rln_b, (short)0, g.N * 4, 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, LPTR(smem + 2048), 16, (unsigned)lane * 16u, soff, 0, 0);
    }
  }
  // RB: the bf16 residual is read in the store layout (8 consecutive columns per lane, one 16-B load
  // per (i, ni)) and redistributed with the inverse v_permlane16_swap
  f32x4 rv[4][2][2];
  uint4 rvb[4][2];
  auto load_half = [&](int mi) {
    if constexpr (DBG == 3) {
      #pragma unroll
      for (int i = 0; i < 4; ++i)
        #pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
          int z = 0;
          asm volatile("v_mov_b32 %0, 0" : "=v"(z));
          rvb[i][ni] = make_uint4(z, z, z, z);
          rv[i][ni][0] = rv[i][ni][1] = f32x4{(float)z, (float)z, (float)z, (float)z};
        }
      return;
    }
    #pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + mi * 128 + wm * 64 + i * 16 + r16;
      const int mc = m < M ? m : 0;
      const long long rrow = g.resid_rows ? (long long)(mc % g.resid_rows) * g.ldc : (long long)mc * g.ldc;
      #pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        if constexpr (RB) {
          rvb[i][ni] = *(const uint4*)(g.resid_t + rrow + n0 + ni * 128 + wn * 32 + (q & 1) * 16 + (q >> 1) * 8);
        } else {
          #pragma unroll
          for (int j = 0; j < 2; ++j)
            rv[i][ni][j] = *(const f32x4*)(g.resid + rrow + n0 + ni * 128 + wn * 32 + j * 16 + q * 4);
        }
      }
    }
  };
  auto unpack_half = [&]() {   // RB: rvb -> rv (columns j*16 + q*4 .. +3 of each (i, ni))
    if constexpr (RB) {
      #pragma unroll
      for (int i = 0; i < 4; ++i)
        #pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
          const uint4 v = rvb[i][ni];
          const auto x = __builtin_amdgcn_permlane16_swap(v.x, v.z, false, false);
          const auto y = __builtin_amdgcn_permlane16_swap(v.y, v.w, false, false);
          rv[i][ni][0] = unpack_h4<F16>(make_uint2(x[0], y[0]));   // bf16, or fp16 (h16 path)
          rv[i][ni][1] = unpack_h4<F16>(make_uint2(x[1], y[1]));
        }
    }
  };
  __builtin_amdgcn_sched_barrier(0);
  load_half(0);
  if constexpr (DBG != 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // parameter DMA (and half 0's rows) landed
  __syncthreads();
  __builtin_amdgcn_sched_barrier(0);
  // column parameters are read from LDS where they are used (registers hold acc + one half's rows)
  float2* cst = (float2*)(smem + 16384);
  auto finish_half = [&](int mi) {
    // compiler memory barrier: the column parameters are re-read from LDS per half (without it the
    // second half's reads are merged with the first's and held live across the stores: spills)
    asm volatile("" ::: "memory");
    unpack_half();
    #pragma unroll
    for (int i = 0; i < 4; ++i) {
      float2 st = make_float2(0.f, 1.f);
      if constexpr (LN) {
        const float2* p = (const float2*)(smem + 3072) + (mi * 128 + wm * 64 + i * 16 + r16) * 3;
        const float2 v[3] = {p[0], p[1], p[2]};
        st = ln_part_combine<3>(v, g.ln_eps);
      }
      float sum = 0.f;
      #pragma unroll
      for (int ni = 0; ni < 2; ++ni)
        #pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int c = ni * 128 + wn * 32 + j * 16 + q * 4;
          f32x4 r = rv[i][ni][j];
          if constexpr (LN) {   // LayerNorm of the residual, the exact expression of layernorm_kernel
            const f32x4 lw = *(const f32x4*)(smem + 1024 + c * 4), lb = *(const f32x4*)(smem + 2048 + c * 4);
            #pragma unroll
            for (int e = 0; e < 4; ++e) r[e] = fmaf((r[e] - st.x) * st.y, lw[e], lb[e]);
          }
          const f32x4 bvv = *(const f32x4*)(smem + c * 4);
          const f32x4 bv = has_bias ? bvv : f32x4{0.f, 0.f, 0.f, 0.f};
          f32x4 o = ((F16 ? acc[mi][ni][i][j] * g.alpha : acc[mi][ni][i][j]) + bv) + r;
          if constexpr (RB) {   // 16-bit output: the statistics describe the rounded values
            #pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = round_h<F16>(o[e]);
          }
          acc[mi][ni][i][j] = o;
          sum += (o[0] + o[1]) + (o[2] + o[3]);
        }
      if constexpr (OPART) {   // this wave's 64 columns of the row: lanes r16 + 16q
        sum += __shfl_xor(sum, 16, 64);
        sum += __shfl_xor(sum, 32, 64);
        const float mc = sum * (1.0f / 64.0f);
        float m2 = 0.f;
        #pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          #pragma unroll
          for (int j = 0; j < 2; ++j)
            #pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float d = acc[mi][ni][i][j][e] - mc;
              m2 = fmaf(d, d, m2);
            }
        m2 += __shfl_xor(m2, 16, 64);
        m2 += __shfl_xor(m2, 32, 64);
        if (q == 0) cst[(mi * 128 + wm * 64 + i * 16 + r16) * 4 + wn] = make_float2(mc, m2);
      }
    }
  };
  auto store_half = [&](int mi) {
    #pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + mi * 128 + wm * 64 + i * 16 + r16;
      const bool ok = m < M;
      const long long row = (long long)(ok ? m : 0) * g.ldc;
      #pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        if (!RB && ok) {
          #pragma unroll
          for (int j = 0; j < 2; ++j)
            *(f32x4*)(g.Cf + row + n0 + ni * 128 + wn * 32 + j * 16 + q * 4) = acc[mi][ni][i][j];
        }
        if (RB || g.Ct) {
          const uint2 X = pack_h4<F16>(acc[mi][ni][i][0]), Y = pack_h4<F16>(acc[mi][ni][i][1]);
          const auto s0 = __builtin_amdgcn_permlane16_swap(X.x, Y.x, false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(X.y, Y.y, false, false);
          if (ok) {
            const uint4 v = make_uint4(s0[0], s1[0], s0[1], s1[1]);
            *(uint4*)((bf16*)g.Ct + row + n0 + ni * 128 + wn * 32 + (q & 1) * 16 + (q >> 1) * 8) = v;
          }
        }
      }
    }
  };
  // sched_barriers keep the phases in this order (the register budget holds one half's rows)
  finish_half(0);
  __builtin_amdgcn_sched_barrier(0);
  load_half(1);   // before the first store
  __builtin_amdgcn_sched_barrier(0);
  store_half(0);
  __builtin_amdgcn_sched_barrier(0);
  finish_half(1);
  __builtin_amdgcn_sched_barrier(0);
  store_half(1);
  if constexpr (OPART) {
    __syncthreads();
    if (threadIdx.x < 256) {
      const int r = threadIdx.x, m = m0 + r;
      const float2* c = cst + r * 4;
      const float2 c0 = c[0], c1 = c[1], c2 = c[2], c3 = c[3];
      const float mean = 0.25f * ((c0.x + c1.x) + (c2.x + c3.x));
      const float d0 = c0.x - mean, d1 = c1.x - mean, d2 = c2.x - mean, d3 = c3.x - mean;
      const float m2 = ((c0.y + c1.y) + (c2.y + c3.y)) + 64.f * ((d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3));
      if (m < M) g.opart[(long long)m * n_tiles_n + (n0 >> 8)] = make_float2(mean, m2);
    }
  }
}

// the residual GEMM in the schedule the options select: two phases per K-tile unless gemm_4phase = 1 (Whisper-large-v2
// bf16 fc2 32.4 -> 31.5, WavLM-large fc2 7.22 -> 7.03 ms/step; at WavLM-base's N = 768 one box measured fc2 1.5 %
// slower, another 2.7 % faster and oproj 1.2 % faster: profiles/r6_ab_gemm_2phase_all.txt, r6_ab_gemm_2phase_residual.txt,
// r6_ab_gemm_2phase_residual_n768.txt)
template <bool LN, bool OP, bool RB, bool F16 = false>
void launch_g8r(dim3 grid, hipStream_t s, const GemmArgs& a) {
  if (sse_opt(OPT_GEMM_4PHASE) == 1)
    hipLaunchKernelGGL((gemm8r_kernel<LN, OP, RB, F16, 0, false>), grid, dim3(512), 0, s, a);
  else
    hipLaunchKernelGGL((gemm8r_kernel<LN, OP, RB, F16, 0, true>), grid, dim3(512), 0, s, a);
}

// the MX GEMM in the schedule the options select (two phases per K-tile unless gemm_4phase = 1)
template <bool TR, int MXE = 0>
void launch_g8mx(dim3 grid, hipStream_t s, const GemmArgs& a) {
  if (sse_opt(OPT_GEMM_4PHASE) == 1)
    hipLaunchKernelGGL((gemm8_kernel<0, TR, false, true, MXE, false>), grid, dim3(512), 0, s, a);
  else
    hipLaunchKernelGGL((gemm8_kernel<0, TR, false, true, MXE, true>), grid, dim3(512), 0, s, a);
}

}  // namespace

int launch_gemm8_bf16(const GemmArgs& a, hipStream_t s) {
  if (a.M <= 0 || a.N % 256 || a.K % 64 || a.K <= 0) return -3;
  // folded-LayerNorm partials: rows of 3..5 column tiles (H = 768 .. 1280; the residual LayerNorm on the
  // load, rpart, 3 only); opart tiles = N / 256
  if ((a.apart && (a.apart_nt < 3 || a.apart_nt > 5)) || (a.rpart && a.rpart_nt != 3) ||
      (a.opart && (a.N < 768 || a.N > 1280)) || (a.apart && !a.bias && a.apart_nt != 3))
    return -3;
  // the FNT = 4 / 5 fold kernels are instantiated for the plain bf16 persistent GEMM only: an fp16 or split
  // fold with 4-5 partials per row would otherwise run the FNT = 3 kernel and read the partials wrongly
  if (a.apart && a.apart_nt != 3 && (a.h16 || a.f16 || a.ct3)) return -3;
  dim3 grid((unsigned)(((a.M + 255) / 256) * (a.N / 256)));
  // OPT_GEMM_NONPERSIST (tests, A/B): the non-persistent LDS-staged kernel for every shape
  if (a.ct3 && (a.resid || a.resid_t || !a.Ct || !a.f16)) return -3;   // split output: persistent kernel only
  if (a.f16) {
    // split-fp16 (SSE_DTYPE_FP16X3): residual GEMMs (fp32 out), ct3 + GELU, or plain fp32 out
    if (a.resid_t || a.rstats || a.rpart || a.opart || a.apart || a.resid_rows || a.alpha == 0.f) return -3;
    if (a.resid) {
      if (!a.Cf || a.Ct) return -3;
      launch_g8r<false, false, false, true>(grid, s, a);
      return hipGetLastError() == hipSuccess ? 0 : -2;
    }
    if (a.ct3 ? (a.act != ACT_GELU || a.Cf) : (a.act != ACT_NONE || !a.Cf || a.Ct)) return -3;
  }
  if (a.h16) {
    // plain fp16 (SSE_DTYPE_FP16): the bf16 path's kernels with fp16 operands (F16 = true, alpha = 1,
    // no split planes); the folded post-LN flow (fp16 residual stream) or non-residual persistent GEMMs
    if (a.f16 || a.ct3 || a.resid || a.rstats || a.resid_rows || a.alpha != 1.f) return -3;
    if (a.resid_t) {
      if (!a.Ct || a.Cf) return -3;
      if (a.rpart) {
        if (a.opart) launch_g8r<true, true, true, true>(grid, s, a);
        else launch_g8r<true, false, true, true>(grid, s, a);
      } else {
        if (a.opart) launch_g8r<false, true, true, true>(grid, s, a);
        else launch_g8r<false, false, true, true>(grid, s, a);
      }
      return hipGetLastError() == hipSuccess ? 0 : -2;
    }
  }
  // (a bf16 GELU_FAST GEMM with an fp32 copy too: the persistent kernel's bf16 GELU is the degree-6 form)
  if ((sse_opt(OPT_GEMM_NONPERSIST) || (a.act == ACT_GELU_FAST && a.Cf && !a.resid && !a.resid_t)) && !a.resid_t &&
      !a.f16 && !a.h16) {
    hipLaunchKernelGGL((gemm8_kernel<0, false, false>), grid, dim3(512), 0, s, a);
  } else if (a.resid_t) {
    // bf16 residual stream (folded post-LN path): bf16 out only
    if (!a.Ct || a.Cf || a.resid || a.resid_rows || a.rstats) return -3;
    if (a.rpart) {
      if (a.opart) launch_g8r<true, true, true>(grid, s, a);
      else launch_g8r<true, false, true>(grid, s, a);
    } else {
      if (a.opart) launch_g8r<false, true, true>(grid, s, a);
      else launch_g8r<false, false, true>(grid, s, a);
    }
  } else if (a.resid) {
    // residual GEMMs: fp32 out (Cf) required; the rstats form is the staged kernel's only
    if (!a.Cf || a.rstats || (a.opart && !a.rpart && a.rln_w)) {
      hipLaunchKernelGGL((gemm8_kernel<0, false, false>), grid, dim3(512), 0, s, a);
    } else if (a.rpart) {
      if (a.opart) launch_g8r<true, true, false>(grid, s, a);
      else launch_g8r<true, false, false>(grid, s, a);
    } else {
      if (a.opart) launch_g8r<false, true, false>(grid, s, a);
      else launch_g8r<false, false, false>(grid, s, a);
    }
  } else {
    // persistent: one block per CU (LDS-bound), at most one per tile
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -2;
    if (!cus[dev] && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return -2;
    const int n_tiles = (int)grid.x;
    const int ncu = sse_stream_cus(s, cus[dev]);   // a CU-masked stream's own CUs
    const int G = n_tiles < ncu ? n_tiles : ncu;
    const int ep = (a.bias ? 1 : 0) | (a.apart ? 2 : 0);
    const bool ph2 = sse_opt(OPT_GEMM_4PHASE) != 1;   // two phases per K-tile (round 6 default)
    auto go2 = [&](auto act, auto ct3, auto f16, auto p2) {
      constexpr int AC = decltype(act)::value;
      constexpr bool C3 = decltype(ct3)::value, F = decltype(f16)::value, P2 = decltype(p2)::value;
      switch (ep) {
        case 0: hipLaunchKernelGGL((gemm8p_kernel<AC, C3, F, 0, 0, 3, P2>), dim3(G), dim3(512), 0, s, a, n_tiles); break;
        case 1: hipLaunchKernelGGL((gemm8p_kernel<AC, C3, F, 1, 0, 3, P2>), dim3(G), dim3(512), 0, s, a, n_tiles); break;
        case 2: hipLaunchKernelGGL((gemm8p_kernel<AC, C3, F, 2, 0, 3, P2>), dim3(G), dim3(512), 0, s, a, n_tiles); break;
        default:
          if constexpr (!F && !C3) {   // bf16 folded LayerNorm: the input's column-tile count
            if (a.apart_nt == 4) {
              hipLaunchKernelGGL((gemm8p_kernel<AC, C3, F, 3, 0, 4, P2>), dim3(G), dim3(512), 0, s, a, n_tiles);
              break;
            }
            if (a.apart_nt == 5) {
              hipLaunchKernelGGL((gemm8p_kernel<AC, C3, F, 3, 0, 5, P2>), dim3(G), dim3(512), 0, s, a, n_tiles);
              break;
            }
          }
          hipLaunchKernelGGL((gemm8p_kernel<AC, C3, F, 3, 0, 3, P2>), dim3(G), dim3(512), 0, s, a, n_tiles);
          break;
      }
    };
    auto go = [&](auto act, auto ct3, auto f16) {
      if (ph2) go2(act, ct3, f16, std::true_type{});
      else go2(act, ct3, f16, std::false_type{});
    };
    using F_ = std::false_type;
    using T_ = std::true_type;
    if (a.h16) {   // plain fp16: GELU_FAST (conv layers, ffn1; ACT_GELU under OPT_GELU_EXACT) or none
      if (a.act == ACT_GELU_FAST)
        go(std::integral_constant<int, ACT_GELU_FAST>{}, F_{}, T_{});
      else if (a.act == ACT_GELU)
        go(std::integral_constant<int, ACT_GELU>{}, F_{}, T_{});
      else
        go(std::integral_constant<int, ACT_NONE>{}, F_{}, T_{});
    } else if (a.f16) {   // split-fp16: ct3 + erf-GELU (conv layers, ffn1) or fp32 out (proj, qkv)
      if (a.ct3)
        go(std::integral_constant<int, ACT_GELU>{}, T_{}, T_{});
      else
        go(std::integral_constant<int, ACT_NONE>{}, F_{}, T_{});
    } else if (a.act == ACT_GELU)
      go(std::integral_constant<int, ACT_GELU>{}, F_{}, F_{});
    else if (a.act == ACT_GELU_FAST)
      go(std::integral_constant<int, ACT_GELU_FAST>{}, F_{}, F_{});
    else
      go(std::integral_constant<int, ACT_NONE>{}, F_{}, F_{});
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// MX-fp8 operands (K % 128 == 0, N % 256 == 0, plain row-major A with lda == K); output fp32 (Cf,
// optional residual), bf16 (Ct) or MX-fp8 (Ct + c_scale, A layout of a GEMM with K = N).
int launch_gemm8_mx(const GemmArgs& a, hipStream_t s) {
  if (a.M <= 0 || a.N % 256 || a.K % 128 || a.K <= 0 || !a.a_scale || !a.b_scale) return -3;
  if (a.rows_per_seg != a.M || a.lda != a.K) return -3;
  if (a.c_scale && (a.Cf || !a.Ct)) return -3;
  dim3 grid((unsigned)(((a.M + 255) / 256) * (a.N / 256)));
  // Non-persistent for every MX shape: the persistent kernel exceeds 256 VGPRs with the MX operand
  // tuples and would spill inside the counted-vmcnt main loop.  Without a residual, or with the bf16
  // residual stream (fc2, round 5), the MFMAs compute C^T and the epilogue stores from registers (no LDS
  // round trip; OPT_GEMM_MX_STAGED keeps the LDS-staged epilogue for A/B runs); fp32 residuals take the
  // staged epilogue.
  if (a.resid && a.resid_t) return -3;
  // register-direct (C^T) epilogue: no residual, or the bf16 residual stream (fc2: resid_t in place, no fp32 out)
  const bool direct = !a.resid && (!a.resid_t || (a.Ct && !a.Cf && !a.c_scale && !a.rstats && !a.rpart && !a.opart &&
                                                   !a.resid_rows));
  const bool plain = a.bias && !a.resid && !a.Cf && a.Ct && !a.rstats && !a.rpart && !a.opart && !a.resid_rows;
  // the fp8 attention's operands: only as the two compile-time forms below
  if (a.n_split) {   // fused Q|K | V (both forms below at once)
    if (!plain || a.resid_t || a.act != ACT_NONE || !a.c_scale || !a.c_scale_rm || !a.vamax || !a.ct2 ||
        a.vamax_rows < 64 || a.n_split % 256 || a.n_split >= a.N || a.ldc != a.n_split || a.ldc2 < a.N - a.n_split)
      return -3;
    launch_g8mx<true, 6>(grid, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
  }
  if (a.c_scale_rm || a.vamax) {
    if (!plain || a.resid_t || a.act != ACT_NONE || (a.c_scale_rm && !a.c_scale) || (a.vamax && a.c_scale) ||
        (a.vamax && a.vamax_rows < 64))
      return -3;
    if (a.c_scale_rm)
      launch_g8mx<true, 4>(grid, s, a);
    else
      launch_g8mx<true, 5>(grid, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
  }
  if (direct && !sse_opt(OPT_GEMM_MX_STAGED)) {
    if (a.resid_t) {   // (direct implies Ct, no Cf / fp8 out / LayerNorm)
      // fc2's compile-time epilogue (MXE 2) is bias + residual, no activation; any other bias / act combination
      // takes the staged epilogue, which reads both at run time
      if (a.bias && a.act == ACT_NONE) launch_g8mx<true, 2>(grid, s, a);
      else launch_g8mx<false>(grid, s, a);
    }
    else if (plain && a.c_scale && a.act == ACT_GELU_FAST)   // fc1
      launch_g8mx<true, 1>(grid, s, a);
    else if (plain && !a.c_scale && a.act == ACT_NONE)      // qkv
      launch_g8mx<true, 3>(grid, s, a);
    else
      launch_g8mx<true>(grid, s, a);
  } else {
    launch_g8mx<false>(grid, s, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
