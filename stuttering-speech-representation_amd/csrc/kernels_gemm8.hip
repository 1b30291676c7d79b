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
#include <string.h>

#include <type_traits>

#include "common.h"

namespace {

constexpr int G8_HALF = 128 * 128;            // one half-tile: 128 rows x 128 B (64 bf16 of K)
constexpr int G8_BUF = 4 * G8_HALF;           // A rows 0-127 | A rows 128-255 | B cols 0-127 | B cols 128-255
constexpr int G8_OPS = 2 * G8_BUF;            // two K-tiles: 128 KiB
constexpr int G8_CLD = 256 + 4;               // epilogue fp32 row stride (floats)
constexpr int G8_EPI = 128 * G8_CLD * 4;      // one 128-row half of the C tile
constexpr int G8_SMEM = G8_OPS > G8_EPI ? G8_OPS : G8_EPI;

// phase k = 4t + p (k >= -8) -> the (tile, half) whose LDS-DMA it issues
SSE_DEV void g8_target(int k, int& tile, int& half) {
  const int t = (k + 8) / 4 - 2, p = (k + 8) & 3;
  tile = p < 2 ? t + 1 : t + 2;
  half = p == 0 ? 3 : (p == 1 ? 1 : (p == 2 ? 0 : 2));
}

SSE_DEV int g8_issued(int k, int nk) {
  if (k < -6) return 0;
  int tile, half;
  g8_target(k, tile, half);
  return tile < nk ? 1 : 0;
}

// retire every half-tile issued at phases <= k-4 (2 DMA instructions per half per wave)
SSE_DEV void g8_wait(int k, int nk) {
  const int n = g8_issued(k, nk) + g8_issued(k - 1, nk) + g8_issued(k - 2, nk) + g8_issued(k - 3, nk);
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
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

// DBG = 1 (SSE_GEMM_DEBUG=skip_epi, timing experiments only): no epilogue, a checksum keeps the MFMAs live.
template <bool RES>
SSE_DEV void g8_epilogue_direct(const GemmArgs& g, f32x4 (&acc)[2][2][4][2], int m0, int n0, int wm, int wn,
                                int q, int r16);

// TR = true: the MFMAs compute C^T blocks (the B fragment is the MFMA's A operand), so every
// lane ends up holding 4 consecutive output columns of one row and the epilogue stores straight
// from registers (see g8_epilogue_direct).  TR = false: C blocks, LDS-staged epilogue.
template <int DBG, bool TR, bool NT>
__global__ __launch_bounds__(512) void gemm8_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[G8_SMEM];   // the ONLY shared object
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
  const int m0 = (bid / n_tiles_n) * 256, n0 = (bid % n_tiles_n) * 256;
  const int nk = K / 64;

  // ---- LDS-DMA sources: buffer descriptors based at the block's first A row / B row; each
  // lane's byte offset is fixed for the whole K loop, the scalar soffset advances by 128 B.
  constexpr int NREC = 0x7FFFFFF0;
  __amdgpu_buffer_rsrc_t a_rsrc, b_rsrc;
  unsigned a_voff[2][2], b_voff[2][2];
  {
    const int mf = m0 < M ? m0 : M - 1;
    const int seg0 = mf / g.rows_per_seg, rr0 = mf - seg0 * g.rows_per_seg;
    const long long a_base = (long long)seg0 * g.seg_stride + (long long)rr0 * g.lda;
    a_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)((const bf16*)g.A + a_base), (short)0, NREC, 0x00020000);
    b_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)((const bf16*)g.B + (long long)n0 * K), (short)0, NREC,
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
        const long long el = (long long)seg * g.seg_stride + (long long)rr * g.lda + ch * 8;
        a_voff[h][s] = (unsigned)((el - a_base) * 2);
        b_voff[h][s] = (unsigned)(((long long)row * K + ch * 8) * 2);
      }
  }
  auto issue = [&](int k) {
    if (k < -6) return;
    int tile, half;
    g8_target(k, tile, half);
    if (tile >= nk) return;
    char* dst = smem + (tile & 1) * G8_BUF + half * G8_HALF;
    const unsigned soff = (unsigned)tile * 128u;
    if (half < 2) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, LPTR(dst + wave * 1024), 16, a_voff[half][0], soff, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, LPTR(dst + (wave + 8) * 1024), 16, a_voff[half][1], soff, 0, 0);
    } else {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, LPTR(dst + wave * 1024), 16, b_voff[half - 2][0], soff, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, LPTR(dst + (wave + 8) * 1024), 16, b_voff[half - 2][1], soff, 0,
                                               0);
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
    __builtin_amdgcn_s_setprio(1);
    #pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      #pragma unroll
      for (int i = 0; i < 4; ++i)
        #pragma unroll
        for (int j = 0; j < 2; ++j)
          c[i][j] = TR ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][ks], af[i][ks], c[i][j], 0, 0, 0)
                       : __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][ks], bf[j][ks], c[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };

  // ---- prologue: phases -6..-1 stage A0(0) B0(0) B1(0) A1(0) A0(1) B0(1)
  for (int k = -6; k < 0; ++k) issue(k);
  g8_wait(-1, nk);
  g8_barrier();
  if (wm == 1) g8_barrier();   // group 1 runs one barrier behind

  // steady K-tiles (t + 2 < nk): every phase issues a half and waits vmcnt(8) with no
  // scalar bookkeeping; the last two K-tiles take the counted tail path.
  auto run_tile = [&](int t, auto steady) {
    constexpr bool ST = decltype(steady)::value;
    const char* buf = smem + (t & 1) * G8_BUF;
    const int k = 4 * t;
    auto issue_wait = [&](int kk) {
      if constexpr (ST) {
        issue(kk);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else {
        issue(kk);
        g8_wait(kk, nk);
      }
    };
    // phase 0: (mi 0, ni 0) reads A rows 0-127 and B cols 0-127
    read_a(buf);
    read_b(buf + 2 * G8_HALF, b0f);
    issue_wait(k);
    g8_barrier();
    mma(acc[0][0], b0f);
    g8_barrier();
    // phase 1: (mi 0, ni 1) reads B cols 128-255
    read_b(buf + 3 * G8_HALF, b1f);
    issue_wait(k + 1);
    g8_barrier();
    mma(acc[0][1], b1f);
    g8_barrier();
    // phase 2: (mi 1, ni 1) reads A rows 128-255
    read_a(buf + G8_HALF);
    issue_wait(k + 2);
    g8_barrier();
    mma(acc[1][1], b1f);
    g8_barrier();
    // phase 3: (mi 1, ni 0) no reads
    issue_wait(k + 3);
    g8_barrier();
    mma(acc[1][0], b0f);
    g8_barrier();
  };
  int t = 0;
  for (; t + 2 < nk; ++t) run_tile(t, std::integral_constant<bool, true>{});
  for (; t < nk; ++t) run_tile(t, std::integral_constant<bool, false>{});
  if (wm == 0) g8_barrier();   // balance group 1's extra barrier
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (DBG == 1) {
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
    if (g.resid) g8_epilogue_direct<true>(g, acc, m0, n0, wm, wn, q, r16);
    else g8_epilogue_direct<false>(g, acc, m0, n0, wm, wn, q, r16);
    return;
  }

  // ---- epilogue: per 128-row half, stage fp32 through LDS, then coalesced 16-B passes -----
  float* Cs = (float*)smem;
  constexpr int CH = 128 * 256 / 4;
  constexpr int UNR = 4;
  const bool has_bias = g.bias != nullptr, has_res = g.resid != nullptr, gelu = g.act == ACT_GELU, gelu_fast = g.act == ACT_GELU_FAST;
  #pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
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
    f32x4 lw = f32x4{1.f, 1.f, 1.f, 1.f}, lb = f32x4{0.f, 0.f, 0.f, 0.f};
    if (g.rstats) {
      lw = *(const f32x4*)(g.rln_w + n);
      lb = *(const f32x4*)(g.rln_b + n);
    }
    for (int base = threadIdx.x; base < CH; base += 512 * UNR) {
      f32x4 v[UNR], rv[UNR];
      float2 st[UNR];
      long long off[UNR];
      bool ok[UNR];
      #pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int row = (base + u * 512) >> 6;
        const int m = m0 + mi * 128 + row;
        ok[u] = m < M;
        off[u] = (long long)(ok[u] ? m : 0) * g.ldc + n;
        v[u] = *(const f32x4*)(Cs + row * G8_CLD + cc);
        rv[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        st[u] = make_float2(0.f, 1.f);
        if (has_res) {
          const long long ro = g.resid_rows ? (long long)((ok[u] ? m : 0) % g.resid_rows) * g.ldc + n : off[u];
          rv[u] = g8_ld<NT>((const f32x4*)(g.resid + ro));
          if (g.rstats) st[u] = g.rstats[ok[u] ? m : 0];
        }
      }
      #pragma unroll
      for (int u = 0; u < UNR; ++u) {
        f32x4 o = v[u] + bv;
        if (gelu) {
          const f32x2 lo = gelu_erf2(f32x2{o[0], o[1]}), hi = gelu_erf2(f32x2{o[2], o[3]});
          o = f32x4{lo.x, lo.y, hi.x, hi.y};
        }
        if (gelu_fast) {
          const f32x2 lo = gelu_sig2(f32x2{o[0], o[1]}), hi = gelu_sig2(f32x2{o[2], o[3]});
          o = f32x4{lo.x, lo.y, hi.x, hi.y};
        }
        f32x4 r = rv[u];
        if (g.rstats) {   // LayerNorm of the residual, the exact expression of layernorm_kernel
          #pragma unroll
          for (int e = 0; e < 4; ++e) r[e] = fmaf((r[e] - st[u].x) * st[u].y, lw[e], lb[e]);
        }
        o += r;
        if (ok[u]) {
          if (g.Cf) g8_st<NT>((f32x4*)(g.Cf + off[u]), o);
          if (g.Ct) {
            const bf16x4 ob = {(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
            g8_st<NT>((bf16x4*)((bf16*)g.Ct + off[u]), ob);
          }
        }
      }
    }
  }
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
SSE_DEV void g8_vmcnt_dyn(int n) {   // n even, 0..62 (vmcnt is 6 bits)
  switch (n >> 1) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(22)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(26)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(28)" ::: "memory"); break;
    case 15: asm volatile("s_waitcnt vmcnt(30)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
    case 17: asm volatile("s_waitcnt vmcnt(34)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(36)" ::: "memory"); break;
    case 19: asm volatile("s_waitcnt vmcnt(38)" ::: "memory"); break;
    case 20: asm volatile("s_waitcnt vmcnt(40)" ::: "memory"); break;
    case 21: asm volatile("s_waitcnt vmcnt(42)" ::: "memory"); break;
    case 22: asm volatile("s_waitcnt vmcnt(44)" ::: "memory"); break;
    case 23: asm volatile("s_waitcnt vmcnt(46)" ::: "memory"); break;
    case 24: asm volatile("s_waitcnt vmcnt(48)" ::: "memory"); break;
    case 25: asm volatile("s_waitcnt vmcnt(50)" ::: "memory"); break;
    case 26: asm volatile("s_waitcnt vmcnt(52)" ::: "memory"); break;
    case 27: asm volatile("s_waitcnt vmcnt(54)" ::: "memory"); break;
    case 28: asm volatile("s_waitcnt vmcnt(56)" ::: "memory"); break;
    case 29: asm volatile("s_waitcnt vmcnt(58)" ::: "memory"); break;
    case 30: asm volatile("s_waitcnt vmcnt(60)" ::: "memory"); break;
    case 31: asm volatile("s_waitcnt vmcnt(62)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

SSE_DEV int g8_count(int k, int nk) {   // vmcnt of g8_wait(k, nk)
  return 2 * (g8_issued(k, nk) + g8_issued(k - 1, nk) + g8_issued(k - 2, nk) + g8_issued(k - 3, nk));
}

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
template <bool RES>
SSE_DEV void g8_epilogue_direct(const GemmArgs& g, f32x4 (&acc)[2][2][4][2], int m0, int n0, int wm, int wn,
                                int q, int r16) {
  const bool has_bias = g.bias != nullptr, has_res = RES && g.resid != nullptr, ln = RES && g.rstats != nullptr;
  const bool gelu = g.act == ACT_GELU, gelu_fast = g.act == ACT_GELU_FAST;
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
  float2 st[4];
  auto load_half = [&](int mi) {
    if (!has_res) return;
    #pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + mi * 128 + wm * 64 + i * 16 + r16;
      const int mc = m < g.M ? m : 0;
      const long long rrow = g.resid_rows ? (long long)(mc % g.resid_rows) * g.ldc : (long long)mc * g.ldc;
      #pragma unroll
      for (int ni = 0; ni < 2; ++ni)
        #pragma unroll
        for (int j = 0; j < 2; ++j)
          rv[i][ni][j] = *(const f32x4*)(g.resid + rrow + n0 + ni * 128 + wn * 32 + j * 16 + q * 4);
      st[i] = ln ? g.rstats[mc] : make_float2(0.f, 1.f);
    }
  };
  auto finish_half = [&](int mi) {   // acc[mi] <- bias, activation, (LayerNorm'd) residual
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
          if (gelu_fast) {
            const f32x2 lo = gelu_sig2(f32x2{o[0], o[1]}), hi = gelu_sig2(f32x2{o[2], o[3]});
            o = f32x4{lo.x, lo.y, hi.x, hi.y};
          }
          if (has_res) {
            f32x4 r = rv[i][ni][j];
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
          if (ok) {
            const uint4 v = make_uint4(s0[0], s1[0], s0[1], s1[1]);
            *(uint4*)((bf16*)g.Ct + row + n0 + ni * 128 + wn * 32 + (q & 1) * 16 + (q >> 1) * 8) = v;
          }
        }
      }
    }
  };
  load_half(0);
  finish_half(0);
  load_half(1);
  store_half(0);
  finish_half(1);
  store_half(1);
}

// RES = false only: residual GEMMs keep the non-persistent LDS-staged kernel (their epilogue
// would need the residual tile in registers next to the accumulators).
template <bool RES>
__global__ __launch_bounds__(512) void gemm8p_kernel(GemmArgs g, int n_tiles) {
  __shared__ __attribute__((aligned(16))) char smem[G8_OPS];   // the ONLY shared object
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
  const int s_full = min(32 * (g.Cf ? 1 : 0) + 16 * (g.Ct ? 1 : 0), 54);

  int round = 0;
  int tile = g8p_tile(b, 0, G, n_tiles);
  if (tile < 0) return;

  constexpr int NREC = 0x7FFFFFF0;
  __amdgpu_buffer_rsrc_t a_rsrc, b_rsrc;
  unsigned a_voff[2][2], b_voff[2][2];
  auto setup = [&](int tl) {
    const int m0 = (tl / n_tiles_n) * 256, n0 = (tl % n_tiles_n) * 256;
    const int mf = m0 < M ? m0 : M - 1;
    const int seg0 = mf / g.rows_per_seg, rr0 = mf - seg0 * g.rows_per_seg;
    const long long a_base = (long long)seg0 * g.seg_stride + (long long)rr0 * g.lda;
    a_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)((const bf16*)g.A + a_base), (short)0, NREC, 0x00020000);
    b_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)((const bf16*)g.B + (long long)n0 * K), (short)0, NREC,
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
        const long long el = (long long)seg * g.seg_stride + (long long)rr * g.lda + ch * 8;
        a_voff[h][s] = (unsigned)((el - a_base) * 2);
        b_voff[h][s] = (unsigned)(((long long)row * K + ch * 8) * 2);
      }
  };
  auto issue = [&](int k) {
    if (k < -6) return;
    int tl, half;
    g8_target(k, tl, half);
    if (tl >= nk) return;
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
    __builtin_amdgcn_s_setprio(1);
    #pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      #pragma unroll
      for (int i = 0; i < 4; ++i)
        #pragma unroll
        for (int j = 0; j < 2; ++j) c[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][ks], af[i][ks], c[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };

  setup(tile);
  for (int k = -6; k < 0; ++k) issue(k);
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
    g8_vmcnt_dyn(g8_count(-1, nk) + S);
    g8_barrier();
    if (wm == 1) g8_barrier();   // group 1 runs one barrier behind

    // FIRST: 0 = steady, 1 = first K-tile (waits leave the previous tile's S stores in flight)
    auto run_tile = [&](int t, auto steady, auto first) {
      constexpr bool ST = decltype(steady)::value;
      constexpr bool FI = decltype(first)::value;
      const char* buf = smem + (t & 1) * G8_BUF;
      const int k = 4 * t;
      auto issue_wait = [&](int kk) {
        issue(kk);
        if constexpr (FI) {
          g8_vmcnt_dyn(g8_count(kk, nk) + S);
        } else if constexpr (ST) {
          asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
          g8_wait(kk, nk);
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
    run_tile(0, std::integral_constant<bool, false>{}, std::integral_constant<bool, true>{});
    int t = 1;
    for (; t + 2 < nk; ++t) run_tile(t, std::integral_constant<bool, true>{}, std::integral_constant<bool, false>{});
    for (; t < nk; ++t) run_tile(t, std::integral_constant<bool, false>{}, std::integral_constant<bool, false>{});
    if (wm == 0) g8_barrier();   // balance group 1's extra barrier: every wave's LDS reads are done

    ++round;
    const int next = g8p_tile(b, round, G, n_tiles);
    if (next >= 0) {
      setup(next);
      for (int k = -6; k < 0; ++k) issue(k);
    }
    g8_epilogue_direct<RES>(g, acc, m0, n0, wm, wn, q, r16);
    if (next < 0) break;
    S = m0 + 256 <= M ? s_full : 0;
    tile = next;
  }
}

}  // namespace

int launch_gemm8_bf16(const GemmArgs& a, hipStream_t s) {
  if (a.M <= 0 || a.N % 256 || a.K % 64 || a.K <= 0) return -3;
  dim3 grid((unsigned)(((a.M + 255) / 256) * (a.N / 256)));
  static const bool skip_epi = [] { const char* e = getenv("SSE_GEMM_DEBUG"); return e && !strcmp(e, "skip_epi"); }();
  // A/B switches: SSE_GEMM_PERSIST=0 (non-persistent LDS-staged kernel for every shape),
  // SSE_GEMM_NT=1 (non-temporal epilogue stores in that kernel)
  const char* npe = getenv("SSE_GEMM_PERSIST");   // read per launch (tests flip it)
  const bool np = npe && npe[0] == '0';
  static const bool nt = [] { const char* e = getenv("SSE_GEMM_NT"); return e && e[0] == '1'; }();
  if (skip_epi) {
    hipLaunchKernelGGL((gemm8_kernel<1, true, false>), grid, dim3(512), 0, s, a);
  } else if (a.resid || np) {
    if (nt)
      hipLaunchKernelGGL((gemm8_kernel<0, false, true>), grid, dim3(512), 0, s, a);
    else
      hipLaunchKernelGGL((gemm8_kernel<0, false, false>), grid, dim3(512), 0, s, a);
  } else {
    // persistent: one block per CU (LDS-bound), at most one per tile
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -2;
    if (!cus[dev] && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return -2;
    const int n_tiles = (int)grid.x;
    const int G = n_tiles < cus[dev] ? n_tiles : cus[dev];
    hipLaunchKernelGGL(gemm8p_kernel<false>, dim3(G), dim3(512), 0, s, a, n_tiles);
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
