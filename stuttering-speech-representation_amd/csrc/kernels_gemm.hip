// MFMA GEMM / implicit-GEMM conv for gfx950 (CDNA4).
//
// One kernel template serves every dense contraction on the hot path:
//   K2  WavLM conv1..6           (SEG mode: overlapping rows, A row t = x[s*t : s*t+k] of a clip)
//   K3  feature projection, K6 QKV / out-proj, K7 FFN, K11 Whisper projections   (plain SEG)
//   K4  pos-conv (grouped, k=128, pad 64) and K10 Whisper conv1/conv2 (k=3, pad 1)  (CONV mode)
// Tiles: rows of 128 bytes along K (64 bf16 / 32 f32 per K-step), staged HBM->LDS with
// global_load_lds_dwordx4 (one 1-KiB wave-instruction = 8 rows), double-buffered, one
// barrier per K-step.  The LDS image is lane-linear; bank conflicts of the ds_read_b128
// fragment reads are removed by an XOR swizzle applied to the SOURCE chunk
// (phys_chunk = chunk ^ ((row >> 1) & 7)), see cdna_hip_programming.md rule 21.
// Math: v_mfma_f32_16x16x32_bf16 (bf16 path) or v_mfma_f32_16x16x4_f32 (exact-f32 path);
// both read the same LDS image: lane group q = lane>>4 consumes 16-B chunks q and q+4.
// Epilogue fuses bias, erf-GELU, fp32 residual add and dual fp32/bf16 stores.
#include <cstdlib>

#include "common.h"

namespace {

template <typename T, int BM, int BN, int WAVES_M, int WAVES_N, int AMODE, int STAGES>
__device__ __forceinline__ void gemm_body(const GemmArgs& g) {
  constexpr int NW = WAVES_M * WAVES_N;
  constexpr int E = 16 / (int)sizeof(T);   // elements per 16-B chunk
  constexpr int BK = 8 * E;                 // elements per 128-B row
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int A_INSTR = BM / 8, B_INSTR = BN / 8;            // 1-KiB glds pieces per tile
  constexpr int SA = (A_INSTR + NW - 1) / NW, SB = (B_INSTR + NW - 1) / NW;
  static_assert(WM % 16 == 0 && WN % 16 == 0, "wave tile");
  // STAGES == 3: every wave issues the same number of pieces per tile, so one counted
  // vmcnt retires exactly the oldest tile while the next one stays in flight.
  static_assert(STAGES == 2 || (A_INSTR % NW == 0 && B_INSTR % NW == 0), "uniform pieces per wave");
  constexpr int P = SA + SB;   // glds per wave per tile (STAGES == 3)
  constexpr int CLD = BN + 4;                 // epilogue: padded fp32 C row (conflict-free b32 writes)
  // the fp32 C tile goes through LDS in row chunks of EPI_ROWS (the whole tile when it fits)
  constexpr int EPI_ROWS = (BM * CLD * 4 <= 80 * 1024 || BM * CLD * 4 <= STAGES * STAGE) ? BM : BM / 2;
  static_assert(BM % EPI_ROWS == 0 && EPI_ROWS % WM == 0, "epilogue chunks must hold whole wave rows");
  constexpr int SMEM = STAGES * STAGE > EPI_ROWS * CLD * 4 ? STAGES * STAGE : EPI_ROWS * CLD * 4;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int n_tiles_n = g.N / BN;
  // XCD-aware remap (bijective): blocks b, b+8, ... share an XCD, so give each XCD a
  // contiguous run of tiles; the N-tiles of one M-tile then reuse the A panel in one L2.
  int bid = blockIdx.x;
  {
    const int nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, x = bid % 8;
    bid = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + bid / 8;
  }
  const int tile_n = bid % n_tiles_n, tile_m = bid / n_tiles_n;
  const int grp = blockIdx.y;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int M = g.M, N = g.N, K = g.K;

  // ---- per-lane source descriptors for the LDS-DMA pieces this wave issues ------------
  // SEG mode: one buffer descriptor per operand based at the block's first row; every lane's
  // byte offset is fixed for the whole K loop and only the scalar soffset advances per K-step
  // (no per-step VALU address math).  Chunks past K read as zero through an out-of-range
  // offset (the descriptor's range check returns 0).  CONV mode keeps per-chunk addresses.
  constexpr unsigned NREC = 0x7FFFFFF0u, OOB = 0x7FFFFFF0u;
  __amdgpu_buffer_rsrc_t a_rsrc, b_rsrc;
  unsigned a_voff[SA], b_voff[SB];
  const char* a_src[SA];
  int a_chunk[SA];
  int a_tb[SA], a_to[SA];     // CONV: seg*T_in, t_out*stride - pad
  {
    const int mf = m0 < M ? m0 : M - 1;
    const int seg0 = mf / g.rows_per_seg, r0 = mf - seg0 * g.rows_per_seg;
    const long long a_base_el = (long long)seg0 * g.seg_stride + (long long)r0 * g.lda;
    a_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)g.A + a_base_el * (long long)sizeof(T)), (short)0,
                                               (int)NREC, 0x00020000);
    const char* b_base = (const char*)g.B + ((long long)grp * N + n0) * K * (long long)sizeof(T);
    b_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)b_base, (short)0, (int)NREC, 0x00020000);
    #pragma unroll
    for (int s = 0; s < SA; ++s) {
      const int piece = wave + NW * s;
      const int row = piece * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ ((row >> 1) & 7);
      int m = m0 + row;
      m = m < M ? m : M - 1;
      a_chunk[s] = ch;
      const int seg = m / g.rows_per_seg, r = m - seg * g.rows_per_seg;
      const long long el = (long long)seg * g.seg_stride + (long long)r * g.lda + ch * E;
      a_voff[s] = (unsigned)((el - a_base_el) * (long long)sizeof(T));
      a_src[s] = (const char*)g.A;
      a_tb[s] = seg * g.T_in;
      a_to[s] = r * g.stride - g.pad;
    }
    #pragma unroll
    for (int s = 0; s < SB; ++s) {
      const int piece = wave + NW * s;
      const int row = piece * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ ((row >> 1) & 7);
      b_voff[s] = (unsigned)(((row < BN ? row : 0) * (long long)K + ch * E) * (long long)sizeof(T));
    }
  }

  auto issue = [&](int kt, int buf) {
    char* st = smem + buf * STAGE;
    const int k0 = kt * BK;
    const unsigned soff = (unsigned)k0 * (unsigned)sizeof(T);
    if (AMODE == AMODE_SEG && k0 + BK <= K) {   // wave-uniform fast path: no per-lane work at all
      #pragma unroll
      for (int s = 0; s < SA; ++s) {
        const int piece = wave + NW * s;
        if (A_INSTR % NW == 0 || piece < A_INSTR)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, LPTR(st + piece * 1024), 16, a_voff[s], soff, 0, 0);
      }
      #pragma unroll
      for (int s = 0; s < SB; ++s) {
        const int piece = wave + NW * s;
        if (B_INSTR % NW == 0 || piece < B_INSTR)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, LPTR(st + A_BYTES + piece * 1024), 16, b_voff[s], soff, 0, 0);
      }
      return;
    }
    #pragma unroll
    for (int s = 0; s < SA; ++s) {
      const int piece = wave + NW * s;
      if (A_INSTR % NW == 0 || piece < A_INSTR) {
        if (AMODE == AMODE_SEG) {
          const unsigned vo = k0 + a_chunk[s] * E < K ? a_voff[s] : OOB;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, LPTR(st + piece * 1024), 16, vo, soff, 0, 0);
        } else {
          const int k = k0 + a_chunk[s] * E;
          const int j = k / g.cin, c = k - j * g.cin;
          const int t = a_to[s] + j;
          const void* src = (k < K && t >= 0 && t < g.T_in)
                                ? (const void*)(a_src[s] + (((long long)(a_tb[s] + t)) * g.ld_in + grp * g.cin + c) *
                                                               (long long)sizeof(T))
                                : g.zero;
          __builtin_amdgcn_global_load_lds(GPTR(src), LPTR(st + piece * 1024), 16, 0, 0);
        }
      }
    }
    #pragma unroll
    for (int s = 0; s < SB; ++s) {
      const int piece = wave + NW * s;
      if (B_INSTR % NW == 0 || piece < B_INSTR) {
        const int row = piece * 8 + (lane >> 3);
        const int ch = (lane & 7) ^ ((row >> 1) & 7);
        const unsigned vo = k0 + ch * E < K ? b_voff[s] : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, LPTR(st + A_BYTES + piece * 1024), 16, vo, soff, 0, 0);
      }
    }
  };

  f32x4 acc[TM][TN];
  #pragma unroll
  for (int i = 0; i < TM; ++i)
    #pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int q = lane >> 4, r16 = lane & 15;
  const int nk = (K + BK - 1) / BK;
  issue(0, 0);
  if (STAGES == 3 && nk > 1) issue(1, 1);
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if constexpr (STAGES == 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (kt + 1 < nk) issue(kt + 1, (kt + 1) & 1);
      cur = kt & 1;
    } else {
      // tile kt landed (tile kt+1 may stay in flight); no wave still reads buffer (kt+2)%3
      if (kt + 1 < nk)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kt + 2 < nk) issue(kt + 2, cur == 0 ? 2 : cur - 1);
    }
    const char* As = smem + cur * STAGE;
    const char* Bs = As + A_BYTES;
    if constexpr (sizeof(T) == 2) {
      #pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 af[TM], bfr[TN];
        #pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wm * WM + i * 16 + r16;
          const int pch = (q + 4 * ks) ^ ((row >> 1) & 7);
          af[i] = *(const bf16x8*)(As + row * 128 + pch * 16);
        }
        #pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int row = wn * WN + j * 16 + r16;
          const int pch = (q + 4 * ks) ^ ((row >> 1) & 7);
          bfr[j] = *(const bf16x8*)(Bs + row * 128 + pch * 16);
        }
        #pragma unroll
        for (int i = 0; i < TM; ++i)
          #pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
      f32x4 a0[TM], a1[TM], b0[TN], b1[TN];
      #pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 16 + r16;
        const int sw = (row >> 1) & 7;
        a0[i] = *(const f32x4*)(As + row * 128 + ((q) ^ sw) * 16);
        a1[i] = *(const f32x4*)(As + row * 128 + ((q + 4) ^ sw) * 16);
      }
      #pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WN + j * 16 + r16;
        const int sw = (row >> 1) & 7;
        b0[j] = *(const f32x4*)(Bs + row * 128 + ((q) ^ sw) * 16);
        b1[j] = *(const f32x4*)(Bs + row * 128 + ((q + 4) ^ sw) * 16);
      }
      #pragma unroll
      for (int e = 0; e < 4; ++e)
        #pragma unroll
        for (int i = 0; i < TM; ++i)
          #pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[i][e], b0[j][e], acc[i][j], 0, 0, 0);
      #pragma unroll
      for (int e = 0; e < 4; ++e)
        #pragma unroll
        for (int i = 0; i < TM; ++i)
          #pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[i][e], b1[j][e], acc[i][j], 0, 0, 0);
    }
    if constexpr (STAGES == 3) cur = cur == 2 ? 0 : cur + 1;
  }

  // ---- epilogue: stage the fp32 tile through LDS, then one coalesced pass per 16-B chunk:
  //      v = acc + bias (act) (+resid) -> fp32 and/or element-type stores -----------------
  float* Cs = (float*)smem;
  constexpr int NT = NW * 64;
  constexpr int CH = EPI_ROWS * BN / 4;       // 16-B chunks per epilogue chunk
  constexpr int UNR = 4;
  const int col0 = grp * N;
  // residual: fp32 (resid) or a bf16 residual stream (resid_t, read in place)
  const bool has_bias = g.bias != nullptr, has_res = g.resid != nullptr || g.resid_t != nullptr;
  const bool gelu = g.act == ACT_GELU, gelu_fast = g.act == ACT_GELU_FAST;
  #pragma unroll
  for (int half = 0; half < BM / EPI_ROWS; ++half) {
    __syncthreads();                          // operand stages (or the previous chunk) fully consumed
    if (wm * WM >= half * EPI_ROWS && wm * WM < (half + 1) * EPI_ROWS) {
      #pragma unroll
      for (int i = 0; i < TM; ++i)
        #pragma unroll
        for (int j = 0; j < TN; ++j)
          #pragma unroll
          for (int r = 0; r < 4; ++r)
            Cs[(wm * WM - half * EPI_ROWS + i * 16 + q * 4 + r) * CLD + wn * WN + j * 16 + r16] = acc[i][j][r];
    }
    __syncthreads();
    for (int base = threadIdx.x; base < CH; base += NT * UNR) {
      f32x4 v[UNR], rv[UNR], bv[UNR];
      long long off[UNR];
      bool ok[UNR];
      #pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int c0 = base + u * NT;
        const int c = c0 < CH ? c0 : CH - 1;
        const int row = c / (BN / 4), cc = (c % (BN / 4)) * 4;
        const int m = m0 + half * EPI_ROWS + row, n = n0 + cc;
        ok[u] = m < M && c0 < CH;
        off[u] = (long long)(ok[u] ? m : 0) * g.ldc + col0 + n;
        v[u] = *(const f32x4*)(Cs + row * CLD + cc);
        bv[u] = has_bias ? *(const f32x4*)(g.bias + col0 + n) : f32x4{0.f, 0.f, 0.f, 0.f};
        rv[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (has_res) {
          const long long ro = g.resid_rows ? (long long)((ok[u] ? m : 0) % g.resid_rows) * g.ldc + col0 + n : off[u];
          if (g.resid_t) {
            const bf16x4 rb = *(const bf16x4*)(g.resid_t + ro);
            rv[u] = f32x4{(float)rb[0], (float)rb[1], (float)rb[2], (float)rb[3]};
          } else {
            rv[u] = *(const f32x4*)(g.resid + ro);
          }
          if (g.rstats) rv[u] = ln_apply4(rv[u], g.rstats[ok[u] ? m : 0], g.rln_w, g.rln_b, col0 + n);
        }
      }
      #pragma unroll
      for (int u = 0; u < UNR; ++u) {
        f32x4 o = v[u] + bv[u];
        if (gelu) {   // packed-fp32 erf-GELU, bit-identical to the scalar form
          const f32x2 lo = gelu_erf2(f32x2{o[0], o[1]}), hi = gelu_erf2(f32x2{o[2], o[3]});
          o = f32x4{lo.x, lo.y, hi.x, hi.y};
        }
        if (gelu_fast) {
          const bool bfo = !g.Cf;   // bf16-only output: the degree-6 form
          const f32x2 lo = gelu_out2(f32x2{o[0], o[1]}, bfo), hi = gelu_out2(f32x2{o[2], o[3]}, bfo);
          o = f32x4{lo.x, lo.y, hi.x, hi.y};
        }
        o += rv[u];
        if (ok[u]) {
          if (g.Cf) *(f32x4*)(g.Cf + off[u]) = o;
          if (g.Ct) {
            if constexpr (sizeof(T) == 2) {
              bf16x4 ob = {(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
              *(bf16x4*)((T*)g.Ct + off[u]) = ob;
            } else {
              *(f32x4*)((T*)g.Ct + off[u]) = o;
            }
          }
        }
      }
    }
  }
}

template <typename T, int BM, int BN, int WAVES_M, int WAVES_N, int AMODE, int STAGES>
__global__ __launch_bounds__(WAVES_M * WAVES_N * 64) void gemm_kernel(GemmArgs g) {
  gemm_body<T, BM, BN, WAVES_M, WAVES_N, AMODE, STAGES>(g);
}

template <typename T, int BM, int BN, int WAVES_M, int WAVES_N, int STAGES>
int launch_cfg(const GemmArgs& a, int amode, int groups, hipStream_t s) {
  dim3 grid((unsigned)(((a.M + BM - 1) / BM) * (a.N / BN)), (unsigned)groups);
  dim3 block(WAVES_M * WAVES_N * 64);
  if (amode == AMODE_SEG)
    hipLaunchKernelGGL((gemm_kernel<T, BM, BN, WAVES_M, WAVES_N, AMODE_SEG, STAGES>), grid, block, 0, s, a);
  else
    hipLaunchKernelGGL((gemm_kernel<T, BM, BN, WAVES_M, WAVES_N, AMODE_CONV, STAGES>), grid, block, 0, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

template <typename T>
int launch_any(const GemmArgs& a, int amode, int groups, hipStream_t s) {
  constexpr int E = 16 / (int)sizeof(T);
  if (a.M <= 0 || a.N <= 0 || a.K <= 0 || a.K % E) return -3;
  if (amode == AMODE_CONV && (a.cin % E)) return -3;
  // bf16 default for the big encoder GEMMs: 256x256 tile, 8 waves (2x4) of 128x64, 2-stage
  // 128 KiB LDS ring (1 block/CU).  Measured on the WavLM-base B=256 shapes vs the 128x128 tile:
  // qkv 837 vs 636, ffn1 691 vs 605, ffn2 931 vs 801, oproj 510 vs 489 TF/s (profiles/r1_gemm_configs.json).
  // Otherwise 128x128, 4 waves of 64x64, 2 stages (2 blocks/CU).  OPT_GEMM_CFG (tests, A/B):
  // 1 = never 256x256, 2 = 256x128 3-stage ring.
  const int force = sse_opt(OPT_GEMM_CFG);
  if (a.apart || a.rpart || a.opart || a.resid_t || a.ct3) {   // folded-LayerNorm epilogues exist in the gemm8 kernels only
    if constexpr (sizeof(T) == 2)
      if (amode == AMODE_SEG && groups == 1 && a.N % 256 == 0 && a.K % 64 == 0) return launch_gemm8_bf16(a, s);
    // a plain bf16 residual stream (Whisper shapes with N % 256 != 0): this file's epilogue reads it
    if (!(a.resid_t && !a.apart && !a.rpart && !a.opart && !a.ct3 && !a.resid && !a.Cf && a.Ct && sizeof(T) == 2))
      return -3;
  }
  if (a.N % 128 == 0 && a.M >= 2048 && force == 2) return launch_cfg<T, 256, 128, 4, 2, 3>(a, amode, groups, s);
  if constexpr (sizeof(T) == 2) {
    // default for plain / SEG-row bf16 GEMMs with N % 256 == 0, K % 64 == 0: the 8-phase
    // ping-pong 256x256 kernel (kernels_gemm8.hip; measured vs this file's 256x256 2-stage loop:
    // qkv 863 vs 760, ffn1 721 vs 653, ffn2 997 vs 880, 4096^3 1353 vs 1192 TF/s).
    // OPT_GEMM_CFG = 3 keeps the 2-stage 256x256 kernel for A/B runs.
    if ((force == 0 || force == 4) && amode == AMODE_SEG && groups == 1 && a.N % 256 == 0 && a.K % 64 == 0 &&
        a.M >= 4096)
      return launch_gemm8_bf16(a, s);
    if (a.N % 256 == 0 && a.M >= 4096 && (force == 0 || force == 3 || force == 4))
      return launch_cfg<T, 256, 256, 2, 4, 2>(a, amode, groups, s);
  }
  if (a.N % 128 == 0) return launch_cfg<T, 128, 128, 2, 2, 2>(a, amode, groups, s);
  if (a.N % 64 == 0) return launch_cfg<T, 128, 64, 4, 1, 2>(a, amode, groups, s);
  if (a.N % 48 == 0) return launch_cfg<T, 128, 48, 4, 1, 2>(a, amode, groups, s);
  return -3;
}

}  // namespace

int launch_gemm_bf16(const GemmArgs& a, int amode, int groups, hipStream_t s) {
  return launch_any<bf16>(a, amode, groups, s);
}
int launch_gemm_f32(const GemmArgs& a, int amode, int groups, hipStream_t s) {
  return launch_any<float>(a, amode, groups, s);
}
