// Short-T attention probe: attention_full_kernel vs attention_pipe_kernel vs attention_pipe2_kernel (option attn_short
// 1 / 0 / 2) on the same
// random WavLM-base-shaped q|k|v|gate rows -- bitwise comparison (first mismatches by clip / row / head /
// column) and event timing of each at the bench's batch sizes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -mllvm -amdgpu-mfma-vgpr-form \
//         tools/attn_probe.hip -o tools/_build/attn_probe
#include "../stuttering-speech-representation_amd/csrc/kernels_misc.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static int g_pipe = 0;
// g_pipe: 0 full, 1 pipelined (double-buffered, one block per CU), 2 two blocks per CU -> option attn_short 1, 0, 2
int sse_opt(int id) { return id == OPT_ATTN_SHORT ? (g_pipe == 0 ? 1 : (g_pipe == 1 ? 0 : 2)) : 0; }
int sse_stream_cus(hipStream_t, int dev_cus) { return dev_cus; }

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(2);                                                                \
    }                                                                              \
  } while (0)

static uint16_t f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
}

static int run(int B, int T, bool h16, bool ragged, int reps) {
  const int nh = 12, H = 768, ldq = 3 * H + 8 * nh, maxd = 320;
  std::vector<uint16_t> hq((size_t)B * T * ldq);
  uint32_t st = 12345u + B * 7 + T;
  auto rnd = [&]() { st = st * 1664525u + 1013904223u; return ((st >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f; };
  for (auto& x : hq) x = f2bf(2.f * rnd());
  std::vector<float> hg(nh), hr((size_t)nh * (2 * maxd + 1));
  for (auto& x : hg) x = 1.f + rnd();
  for (auto& x : hr) x = rnd();
  std::vector<int> hl(B);
  for (int b = 0; b < B; ++b) hl[b] = ragged ? (b % 5 == 0 ? T : 1 + (int)((T - 1) * (0.5f + 0.5f * rnd()))) : T;
  void *dq, *dout[3];
  float *dg, *dr;
  int* dl;
  const size_t ob = (size_t)B * T * H * 2;
  CK(hipMalloc(&dq, hq.size() * 2));
  CK(hipMalloc(&dout[0], ob));
  CK(hipMalloc(&dout[1], ob));
  CK(hipMalloc(&dout[2], ob));
  CK(hipMalloc(&dg, nh * 4));
  CK(hipMalloc(&dr, hr.size() * 4));
  CK(hipMalloc(&dl, B * 4));
  CK(hipMemcpy(dq, hq.data(), hq.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dg, hg.data(), nh * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dr, hr.data(), hr.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dl, hl.data(), B * 4, hipMemcpyHostToDevice));
  float ms[3] = {0, 0, 0};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int k = 0; k < 3; ++k) {
    CK(hipMemset(dout[k], 0, ob));
    AttnArgs a{};
    a.qkv = dq;
    a.out = dout[k];
    a.T = T, a.H = H, a.nh = nh, a.ldq = ldq;
    a.scale = 0.125f;
    a.gconst = dg, a.relb = dr, a.maxd = maxd;
    a.tlen = ragged ? dl : nullptr;
    g_pipe = k;
    int rc = h16 ? launch_attention<f16>(a, B, 0) : launch_attention<bf16>(a, B, 0);
    CK(hipDeviceSynchronize());
    if (rc) {
      std::printf("launch rc %d\n", rc);
      return 1;
    }
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r) (void)(h16 ? launch_attention<f16>(a, B, 0) : launch_attention<bf16>(a, B, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms[k], e0, e1));
    ms[k] /= reps;
  }
  if (!h16 && !ragged && T == 149 && B >= 128) {   // where a head's time goes: loads only / compute only
    AttnArgs a{};
    a.qkv = dq, a.out = dout[1], a.T = T, a.H = H, a.nh = nh, a.ldq = ldq, a.scale = 0.125f;
    a.gconst = dg, a.relb = dr, a.maxd = maxd;
    float md[2];
    for (int d = 0; d < 2; ++d) {
      auto go = [&] { return d == 0 ? launch_attention_pipe<true, 10, false, false, 1>(a, B, 0)
                                    : launch_attention_pipe<true, 10, false, false, 2>(a, B, 0); };
      (void)go();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, 0));
      for (int r = 0; r < reps; ++r) (void)go();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&md[d], e0, e1));
      md[d] /= reps;
    }
    std::printf("  pipe B=%d: loads+waits only %.2f us, compute only %.2f us\n", B, 1e3 * md[0], 1e3 * md[1]);
    CK(hipMemset(dout[1], 0, ob));
    g_pipe = 1;
    (void)launch_attention<bf16>(a, B, 0);
    CK(hipDeviceSynchronize());   // (dout[1] restored for the comparison)
  }
  std::vector<uint16_t> o0(ob / 2), o1(ob / 2);
  CK(hipMemcpy(o0.data(), dout[0], ob, hipMemcpyDeviceToHost));
  long long bad[3] = {0, 0, 0};
  for (int k = 1; k < 3; ++k) {
    CK(hipMemcpy(o1.data(), dout[k], ob, hipMemcpyDeviceToHost));
    int shown = 0;
    for (int b = 0; b < B; ++b)
      for (int t = 0; t < hl[b]; ++t)
        for (int c = 0; c < H; ++c) {
          const size_t i = ((size_t)b * T + t) * H + c;
          if (o0[i] != o1[i]) {
            if (shown < 8) {
              std::printf("  mismatch (pipe %d) clip %d row %d head %d col %d: %04x vs %04x\n", k, b, t, c / 64, c % 64, o0[i],
                          o1[i]);
              ++shown;
            }
            ++bad[k];
          }
        }
  }
  std::printf("B=%d T=%d %s%s: full %.2f us, pipe %.2f us, pipe2 %.2f us, mismatches %lld / %lld\n", B, T,
              h16 ? "fp16" : "bf16", ragged ? " ragged" : "", 1e3 * ms[0], 1e3 * ms[1], 1e3 * ms[2], bad[1], bad[2]);
  CK(hipFree(dq));
  CK(hipFree(dout[0]));
  CK(hipFree(dout[1]));
  CK(hipFree(dout[2]));
  CK(hipFree(dg));
  CK(hipFree(dr));
  CK(hipFree(dl));
  return bad[1] || bad[2] ? 1 : 0;
}

int main() {
  int fails = 0;
  fails += run(6, 149, false, false, 3);
  fails += run(6, 49, false, false, 3);
  fails += run(7, 149, false, true, 3);
  fails += run(128, 149, false, false, 20);
  fails += run(256, 149, false, false, 20);
  fails += run(128, 149, true, false, 20);
  fails += run(48, 149, false, true, 5);
  fails += run(256, 149, true, true, 10);
  std::printf("%s\n", fails ? "DIFFER" : "all identical");
  return 0;
}
