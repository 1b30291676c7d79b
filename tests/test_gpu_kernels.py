"""Kernel-level numerics: the MFMA GEMM (all epilogue variants, ragged M, K tails) against a
plain PyTorch fp32 reference of the same op."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(a, b, bias, resid, act):
    y = a.float() @ b.float().T
    if bias is not None:
        y = y + bias
    if act in ("gelu", "gelu_fast"):
        y = torch.nn.functional.gelu(y)
    if resid is not None:
        y = y + resid
    return y


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(1, 128, 64), (149, 768, 768), (1000, 512, 1536), (4099, 256, 3072),
                                   (300, 64, 40), (77, 48, 96), (2048, 2432, 768), (5000, 2560, 200),
                                   (4096, 768, 3072)])
@pytest.mark.parametrize("epi", ["plain", "bias_gelu", "bias_resid"])
def test_gemm_vs_torch(dtype, M, N, K, epi):
    from ssr_amd.model import gemm
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K)
    a = torch.randn(M, K, device="cuda", generator=g).to(dtype)
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(dtype)
    bias = torch.randn(N, device="cuda", generator=g) if epi != "plain" else None
    resid = torch.randn(M, N, device="cuda", generator=g) if epi == "bias_resid" else None
    act = "gelu" if epi == "bias_gelu" else None
    got = gemm(a, b, bias, resid, act)
    ref = _ref(a, b, bias, resid, act)
    err = ((got - ref).norm() / ref.norm()).item()
    tol = 1e-6 if dtype == torch.float32 else 1e-5      # bf16 operands are exact in fp32; only sums differ
    assert err <= tol, err
    if dtype == torch.bfloat16:
        gt = gemm(a, b, bias, resid, act, out_dtype=torch.bfloat16)
        assert ((gt.float() - ref).norm() / ref.norm()).item() <= 5e-3


def test_gemm_rejects_bad_shapes():
    from ssr_amd.model import gemm
    a = torch.randn(10, 30, device="cuda")       # K % 4 != 0 for fp32 chunks is allowed only if K%4==0
    b = torch.randn(100, 30, device="cuda")      # N = 100: no tile config
    with pytest.raises(Exception):
        gemm(a, b)


@pytest.mark.parametrize("M,N,K", [(4099, 512, 768), (8192, 768, 3072), (4100, 2560, 136), (4133, 768, 64),
                                   (5000, 256, 128), (6000, 512, 192), (4096, 256, 256)])
def test_gemm_tile_configs_agree(M, N, K):
    """The default (8-phase ping-pong 256x256 where it applies), the 128x128 tile (gemm_cfg=1),
    the 256x128 3-stage ring (gemm_cfg=2) and the 2-stage 256x256 kernel (gemm_cfg=3) accumulate every output
    in the same K order: results are bit-identical (K-tile counts 1, 2, 3, 4, 12, 48 cover the
    8-phase prologue / steady / tail paths)."""
    from ssr_amd import _lib
    from ssr_amd.model import gemm
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    resid = torch.randn(M, N, device="cuda", generator=g)
    outs = []
    for cfg in (0, 1, 2, 3):
        with _lib.option("gemm_cfg", cfg):
            outs.append(gemm(a, b, bias, resid, None))
    ref = _ref(a, b, bias, resid, None)
    for o in outs:
        assert ((o - ref).norm() / ref.norm()).item() <= 1e-5
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2]) and torch.equal(outs[0], outs[3])


@pytest.mark.parametrize("M,N,K", [(149, 768, 768), (4099, 3072, 768), (1000, 512, 1536)])
def test_gemm_fast_gelu_epilogue(M, N, K):
    """The bf16 path's GELU (gelu_fast2: clamped odd minimax polynomial for Phi, no transcendental)
    in the GEMM epilogue against torch's exact erf-GELU: fp32 output within 5e-5 rel-L2 on N(0, 4)
    pre-activations (the fp32 restatement tools/fit_gelu.py gives 1.7e-5), bf16 output within the
    bf16 rounding bar."""
    from ssr_amd.model import gemm
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = (2.0 * torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()   # pre-acts ~N(0, 4)
    bias = torch.randn(N, device="cuda", generator=g)
    ref = _ref(a, b, bias, None, "gelu")
    got = gemm(a, b, bias, None, "gelu_fast")
    assert ((got - ref).norm() / ref.norm()).item() <= 5e-5
    gt = gemm(a, b, bias, None, "gelu_fast", out_dtype=torch.bfloat16)
    assert ((gt.float() - ref).norm() / ref.norm()).item() <= 5e-3


def test_fast_gelu_pointwise():
    """gelu_fast2 over a dense grid through the GEMM (a = x, b = 1, K = 64 with one non-zero
    column) against fp64 erf: max abs error <= 1e-4 (fit: 7.3e-5, tools/fit_gelu.py), relative
    <= 1e-4 for x >= 0.5, relu beyond the clamp (Phi(4.5) = 1 exactly, Phi(-4.5) = 3e-8)."""
    from ssr_amd.model import gemm
    x = torch.linspace(-12, 12, 256 * 1024, dtype=torch.float64)
    a = torch.zeros(x.numel(), 64, dtype=torch.float32)
    a[:, 0] = x.float()
    b = torch.zeros(256, 64, dtype=torch.float32)
    b[:, 0] = 1.0
    # fp32 operands (exact-f32 MFMA): pre-activation = x exactly; the epilogue is shared code
    got = gemm(a.cuda(), b.cuda(), None, None, "gelu_fast")[:, 0].double().cpu()
    xe = a[:, 0].double()
    ref = xe * 0.5 * (1.0 + torch.erf(xe / 2 ** 0.5))
    err = (got - ref).abs()
    assert err.max().item() <= 1e-4, err.max().item()
    m = xe >= 0.5
    assert (err[m] / ref[m].abs()).max().item() <= 1e-4
    assert torch.equal(got[xe > 4.5], xe[xe > 4.5].float().double())   # Phi(4.5) = 1 exactly
    neg = xe < -4.5
    assert (got[neg].abs() <= 1e-7 * xe[neg].abs()).all()              # Phi(-4.5) = 3e-8


def test_fast_gelu_pointwise_bf16_out():
    """A bf16-only output takes the degree-6 form (common.h gelu_bf2: clamp 4, max abs error 2.2e-4,
    1/18 of the bf16 half-ulp at |y| = 1): every bf16 x in [-12, 12] through the persistent GEMM
    (b = 1 in one K column, so the pre-activation is x exactly) against the fp32 restatement below
    (fused multiply-adds as on the GPU), rounded to bf16 -- equal up to one bf16 step where the fp64
    emulation of an fp32 fma double-rounds -- and against fp64 erf within the fit error plus half a
    bf16 ulp."""
    from ssr_amd.model import gemm
    x = torch.unique(torch.linspace(-12, 12, 1 << 20).bfloat16().float())
    M = x.numel()
    a = torch.zeros(M, 64, dtype=torch.bfloat16)
    a[:, 0] = x.bfloat16()
    b = torch.zeros(256, 64, dtype=torch.bfloat16)
    b[:, 0] = 1.0
    got = gemm(a.cuda(), b.cuda(), None, None, "gelu_fast", out_dtype=torch.bfloat16)[:, 0].float().cpu()
    c = [2.368073737e-08, -1.652635206e-06, 4.923747110e-05, -8.292031125e-04, 8.865549229e-03,
         -6.484667212e-02, 3.981720209e-01]

    def fma32(a, b, d):   # fp32 fused multiply-add: the fp64 product of two fp32 values is exact
        return (a.double() * b.double() + d.double()).float()

    xc = x.clamp(-4.0, 4.0)
    s = xc * xc
    p = torch.full_like(x, c[0])
    for k in c[1:]:
        p = fma32(p, s, torch.full_like(x, k))
    poly = (x * fma32(xc, p, torch.full_like(x, 0.5))).bfloat16().float()
    step = (got.view(torch.int32) - poly.view(torch.int32)).abs() >> 16   # bf16 code distance
    step[got == poly] = 0                                                  # -0 == +0
    assert (step <= 1).all() and (step == 0).float().mean().item() >= 0.999
    xd = x.double()
    ref = xd * 0.5 * (1.0 + torch.erf(xd / 2 ** 0.5))
    half_ulp = torch.ldexp(torch.ones_like(ref), torch.frexp(ref.abs())[1] - 9)   # bf16: 8 mantissa bits
    assert ((got.double() - ref).abs() <= 2.2e-4 + half_ulp).all()
    assert torch.equal(got[x > 4.0], x[x > 4.0])   # Phi(4) = 1 exactly


@pytest.mark.parametrize("M,N,K", [(16421, 1024, 64), (16421, 1024, 128), (16421, 768, 192), (16384, 1024, 256),
                                   (16421, 1024, 768), (9000, 2560, 768), (300, 512, 512)])
@pytest.mark.parametrize("epi", ["plain", "bias_gelu_fast", "bias_f32_and_bf16"])
def test_gemm_persistent_agrees(M, N, K, epi):
    """The persistent 8-phase kernel (default for GEMMs without a residual: blocks walk several
    tiles, the next tile's prologue is issued before this tile's stores, which stay in flight)
    against its round-1..5 four-phase schedule (gemm_4phase=1; the default runs two 32-MFMA phases per
    K-tile), the non-persistent kernel (gemm_nonpersist=1) and the 2-stage kernel (gemm_cfg=3):
    bit-identical.  Tile counts above the CU count, ragged M, K-tile counts 1, 2, 3, 4, 12 and every
    output combination."""
    from ssr_amd.model import gemm
    from ssr_amd import _lib
    import ctypes
    g = torch.Generator(device="cuda").manual_seed(M + N + 7 * K)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g) if epi != "plain" else None
    act = "gelu_fast" if epi == "bias_gelu_fast" else None

    def run():
        if epi != "bias_f32_and_bf16":
            return (gemm(a, b, bias, None, act, out_dtype=torch.bfloat16),)
        cf = torch.empty(M, N, device="cuda")
        ct = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        z = torch.zeros(64, device="cuda")
        _lib.check(_lib.lib().sse_gemm(_lib.SSE_DTYPE_BF16, a.data_ptr(), b.data_ptr(), bias.data_ptr(), None,
                                       cf.data_ptr(), ct.data_ptr(), M, N, K, 0, z.data_ptr(),
                                       ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "sse_gemm")
        return cf, ct

    outs = []
    for name, v in (("gemm_cfg", 0), ("gemm_4phase", 1), ("gemm_nonpersist", 1), ("gemm_cfg", 3)):
        with _lib.option(name, v):
            outs.append(run())
            torch.cuda.synchronize()
    ref = _ref(a, b, bias, None, "gelu" if act else None)
    assert ((outs[0][0].float() - ref).norm() / ref.norm()).item() <= 5e-3
    for o in outs[1:]:
        for x, y in zip(outs[0], o):
            assert torch.equal(x, y)


@pytest.mark.parametrize("M,N,act", [(40704, 2560, 0), (40704, 3072, 2), (11448, 2560, 0)])
def test_lnfold_gemm_position_invariant(M, N, act):
    """The folded-LayerNorm GEMM (sse_gemm_lnfold, the bf16 post-LN path's QKV / FFN1): the persistent
    kernel equals the non-persistent one bit for bit, and a row's result does not depend on its
    position inside a 256-row tile (rows shifted by 128 and by whole tiles give the same bits).  Before
    the library was built with -ffp-contract=off, instances of the LayerNorm-statistics expression
    were contracted differently per tile position and 1-ulp bf16 flips appeared in ~4 % of clips."""
    import ctypes
    from ssr_amd import _lib
    L = _lib.lib()
    g = torch.Generator(device="cuda").manual_seed(3)
    K = 768
    a = (torch.randn(M, K, device="cuda", generator=g) * 2 + 0.3).bfloat16()
    b = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g) * 0.1
    acol = b.float().sum(1)
    af = a.float().view(M, 3, 256)
    mean = af.mean(2)
    part = torch.stack([mean, ((af - mean[..., None]) ** 2).sum(2)], -1).contiguous()
    z = torch.zeros(64, device="cuda")

    def run(a_, part_, nonpersist=0):
        ct = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        with _lib.option("gemm_nonpersist", nonpersist):
            rc = L.sse_gemm_lnfold(a_.data_ptr(), b.data_ptr(), bias.data_ptr(), acol.data_ptr(), part_.data_ptr(),
                                   ct.data_ptr(), M, N, K, act, ctypes.c_float(1e-5), z.data_ptr(),
                                   ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0
        return ct
    p = run(a, part)
    assert torch.equal(p, run(a, part, 1))
    for sh in (128, 256 * 43 + 64):
        q = torch.roll(run(torch.roll(a, sh, 0), torch.roll(part, sh, 0)), -sh, 0)
        assert torch.equal(p, q), sh
    # and against a torch fp32 restatement of the fold (bf16 output: within one bf16 ulp-scale)
    rstd = 1.0 / torch.sqrt(part[..., 1].sum(1) / 768 + ((part[..., 0] - part[..., 0].mean(1, keepdim=True)) ** 2).sum(1)
                            * 256 / 768 + 1e-5)
    ref = rstd[:, None] * (a.float() @ b.float().T) + bias - (rstd * part[..., 0].mean(1))[:, None] * acol
    if act == 2:
        ref = torch.nn.functional.gelu(ref)
    assert ((p.float() - ref).abs() <= 1e-2 * ref.abs() + 2e-2).all()


@pytest.mark.parametrize("model,dtype,B,L", [("wavlm-base", "bf16", 5, 48000), ("whisper-small", "fp8", 2, 480000),
                                             ("wavlm-large", "bf16", 3, 48000)])
def test_gemm_schedules_bit_identical_in_model(model, dtype, B, L):
    """The 8-wave GEMMs' K-tile schedules (option gemm_4phase: 0 = two 32-MFMA phases per K-tile, the default;
    1 = four 16-MFMA phases) give every accumulator the same K-steps in the same order: whole-model embeddings are
    bit-identical across them (every GEMM form the model runs: conv, fold + GELU, residual stream with partials,
    MX QKV / fc1 / fc2)."""
    from ssr_amd import _lib, config as C, synth
    from ssr_amd.model import SSEModel
    spec = {"wavlm-base": C.WAVLM_BASE, "whisper-small": C.WHISPER_SMALL, "wavlm-large": C.WAVLM_LARGE}[model]
    m = SSEModel(spec, synth.synth_state_dict(spec), device="cuda:0", dtype=dtype)
    w = torch.from_numpy(synth.synth_clips(B, L, seed=B + 1)).cuda()
    idx = spec.default_layer_indices()
    ref = m.embed(w, idx)
    with _lib.option("gemm_4phase", 1):
        assert torch.equal(m.embed(w, idx), ref)
