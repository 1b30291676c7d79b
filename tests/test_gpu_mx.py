"""GPU parity of the MX-fp8 path (SSE_DTYPE_FP8, BASELINE configs[4] "Whisper-large fp8 MFMA
encoder"): the device quantisers and the MX GEMM against the numpy restatement (oracle/mx.py),
then the fp8 Whisper encoder end to end.

Tolerances (written here, stated in DESIGN.md §4):
* quantisation (GPU kernel, LayerNorm / GEMM-epilogue producers): bit-identical codes and scales to
  the restatement applied to the same fp32 values;
* MX GEMM: error <= 1e-4 of max|C| against the fp64 product of the dequantised operands (measured
  1.6-2.9e-5: v_mfma_scale_f32_16x16x128_f8f6f4 does not round like an fp32 fma chain over its 128
  products; the bf16 kernels' bar is 1e-5);
* fp8 encoder embeddings vs the fp32 oracle / the reference's fixture: rel-L2 <= 0.08 and cosine
  >= 0.995 (e4m3 keeps 3 mantissa bits: ~2^-5 relative error per operand element; the bf16 path's
  bar is 3e-2; round 4 tightened from 0.12 / 0.99 against the observed <= 0.067).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import mx

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return np.linalg.norm(a - b, axis=-1) / np.linalg.norm(b, axis=-1)


def _cos(a, b):
    return np.sum(a * b, axis=-1) / (np.linalg.norm(a, axis=-1) * np.linalg.norm(b, axis=-1))


@pytest.mark.parametrize("role", [0, 1])
def test_gpu_quantiser_matches_restatement(role):
    from ssr_amd.model import mx_quantize, mx_quantize_host
    rng = np.random.default_rng(10 + role)
    R, K = 700, 1280
    x = (rng.standard_normal((R, K)) * np.exp(rng.uniform(-6, 6, (R, 1)))).astype(np.float32)
    x[3] = 0.0
    q, sc = mx_quantize(torch.from_numpy(x).cuda(), role)
    qh, sch = mx_quantize_host(x, role)
    assert np.array_equal(q.cpu().numpy(), qh)
    assert np.array_equal(mx.exps_from_scales(sc.cpu().numpy(), R, K, role), mx.exps_from_scales(sch, R, K, role))


@pytest.mark.parametrize("R,H", [(300, 1280), (257, 768), (64, 512), (131, 384)])
def test_layernorm_mx_producer(R, H):
    """The LN -> MX-fp8 producer of the fp8 encoder (layernorm_mx8_kernel via the sse_layernorm_mx hook): its codes
    and scales against oracle/mx.py applied to an fp32 LayerNorm of the same bf16 rows.  The kernel's fp32 statistics
    sum in a different order than numpy, so a value next to a rounding boundary may take the neighbouring code: >= 99.5 %
    of codes equal, >= 99.9 % within one code, >= 99.5 % of scales equal.  Round 6 stores chunk pairs as 16-B stores (lane
    pairs swap 8-B pieces): H = 1280 (3 chunks: a pair + a lone partial chunk), 768 (a pair with a partial chunk),
    512 (a lone full chunk), 384 (a lone partial chunk) -- a misplaced piece would break whole 8-byte runs."""
    import ctypes
    from ssr_amd import _lib
    from ssr_amd.model import mx_scale_bytes
    rng = np.random.default_rng(R + H)
    x = (rng.standard_normal((R, H)) * 2.0 + rng.standard_normal((R, 1)) * 3.0).astype(np.float32)
    xb = torch.from_numpy(x).to(torch.bfloat16)
    w = (1.0 + 0.2 * rng.standard_normal(H)).astype(np.float32)
    b = (0.1 * rng.standard_normal(H)).astype(np.float32)
    q = torch.full((R + 8, H), 0xA5, dtype=torch.uint8, device="cuda")
    sc = torch.zeros(mx_scale_bytes(R, H), dtype=torch.uint8, device="cuda")
    xd, wd, bd = xb.cuda(), torch.from_numpy(w).cuda(), torch.from_numpy(b).cuda()
    rc = _lib.lib().sse_layernorm_mx(xd.data_ptr(), wd.data_ptr(), bd.data_ptr(), R, H, ctypes.c_float(1e-5),
                                     q.data_ptr(), sc.data_ptr(), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    _lib.check(rc, "sse_layernorm_mx")
    torch.cuda.synchronize()
    assert bool((q[R:] == 0xA5).all()), "store past row R"
    xf = xb.float().numpy().astype(np.float64)
    mean = xf.mean(1, keepdims=True)
    var = ((xf - mean) ** 2).mean(1, keepdims=True)
    ln = (((xf - mean) / np.sqrt(var + 1e-5)) * w + b).astype(np.float32)
    q0, _, e0 = mx.quantize(ln, 0)
    qg = q[:R].cpu().numpy()
    assert (qg == q0).mean() >= 0.995
    assert (np.abs(qg.astype(np.int16) - q0.astype(np.int16)) <= 1).mean() >= 0.999   # sign-magnitude codes
    assert (mx.exps_from_scales(sc.cpu().numpy(), R, H, 0) == e0).mean() >= 0.995


def _operands(M, N, K, seed):
    rng = np.random.default_rng(seed)
    a = rng.standard_normal((M, K)).astype(np.float32)
    b = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float32)
    qa, sa, ea = mx.quantize(a, 0)
    qb, sb, eb = mx.quantize(b, 1)
    A = mx.dequantize(qa, ea)
    B = mx.dequantize(qb, eb)
    dev = lambda v: torch.from_numpy(v).cuda()
    return (dev(qa), dev(sa), dev(qb), dev(sb)), A, B


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (300, 512, 256), (1000, 768, 1280), (257, 256, 5120),
                                   (2048, 3840, 384)])
def test_gemm_mx_matches_dequantised_product(M, N, K):
    from ssr_amd.model import gemm_mx
    ops, A, B = _operands(M, N, K, seed=M + N + K)
    rng = np.random.default_rng(1)
    bias = rng.standard_normal(N).astype(np.float32)
    resid = rng.standard_normal((M, N)).astype(np.float32)
    ref = A @ B.T
    got = gemm_mx(*ops).cpu().numpy()
    scale = np.abs(ref).max()
    err = np.abs(got - ref).max() / scale
    print("gemm_mx", M, N, K, "max rel err", err)
    assert err <= 1e-4
    got = gemm_mx(*ops, bias=torch.from_numpy(bias).cuda(), resid=torch.from_numpy(resid).cuda()).cpu().numpy()
    assert np.abs(got - (ref + bias + resid)).max() / scale <= 1e-4
    # bf16 output = the fp32 result rounded (same accumulation)
    f = gemm_mx(*ops, bias=torch.from_numpy(bias).cuda())
    h = gemm_mx(*ops, bias=torch.from_numpy(bias).cuda(), out="bf16")
    assert torch.equal(f.to(torch.bfloat16), h)


@pytest.mark.parametrize("act", ["gelu", "gelu_fast"])
def test_gemm_mx_fp8_output_is_the_quantised_result(act):
    """Ct in MX-fp8 (the fc1 -> fc2 hand-off): bytes and scales equal the restatement's
    quantisation of the same GEMM's fp32 result (A layout, K = N)."""
    from ssr_amd.model import gemm_mx
    M, N, K = 600, 1024, 256
    ops, A, B = _operands(M, N, K, seed=7)
    bias = torch.from_numpy(np.random.default_rng(3).standard_normal(N).astype(np.float32)).cuda()
    f = gemm_mx(*ops, bias=bias, act=act).cpu().numpy()
    q, sc = gemm_mx(*ops, bias=bias, act=act, out="fp8")
    if act == "gelu_fast":
        # the fp8-out epilogue uses the lower-degree GELU (common.h gelu_fp8out2, max abs error 8.2e-4,
        # below the e4m3 half-step): restated here from the pre-activation, so the bytes agree except
        # where the two evaluations (fused fma on the GPU, numpy here) straddle an e4m3 rounding boundary
        # (observed: 0.7 % of the bytes, each one e4m3 step)
        import sys, os
        sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
        from fit_gelu import gelu_fast as gelu_poly
        coef = np.array([3.963519037e-01, -6.208017841e-02, 7.574830670e-03, -5.630472442e-04, 2.229058919e-05,
                         -3.503167250e-07])
        z = gemm_mx(*ops, bias=bias, act=None).cpu().numpy()
        q0, _, e0 = mx.quantize(gelu_poly(z, coef, 3.5), 0)
        qg = q.cpu().numpy().copy()
        qg[qg == 0x80] = 0   # -0 (tails past the clamp: x Phi(-3.5) < 0) equals +0
        q0 = q0.copy()
        q0[q0 == 0x80] = 0
        assert (qg == q0).mean() >= 0.98
        assert (np.abs(qg.astype(np.int16) - q0.astype(np.int16)) <= 1).mean() >= 0.999   # sign-magnitude codes
        assert (mx.exps_from_scales(sc.cpu().numpy(), M, N, 0) == e0).mean() >= 0.995
        assert np.abs(gelu_poly(z, coef, 3.5) - f).max() <= 1e-3 * max(1.0, np.abs(z).max())
        return
    q0, _, e0 = mx.quantize(f, 0)
    assert np.array_equal(q.cpu().numpy(), q0)
    assert np.array_equal(mx.exps_from_scales(sc.cpu().numpy(), M, N, 0), e0)
    if act == "gelu":
        from scipy.special import erf
        z = A @ B.T + bias.cpu().numpy()
        g = 0.5 * z * (1 + erf(z / np.sqrt(2)))
        assert np.abs(f - g).max() <= 1e-4 * np.abs(z).max()


def test_gemm_mx_rejects_bad_shapes():
    from ssr_amd._lib import SSEError
    from ssr_amd.model import gemm_mx
    ops, _, _ = _operands(64, 256, 128, seed=1)
    q, s = mx.quantize(np.ones((100, 128), np.float32), 1)[:2]
    with pytest.raises(SSEError):
        gemm_mx(ops[0], ops[1], torch.from_numpy(q).cuda(), torch.from_numpy(s).cuda())   # N = 100


def _mx_spec():
    from ssr_amd import config as C
    return C.WhisperSpec(d_model=512, layers=3, heads=8, ffn=2048, name="whisper-mx-test")


def test_whisper_fp8_encoder_vs_oracle():
    """fp8 encoder (LayerNorm -> MX operand, MX QKV / fc1 (MX out) / fc2) vs the fp32 oracle; the
    bf16 build of the same weights for scale; every hidden state through sse_hidden_states too."""
    from ssr_amd import synth
    from ssr_amd.model import SSEModel
    from oracle.whisper import WhisperOracle
    spec = _mx_spec()
    sd = synth.synth_whisper_state_dict(spec, seed=21)
    clips = synth.synth_clips(2, 48000, seed=99)
    idx = [spec.layers, spec.layers - 1, 1, 0]
    ref = WhisperOracle(spec, sd).embed(clips, idx)
    res = {}
    for dtype in ("bf16", "fp8"):
        m = SSEModel(spec, sd, device="cuda:0", dtype=dtype)
        got = m.embed(torch.from_numpy(clips).cuda(), idx).cpu().numpy()
        res[dtype] = got
        print(dtype, "rel-L2", _rel(got, ref).max(), "cos", _cos(got, ref).min())
        del m
    assert np.isfinite(res["fp8"]).all()
    assert _rel(res["fp8"], ref).max() <= 0.08 and _cos(res["fp8"], ref).min() >= 0.995
    # hidden_states[0] (conv front end, bf16 in both) is identical in the two builds
    assert np.array_equal(res["fp8"][:, 3], res["bf16"][:, 3])
    # batch independence: clip 1 alone == clip 1 in the batch
    m = SSEModel(spec, sd, device="cuda:0", dtype="fp8")
    one = m.embed(torch.from_numpy(clips[1:2]).cuda(), idx).cpu().numpy()
    assert np.array_equal(one[0], res["fp8"][1])


@pytest.mark.slow
def test_whisper_large_v2_fp8_vs_reference_fixture():
    p = os.path.join(GOLDEN, "whisper_large_v2.npz")
    if not os.path.exists(p):
        pytest.skip("large-v2 fixture not generated")
    from ssr_amd import config as C, synth
    from ssr_amd.model import SSEModel
    g = np.load(p)
    clip = synth.synth_clips(1, 48000, seed=4321, first_clip=0)[0]
    sd = synth.synth_whisper_state_dict(C.WHISPER_LARGE_V2, seed=11)
    idx = [int(i) for i in g["layer_indices"]]
    m = SSEModel(C.WHISPER_LARGE_V2, sd, device="cuda:0", dtype="fp8")
    got = m.embed(torch.from_numpy(clip).cuda(), idx).cpu().numpy()[0]
    rel, cos = _rel(got, g["emb"][0]).max(), _cos(got, g["emb"][0]).min()
    print("fp8 whisper-large-v2 rel-L2", rel, "cos", cos)
    assert rel <= 0.08 and cos >= 0.995

