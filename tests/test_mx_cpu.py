"""CPU checks of the MX-fp8 operand format (SSE_DTYPE_FP8, BASELINE configs[4]): the numpy
restatement (oracle/mx.py) against an exhaustive nearest-even search, and libsse.so's host weight
quantiser (sse_mx_quantize_host, what sse_model_create applies) against the restatement, bit for
bit.  The GPU quantisers are pinned to the same bytes in tests/test_gpu_mx.py."""
import ctypes

import numpy as np
import pytest

from oracle import mx


def _all_e4m3():
    codes = np.arange(256, dtype=np.uint8)
    v = mx.e4m3_decode(codes)
    ok = ~np.isnan(v)
    return codes[ok], v[ok]


def test_e4m3_encode_is_round_to_nearest_even():
    codes, vals = _all_e4m3()
    # every finite code round-trips (the two zeros keep their sign)
    assert np.array_equal(mx.e4m3_encode(vals), codes)
    pos = np.unique(vals[vals >= 0])
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-448, 448, 20000), rng.standard_normal(20000) * 1e-2,
                        (pos[1:] + pos[:-1]) / 2, -(pos[1:] + pos[:-1]) / 2])   # midpoints: ties
    got = mx.e4m3_encode(x)
    dv = mx.e4m3_decode(got)
    # nearest representable, ties to the even code
    d = np.abs(pos[None, :] - np.abs(x)[:, None])
    best = d.min(axis=1)
    assert np.all(np.abs(np.abs(dv) - np.abs(x)) <= best + 0.0)
    tie = np.isclose(np.abs(x)[:, None], (pos[1:] + pos[:-1])[None, :] / 2, rtol=0, atol=0).any(axis=1)
    assert np.all((got[tie] & 1) == 0)


def test_scale_exponent_never_saturates():
    rng = np.random.default_rng(1)
    amax = np.abs(rng.standard_normal(10000).astype(np.float32)) * np.float32(10.0) ** rng.integers(-20, 20, 10000)
    eb = mx.scale_exp(amax).astype(np.int64)
    scaled = amax.astype(np.float64) * np.ldexp(1.0, 127 - eb)
    assert np.all(scaled <= 448.0)
    assert np.all(scaled > 224.0)          # and is the smallest such exponent
    assert mx.scale_exp(np.float32(0.0)) == 0


def test_scale_layouts_are_bijective():
    from ssr_amd import _lib
    L = _lib.lib()
    for K in (128, 1280):
        R = 512
        r, b = np.meshgrid(np.arange(R), np.arange(K // 32), indexing="ij")
        for role, fn in ((0, mx.a_scale_off), (1, mx.b_scale_off)):
            off = fn(r, b, K // 128).ravel()
            assert len(np.unique(off)) == off.size == mx.scale_bytes(R, K)
            assert off.min() == 0 and off.max() == off.size - 1
            for rr, bb in ((0, 0), (17, 3), (300, K // 32 - 1), (511, 5)):
                bb = bb % (K // 32)
                assert L.sse_mx_scale_offset(role, rr, bb, K) == fn(rr, bb, K // 128)
        assert L.sse_mx_scale_bytes(R, K) == mx.scale_bytes(R, K)
    assert L.sse_mx_scale_bytes(10, 100) == 0 and L.sse_mx_scale_offset(0, 0, 0, 100) == -1


@pytest.mark.parametrize("role", [0, 1])
def test_host_quantiser_matches_restatement(role):
    from ssr_amd.model import mx_quantize_host
    rng = np.random.default_rng(2 + role)
    R, K = 300, 384
    x = rng.standard_normal((R, K)).astype(np.float32)
    x[0] = 0.0                                          # all-zero blocks
    x[1, :32] = 1e-30                                   # tiny block
    x[2] *= 1e4
    x[3, ::7] = 448.0 * 2.0 ** -3                       # exact powers / boundaries
    x[4] = np.float32(2.0 ** -12) * rng.standard_normal(K).astype(np.float32)   # e4m3 subnormals after scaling
    q, sc = mx_quantize_host(x, role)
    q0, sc0, eb = mx.quantize(x, role)
    assert np.array_equal(q, q0)
    assert np.array_equal(mx.exps_from_scales(sc, R, K, role), eb)
    # in each block's scaled units y = x * 2^-E the error is at most half an e4m3 step of |y|
    y = x.reshape(R, K // 32, 32).astype(np.float64) * np.ldexp(1.0, 127 - eb.astype(np.int64))[:, :, None]
    ulp = np.ldexp(1.0, np.maximum(np.floor(np.log2(np.maximum(np.abs(y), 1e-300))), -6).astype(np.int64) - 3)
    err = np.abs(mx.e4m3_decode(q0).reshape(R, K // 32, 32) - y)
    assert np.all(err <= ulp / 2)


def test_fp8_model_config_rules():
    """SSE_DTYPE_FP8 is the Whisper encoder mode and needs 256-multiples (MX GEMM tile)."""
    from ssr_amd import _lib, config as C
    L = _lib.lib()
    for spec in (C.WAVLM_BASE, C.WHISPER_TINY):   # WavLM, and d_model 384 (not a 256 multiple)
        cfg = _lib.make_cfg(spec)
        n = L.sse_weight_floats(ctypes.byref(cfg))
        w = np.zeros(n, dtype=np.float32)
        h = ctypes.c_void_p()
        rc = L.sse_model_create(ctypes.byref(cfg), w.ctypes.data, w.nbytes, 0, _lib.SSE_DTYPE_FP8, ctypes.byref(h))
        assert rc == -3, spec.name
