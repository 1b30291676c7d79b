"""TEST INFRASTRUCTURE ONLY (checker, never shipped or measured): numpy restatement of the MX-fp8
operand format the SSE_DTYPE_FP8 Whisper path uses for its QKV / fc1 / fc2 GEMMs.

The reference computes these GEMMs in fp32 (HF/models/whisper/modeling_whisper.py:372-407 via
REF/whisper_embeddings_large.py:250-254); fp8 is this build's BASELINE configs[4] throughput mode,
so there is no reference golden for the quantised values themselves.  This module restates the
published formats the kernels implement, and the tests pin the GPU (and the host weight
quantiser) to it bit-exactly:

* OCP 8-bit floating point, E4M3 ("e4m3fn": bias 7, no infinities, max 448, subnormals
  m * 2^-9), conversion by round-to-nearest-even;
* OCP Microscaling (MX): blocks of 32 consecutive K elements share an E8M0 scale 2^E.  The block
  exponent is the smallest E with max|x| <= 448 * 2^E (so nothing saturates), clamped to
  [-127, 127]; an all-zero block gets E = -127.  Element = RNE_e4m3(x * 2^-E).
* the scale tensors' tile layouts (1 KiB per 256 rows x 128 K), restated from common.h
  mx_a_scale_off / mx_b_scale_off.
"""
from __future__ import annotations

import numpy as np

E4M3_MAX = 448.0


def e4m3_decode(codes: np.ndarray) -> np.ndarray:
    c = np.asarray(codes, dtype=np.uint8).astype(np.int32)
    s = np.where(c & 0x80, -1.0, 1.0)
    e = (c >> 3) & 15
    m = c & 7
    v = np.where(e == 0, np.ldexp(m / 8.0, -6), np.ldexp(1.0 + m / 8.0, e - 7))
    v = np.where((e == 15) & (m == 7), np.nan, v)
    return (s * v).astype(np.float64)


def e4m3_encode(y: np.ndarray) -> np.ndarray:
    """RNE to e4m3fn of |y| <= 448 (larger magnitudes saturate to 448)."""
    y = np.asarray(y, dtype=np.float64)
    sign = np.where(np.signbit(y), 0x80, 0).astype(np.uint8)
    a = np.minimum(np.abs(y), E4M3_MAX)
    out = np.zeros(a.shape, dtype=np.uint8)
    sub = a < 2.0 ** -6
    out[sub] = np.rint(a[sub] * 512.0).astype(np.uint8)              # np.rint: ties to even; 8 -> 0x08
    an = a[~sub]
    e = np.floor(np.log2(an)).astype(np.int64)
    # guard log2 rounding at exact powers of two
    e = np.where(np.ldexp(1.0, e) > an, e - 1, e)
    e = np.where(np.ldexp(1.0, e + 1) <= an, e + 1, e)
    m = np.rint(np.ldexp(an, 3 - e))                                  # in [8, 16]
    carry = m >= 16
    m = np.where(carry, 8, m)
    e = np.where(carry, e + 1, e)
    out[~sub] = ((e + 7) << 3 | (m.astype(np.int64) - 8)).astype(np.uint8)
    return out | sign


def scale_exp(amax: np.ndarray) -> np.ndarray:
    """Biased E8M0 byte of each block maximum (float32 amax, as the kernels hold it)."""
    a = np.asarray(amax, dtype=np.float32)
    bits = a.view(np.uint32).astype(np.int64)
    be = (bits >> 23) & 255
    mant = bits & 0x7FFFFF
    E = be - 127 - np.where(mant <= 0x600000, 8, 7)
    E = np.clip(E, -127, 127)
    return np.where(be == 0, 0, E + 127).astype(np.uint8)


def a_scale_off(m, blk, kt):
    m = np.asarray(m, dtype=np.int64)
    blk = np.asarray(blk, dtype=np.int64)
    return ((m >> 8) * kt + (blk >> 2)) * 1024 + ((((m >> 6) & 3) * 4 + (blk & 3)) * 16 + (m & 15)) * 4 + ((m >> 4) & 3)


def b_scale_off(n, blk, kt):
    n = np.asarray(n, dtype=np.int64)
    blk = np.asarray(blk, dtype=np.int64)
    return (((n >> 8) * kt + (blk >> 2)) * 1024 + ((((n >> 5) & 3) * 4 + (blk & 3)) * 16 + (n & 15)) * 4 +
            ((n >> 7) & 1) * 2 + ((n >> 4) & 1))


def scale_bytes(R: int, K: int) -> int:
    return ((R + 255) // 256) * (K // 128) * 1024


def quantize(x: np.ndarray, role: int = 0):
    """fp32 x [R][K] -> (e4m3 codes [R][K], scale tensor in the role's layout, per-block exponents
    [R][K/32] biased)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    R, K = x.shape
    assert K % 128 == 0
    blocks = x.reshape(R, K // 32, 32)
    eb = scale_exp(np.abs(blocks).max(axis=2))
    inv = np.ldexp(np.float32(1.0), 127 - eb.astype(np.int32)).astype(np.float32)   # exact 2^-E (fp32)
    y = blocks * inv[:, :, None]                                                       # exact scaling in fp32
    q = e4m3_encode(y).reshape(R, K)
    sc = np.full(scale_bytes(R, K), 0x7F, dtype=np.uint8)
    r, b = np.meshgrid(np.arange(R), np.arange(K // 32), indexing="ij")
    off = (b_scale_off if role else a_scale_off)(r, b, K // 128)
    sc[off.ravel()] = eb.ravel()
    return q, sc, eb


def dequantize(q: np.ndarray, eb: np.ndarray) -> np.ndarray:
    """codes [R][K] and block exponents [R][K/32] -> float64 values."""
    R, K = q.shape
    v = e4m3_decode(q).reshape(R, K // 32, 32)
    return (v * np.ldexp(1.0, eb.astype(np.int64) - 127)[:, :, None]).reshape(R, K)


def exps_from_scales(sc: np.ndarray, R: int, K: int, role: int = 0) -> np.ndarray:
    r, b = np.meshgrid(np.arange(R), np.arange(K // 32), indexing="ij")
    off = (b_scale_off if role else a_scale_off)(r, b, K // 128)
    return np.asarray(sc)[off]
