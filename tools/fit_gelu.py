#!/usr/bin/env python3
"""Coefficients of gelu_fast2 (csrc/common.h), the bf16 path's GELU.

gelu(x) = x * Phi(x), Phi(x) = 1/2 + xc * R(xc^2), xc = clamp(x, -C, C).  R (degree DEG - 1 in s = x^2)
is the minimax fit (LP) of Phi(x) - 1/2 on 0 <= x <= C, weighted by max(x, 1) (the gelu error is
x times the Phi error), with R constrained so that Phi(C) = 1 exactly (beyond the clamp the form is
exactly relu).  No transcendental: the kernel evaluates 2 v_med3 + 11 packed-fp32 ops per pair.
Prints the coefficients (highest degree first, the Horner order of the kernel) and the error of an
fp32 evaluation against fp64 erf.
"""
import numpy as np
from scipy.optimize import linprog
from scipy.special import ndtr

C_CLAMP, DEG = 4.5, 9


def fit(c, n, npts=6000):
    x = np.linspace(0, c, npts)
    f = ndtr(x) - 0.5
    A = np.stack([x ** (2 * k + 1) for k in range(n)], 1)
    w = np.maximum(x, 1.0)
    Aub = np.vstack([np.hstack([A * w[:, None], -np.ones((npts, 1))]), np.hstack([-A * w[:, None], -np.ones((npts, 1))])])
    bub = np.concatenate([f * w, -f * w])
    Aeq = np.hstack([np.array([[c ** (2 * k + 1) for k in range(n)]]), [[0]]])
    r = linprog(np.r_[np.zeros(n), 1], A_ub=Aub, b_ub=bub, A_eq=Aeq, b_eq=[0.5], bounds=[(None, None)] * (n + 1),
                method="highs")
    return r.x[:n]


def gelu_fast(x, a, c=C_CLAMP):
    """fp32 restatement of gelu_fast2 (same operation order)."""
    x = np.asarray(x, np.float32)
    xc = np.clip(x, np.float32(-c), np.float32(c))
    s = (xc * xc).astype(np.float32)
    p = np.float32(a[-1])
    for k in reversed(range(len(a) - 1)):
        p = (p * s + np.float32(a[k])).astype(np.float32)
    return (x * (xc * p + np.float32(0.5))).astype(np.float32)


def nudge(a, c=C_CLAMP):
    """Move the constant coefficient by whole fp32 ulps so that the kernel's fp32 evaluation gives
    Phi(c) = 1 exactly and Phi(-c) as close to 0 as fp32 allows (beyond the clamp: relu)."""
    f32 = np.float32

    def fma(x, y, z):   # fp32 fma: the product of two fp32 values is exact in fp64
        return f32(np.float64(f32(x)) * np.float64(f32(y)) + np.float64(f32(z)))

    def phi(b, xc):
        s = f32(f32(xc) * f32(xc))
        p = b[-1]
        for k in range(len(b) - 2, -1, -1):
            p = fma(p, s, b[k])
        return fma(xc, p, 0.5)

    b = [f32(v) for v in a]
    best = None
    for k in range(-4000, 4001):
        cand = [np.int32(b[0].view(np.int32) + k).view(np.float32)] + b[1:]
        r = abs(float(phi(cand, -c))) + abs(float(phi(cand, c)) - 1.0)
        if best is None or r < best[0]:
            best = (r, cand)
    return np.array(best[1], np.float64)


def main():
    a = nudge(fit(C_CLAMP, DEG))
    print("coefficients (Horner order):", ", ".join("%.9e" % v for v in a[::-1]))
    x = np.linspace(-12, 12, 4000001).astype(np.float32)
    out = gelu_fast(x, a)
    ref = x.astype(np.float64) * ndtr(x.astype(np.float64))
    err = np.abs(out - ref)
    print("fp32 max abs err %.2e" % err.max())
    print("Phi(+-C) - (1, 0):", gelu_fast(np.float32(C_CLAMP), a) / C_CLAMP - 1, gelu_fast(np.float32(-C_CLAMP), a) / -C_CLAMP)


if __name__ == "__main__":
    main()
