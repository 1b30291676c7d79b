#!/usr/bin/env python3
"""Coefficients of gelu_sig2 (csrc/common.h), the bf16 path's GELU.

gelu(x) = x * Phi(x), Phi(x) = 1 / (1 + 2^(x * P(min(x^2, c^2)))).  P (degree d in s = x^2) is the
linearised minimax fit (LP) of -log2(e) * logit(Phi(x)) / x on 0 < x <= c, weighted by the
sensitivity of gelu to the exponent.  Prints the coefficients (highest degree first, the Horner
order of the kernel) and the error of an fp32 evaluation against fp64 erf.
"""
import numpy as np
from scipy.optimize import linprog
from scipy.special import expit, logit, ndtr

C_CLAMP, DEG = 5.0, 6
L2E = 1.4426950408889634


def fit(c, d, n=8000):
    x = np.linspace(1e-3, c, n)
    s = x * x
    g = logit(ndtr(x)) / x
    sig = expit(x * g)
    w = x * x * sig * (1 - sig)                     # d gelu / d g
    V = np.vstack([s ** k for k in range(d + 1)]).T
    sc = np.abs(V).max(0)
    Vs = V / sc
    nv = d + 2
    cost = np.zeros(nv)
    cost[-1] = 1
    A = np.vstack([np.hstack([w[:, None] * Vs, -np.ones((n, 1))]), np.hstack([-w[:, None] * Vs, -np.ones((n, 1))])])
    b = np.concatenate([w * g, -w * g])
    r = linprog(cost, A_ub=A, b_ub=b, bounds=[(None, None)] * nv, method="highs")
    return r.x[:-1] / sc


def main():
    a = -fit(C_CLAMP, DEG) * L2E                    # exponent for exp2, sign folded in
    print("coefficients (Horner order):", ", ".join("%.9e" % v for v in a[::-1]))
    x = np.linspace(-12, 12, 4000001).astype(np.float32)
    s = np.minimum(x * x, np.float32(C_CLAMP ** 2))
    p = np.float32(a[-1])
    for k in reversed(range(len(a) - 1)):
        p = (p * s + np.float32(a[k])).astype(np.float32)
    u = (x * p).astype(np.float32)
    d = (np.exp2(u.astype(np.float64)).astype(np.float32) + np.float32(1)).astype(np.float32)
    out = (x * (1 / d).astype(np.float32)).astype(np.float32)
    ref = x.astype(np.float64) * ndtr(x.astype(np.float64))
    err = np.abs(out - ref)
    m = np.abs(ref) > 1e-3
    print("fp32 abs err %.2e, rel err (|gelu| > 1e-3) %.2e" % (err.max(), (err[m] / np.abs(ref[m])).max()))


if __name__ == "__main__":
    main()
