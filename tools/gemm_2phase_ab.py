#!/usr/bin/env python3
"""The persistent bf16 GEMM's two 32-MFMA phases per K-tile (default) against option gemm_4phase = 1: bit-identity
schedule (each accumulator sees the same K-steps in the same order) on the model shapes and ragged M / short K, then
per-shape timing both ways.  Usage: python tools/gemm_2phase_ab.py"""
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

importlib.import_module("stuttering-speech-representation_amd")
from ssr_amd import _lib  # noqa: E402
from ssr_amd.model import gemm  # noqa: E402

SHAPES = [(38144, 2560, 768, None), (38144, 3072, 768, "gelu_fast"), (1228544, 512, 1536, "gelu_fast"),
          (38144, 768, 512, None), (4097, 512, 64, None), (4351, 768, 128, "gelu_fast"), (301, 256, 192, None),
          (8192, 8192, 8192, None), (65536, 512, 8192, None), (4096, 4096, 4096, None)]


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


res = {}
ok = True
for M, N, K, act in SHAPES:
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    f = lambda: gemm(x, w, bias, act=act, out_dtype=torch.bfloat16)  # noqa: E731
    ref = f()
    with _lib.option("gemm_4phase", 1):
        got = f()
    same = bool(torch.equal(ref, got))
    ok &= same
    fl = 2.0 * M * N * K
    t2 = timeit(f)
    with _lib.option("gemm_4phase", 1):
        t4 = timeit(f)
    t2b = timeit(f)
    res[f"{M}x{N}x{K} {act}"] = {"bit_identical": same, "tflops_4phase": round(fl / t4 / 1e9, 1),
                                 "tflops_2phase": round(fl / min(t2, t2b) / 1e9, 1)}
    print(f"{M}x{N}x{K} {act}", res[f"{M}x{N}x{K} {act}"], flush=True)
    del x, w
print(json.dumps(res))
sys.exit(0 if ok else 1)
