#!/usr/bin/env python3
"""Long-K bf16 GEMM shapes: the persistent kernel, the non-persistent kernel (option gemm_nonpersist) and hipBLASLt
(torch.addmm), to separate the main loop from tile order / L2 reuse.  Usage: python tools/gemm_longk_probe.py"""
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

importlib.import_module("stuttering-speech-representation_amd")
from ssr_amd import _lib  # noqa: E402
from ssr_amd.model import gemm  # noqa: E402

SHAPES = [(8192, 8192, 8192), (65536, 512, 8192), (16384, 1024, 8192), (4096, 4096, 4096), (38144, 768, 3072),
          (1228544, 512, 1536)]


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
for M, N, K in SHAPES:
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    bias = torch.randn(N, device="cuda")
    b16 = bias.bfloat16()
    fl = 2.0 * M * N * K
    row = {}
    for name, opt in (("persistent", 0), ("nonpersistent", 1)):
        with _lib.option("gemm_nonpersist", opt):
            row[name] = round(fl / timeit(lambda: gemm(x, w, bias, out_dtype=torch.bfloat16)) / 1e9, 1)
    row["hipblaslt"] = round(fl / timeit(lambda: torch.addmm(b16, x, w.t())) / 1e9, 1)
    res[f"{M}x{N}x{K}"] = row
    print(f"{M}x{N}x{K}", row, flush=True)
    del x, w
print(json.dumps(res))
