#!/usr/bin/env python3
"""Persistent bf16 GEMM timing experiments (sse_set_option gemm_xp): 0 production, 1 no stores,
2 no epilogue, 3 staggered start, 4 polynomial GELU, 5 compile-time bias/no-fold, 6 = 4 + 5."""
import importlib, os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
importlib.import_module("stuttering-speech-representation_amd")
from ssr_amd import _lib
from ssr_amd.model import gemm

SHAPES = {"qkv": (38144, 2560, 768, None), "ffn1": (38144, 3072, 768, "gelu_fast"),
          "conv1": (1228544, 512, 1536, "gelu_fast"), "sq4096": (4096, 4096, 4096, None)}
xps = [int(v) for v in sys.argv[1:]] or [0, 1, 2, 3, 4, 5, 6]
res = {}
for name, (M, N, K, act) in SHAPES.items():
    a = torch.randn(M, K, device="cuda").bfloat16()
    b = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    bias = torch.randn(N, device="cuda")
    for rep in range(2):
        for xp in xps:
            _lib.lib().sse_set_option(b"gemm_xp", xp)
            for _ in range(3):
                gemm(a, b, bias, None, act, out_dtype=torch.bfloat16)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 20
            e0.record()
            for _ in range(n):
                gemm(a, b, bias, None, act, out_dtype=torch.bfloat16)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / n
            res.setdefault(f"{name}@{xp}", []).append(round(2 * M * N * K / ms / 1e9, 1))
    _lib.lib().sse_set_option(b"gemm_xp", 0)
    print(json.dumps({k: v for k, v in res.items() if k.startswith(name)}), flush=True)
