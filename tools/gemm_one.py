#!/usr/bin/env python3
"""Run one GEMM shape N times (for rocprofv3 PMC passes): gemm_one.py M N K epi cfg reps.
epi: plain | gelu (bf16 out) | res (fp32 out + fp32 residual)."""
import importlib, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
importlib.import_module("stuttering-speech-representation_amd")
from ssr_amd import _lib
from ssr_amd.model import gemm

M, N, K = (int(v) for v in sys.argv[1:4])
epi, cfg, reps = sys.argv[4], sys.argv[5], int(sys.argv[6])
_lib.lib().sse_set_option(b"gemm_cfg", int(cfg))
g = torch.Generator(device="cuda").manual_seed(1)
a = (2 * torch.rand(M, K, device="cuda", generator=g) - 1).bfloat16()
b = ((2 * torch.rand(N, K, device="cuda", generator=g) - 1) / K ** 0.5).bfloat16()
bias = torch.randn(N, device="cuda", generator=g)
resid = torch.randn(M, N, device="cuda", generator=g) if epi == "res" else None
for _ in range(reps):
    gemm(a, b, bias, resid, "gelu" if epi == "gelu" else None,
         out_dtype=torch.float32 if epi == "res" else torch.bfloat16)
torch.cuda.synchronize()
print("done")
