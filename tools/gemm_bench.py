#!/usr/bin/env python3
"""Microbenchmark of the MFMA GEMM on the WavLM-base B=256 shapes (HIP-event timing)."""
import importlib, os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
importlib.import_module("stuttering-speech-representation_amd")
from ssr_amd import _lib
from ssr_amd.model import gemm

SHAPES = {"qkv": (38144, 2432, 768, None), "oproj": (38144, 768, 768, "res"), "ffn1": (38144, 3072, 768, "gelu"), "ffn1_noact": (38144, 3072, 768, None),
          "conv1": (1228544, 512, 1536, "gelu"), "conv1_noact": (1228544, 512, 1536, None),
          "ffn2": (38144, 768, 3072, "res"), "proj": (38144, 768, 512, None), "sq4096": (4096, 4096, 4096, None)}
cfgs = sys.argv[1:] or ["0"]
res = {}
for cfg, (name, (M, N, K, epi)) in [(c, kv) for kv in SHAPES.items() for c in cfgs]:
    _lib.lib().sse_set_option(b"gemm_cfg", int(cfg))
    if name == "qkv":
        N = 2560      # ldq padded to 256 (sse_model.hip build_wavlm)
    a = torch.randn(M, K, device="cuda").bfloat16()
    b = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    bias = torch.randn(N, device="cuda")
    resid = torch.randn(M, N, device="cuda") if epi == "res" else None
    act = "gelu" if epi == "gelu" else None
    outd = torch.float32 if epi == "res" else torch.bfloat16
    for _ in range(3):
        gemm(a, b, bias, resid, act, out_dtype=outd)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    e0.record()
    for _ in range(n):
        gemm(a, b, bias, resid, act, out_dtype=outd)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    res[f"{name}@{cfg}"] = {"ms": round(ms, 4), "tflops": round(2 * M * N * K / ms / 1e9, 1)}
# vendor library on the same shapes for scale (torch bf16 matmul -> hipBLASLt; plain GEMM only)
for name, (M, N, K, epi) in SHAPES.items():
    if name == "qkv":
        N = 2560
    a = torch.randn(M, K, device="cuda").bfloat16()
    b = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    for _ in range(3):
        a @ b.T
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        a @ b.T
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    res[f"{name}@torch"] = {"ms": round(ms, 4), "tflops": round(2 * M * N * K / ms / 1e9, 1)}
print(json.dumps(res))
