#!/usr/bin/env python3
"""Time the 8-phase GEMM on the path's shapes (HIP events, 20 reps).  Run once plainly and once
with SSE_GEMM_DEBUG=skip_epi to split mainloop from epilogue time."""
import importlib, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
importlib.import_module("stuttering-speech-representation_amd")
from ssr_amd.model import gemm

SHAPES = {"qkv": (38144, 2560, 768, "bias"), "oproj": (38144, 768, 768, "res"), "ffn1": (38144, 3072, 768, "gelu"),
          "ffn2": (38144, 768, 3072, "res"), "conv3x": (614144, 512, 1536, "gelu"),
          "k768sq": (8192, 8192, 768, "plain"), "sq4096": (4096, 4096, 4096, "plain")}
res = {}
for name, (M, N, K, epi) in SHAPES.items():
    g = torch.Generator(device="cuda").manual_seed(1)
    a = (2 * torch.rand(M, K, device="cuda", generator=g) - 1).bfloat16()
    b = ((2 * torch.rand(N, K, device="cuda", generator=g) - 1) / K ** 0.5).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g) if epi != "plain" else None
    resid = torch.randn(M, N, device="cuda", generator=g) if epi == "res" else None
    act = "gelu_fast" if epi == "gelu" else None
    outd = torch.float32 if epi == "res" else torch.bfloat16
    for _ in range(3):
        gemm(a, b, bias, resid, act, out_dtype=outd)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        gemm(a, b, bias, resid, act, out_dtype=outd)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    res[name] = {"ms": round(ms, 4), "tflops": round(2 * M * N * K / ms / 1e9, 1)}
    del a, b, bias, resid
    torch.cuda.empty_cache()
print(json.dumps({"mode": os.environ.get("SSE_GEMM_DEBUG", "normal"), "res": res}))
