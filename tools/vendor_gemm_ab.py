#!/usr/bin/env python3
"""The path's GEMMs against the vendor library on the bench shapes (HIP-event timing, one box).

bf16: libsse's persistent 8-phase GEMM (sse_gemm: bias, bf16 out) vs torch.addmm (hipBLASLt, bias epilogue,
bf16 out) on the WavLM-base B = 256 x 3 s shapes.  fp8: libsse's MX-fp8 GEMM (sse_gemm_mx, E8M0 block scales
per 32 K-elements, bf16 out) vs torch._scaled_mm (hipBLASLt, e4m3 with per-tensor scales -- a coarser format
than MX, so the cheaper of the two) on the Whisper-large-v2 B = 128 x 30 s shapes.  Run it under
`rocprofv3 --kernel-trace --stats` to see which hipBLASLt kernels (macro tiles) the library picked.
Usage: python tools/vendor_gemm_ab.py [--reps N] [--json out.json]
"""
import argparse
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

importlib.import_module("stuttering-speech-representation_amd")
from ssr_amd.model import gemm, gemm_mx, mx_quantize  # noqa: E402

# (M, N, K): WavLM-base B = 256 x 3 s (M = 256 x 149 frames; conv1: 256 x 4799 frames, K = 3 taps x 512)
BF16 = {"qkv": (38144, 2560, 768), "ffn1": (38144, 3072, 768), "oproj": (38144, 768, 768),
        "ffn2": (38144, 768, 3072), "conv1": (1228544, 512, 1536), "sq8192": (8192, 8192, 8192)}
# Whisper-large-v2 B = 128 x 30 s: M = 128 x 1500 frames, D = 1280, F = 5120
FP8 = {"qkv": (192000, 3840, 1280), "fc1": (192000, 5120, 1280), "fc2": (192000, 1280, 5120),
       "sq8192": (8192, 8192, 8192)}


def timeit(fn, reps):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(7)
    res = {}
    for name, (M, N, K) in BF16.items():
        x = torch.randn(M, K, device=dev, generator=g).bfloat16()
        w = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).bfloat16()
        bias = torch.randn(N, device=dev, generator=g)
        bias16 = bias.bfloat16()
        fl = 2.0 * M * N * K
        ours = timeit(lambda: gemm(x, w, bias, out_dtype=torch.bfloat16), a.reps)
        vend = timeit(lambda: torch.addmm(bias16, x, w.t()), a.reps)
        d = (gemm(x, w, bias, out_dtype=torch.bfloat16).float() - torch.addmm(bias16, x, w.t()).float()).norm()
        rel = float(d / torch.addmm(bias16, x, w.t()).float().norm())
        res[f"bf16 {name} {M}x{N}x{K}"] = {"sse_ms": round(ours, 4), "sse_tflops": round(fl / ours / 1e9, 1),
                                          "hipblaslt_ms": round(vend, 4), "hipblaslt_tflops": round(fl / vend / 1e9, 1),
                                          "rel_l2_between": round(rel, 5)}
        print(name, res[f"bf16 {name} {M}x{N}x{K}"], flush=True)
        del x, w
    f8 = torch.float8_e4m3fn
    for name, (M, N, K) in FP8.items():
        x = torch.randn(M, K, device=dev, generator=g)
        w = torch.randn(N, K, device=dev, generator=g) / K ** 0.5
        bias = torch.randn(N, device=dev, generator=g)
        fl = 2.0 * M * N * K
        xq, xs = mx_quantize(x)
        wq, ws = mx_quantize(w, 1)
        ours = timeit(lambda: gemm_mx(xq, xs, wq, ws, bias, out="bf16"), a.reps)
        sa = (x.abs().max() / 448.0).float()
        sb = (w.abs().max() / 448.0).float()
        x8 = (x / sa).to(f8)
        w8 = (w / sb).to(f8)
        del x, w
        vend_fn = lambda: torch._scaled_mm(x8, w8.t(), scale_a=sa, scale_b=sb, bias=bias.bfloat16(),  # noqa: E731
                                           out_dtype=torch.bfloat16)
        try:
            vend = timeit(vend_fn, a.reps)
            vt = round(fl / vend / 1e9, 1)
            vend = round(vend, 4)
        except Exception as e:   # noqa: BLE001 -- report what the library refused
            vend, vt = f"unavailable: {type(e).__name__}: {str(e)[:120]}", None
        res[f"fp8 {name} {M}x{N}x{K}"] = {"sse_mx_ms": round(ours, 4), "sse_mx_tflops": round(fl / ours / 1e9, 1),
                                         "hipblaslt_e4m3_tensor_scale_ms": vend, "hipblaslt_tflops": vt}
        print(name, res[f"fp8 {name} {M}x{N}x{K}"], flush=True)
        del xq, wq, x8, w8
        torch.cuda.empty_cache()
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
