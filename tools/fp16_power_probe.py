"""Why the fp16 path's GEMMs run a few % slower than bf16's with the same instruction stream.

The same library kernel (gemm8p_kernel, the persistent 8-phase GEMM; fp16 = its F16 instantiation: the f16 MFMA
instead of the bf16 one, fp16 packing) is timed on WavLM-shaped GEMMs with operands of four kinds, interleaved
rounds on one box:
  bf16        N(0, 1) operands in bf16 (the bf16 path)
  fp16        the same values in fp16 (10 mantissa bits set at random)
  fp16_bf16v  fp16 operands holding bf16-representable values (the low 3 mantissa bits zero)
  bf16_zero   bf16 operands of zeros (no multiplier toggling)
If the fp16 slowdown follows the operand bits (fp16_bf16v as fast as bf16, zeros faster still), it is the matrix
core's data-dependent power under the chip's power limit (clock give-back), not the code.
Usage (GPU box): python tools/fp16_power_probe.py [rounds]
       rocprofv3 --pmc GRBM_GUI_ACTIVE -d <dir> -o c --output-format csv -- python3 tools/fp16_power_probe.py pmc
         then python3 tools/fp16_power_probe.py clocks <dir>/c_counter_collection.csv: the same launches, 5 per
         (shape, operand kind) in a fixed order, and the clock each ran at (GRBM_GUI_ACTIVE / 8 XCDs / duration)
"""
import ctypes
import importlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
importlib.import_module("stuttering-speech-representation_amd")
from ssr_amd import _lib  # noqa: E402


def gemm(code, a, b, bias, ct, M, N, K, act, z):
    d = _lib.sse_gemm_desc()
    d.dtype, d.M, d.N, d.K, d.ldc, d.act = code, M, N, K, N, act
    d.a, d.b, d.zero, d.bias, d.ct = a.data_ptr(), b.data_ptr(), z.data_ptr(), bias.data_ptr(), ct.data_ptr()
    rc = _lib.lib().sse_gemm_ex(ctypes.byref(d), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    _lib.check(rc, "sse_gemm_ex")


def clocks(path):
    """Per (shape, kind) group of 5 consecutive GEMM dispatches of a `pmc` run: mean effective clock."""
    import csv
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and "gemm8" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    labels = [(n, k) for n, *_ in SHAPES for k in KINDS]
    out = {}
    for i, (n, k) in enumerate(labels):
        grp = rows[5 * i:5 * i + 5]
        if len(grp) < 5:
            break
        mhz = [float(r["Counter_Value"]) / 8.0 / ((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9) / 1e6
               for r in grp]
        us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3 for r in grp]
        out.setdefault(n, {})[k] = {"mhz": round(sum(mhz) / len(mhz)), "us": round(sorted(us)[len(us) // 2], 1),
                                     "cycles_per_xcd": round(float(grp[2]["Counter_Value"]) / 8)}
        print(n, k, out[n][k], flush=True)
    print(json.dumps(out))


SHAPES = [("conv1_like", 262144, 512, 1536, 2), ("ffn1_like", 38144, 3072, 768, 2), ("qkv_like", 38144, 2560, 768, 0),
          ("k3072", 38144, 768, 3072, 0), ("sq8192", 8192, 8192, 8192, 0)]
KINDS = ["bf16", "fp16", "fp16_bf16v", "bf16_zero"]


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "clocks":
        return clocks(sys.argv[2])
    pmc = len(sys.argv) > 1 and sys.argv[1] == "pmc"
    rounds = 1 if pmc else (int(sys.argv[1]) if len(sys.argv) > 1 else 3)
    z = torch.zeros(64, device="cuda")
    res = {}
    for name, M, N, K, act in SHAPES:
        g = torch.Generator(device="cuda").manual_seed(M + N + K)
        a32 = torch.randn(M, K, device="cuda", generator=g)
        b32 = torch.randn(N, K, device="cuda", generator=g) / K ** 0.5
        bias = torch.randn(N, device="cuda", generator=g) * 0.1
        ops = {"bf16": (1, a32.bfloat16(), b32.bfloat16()),
               "fp16": (4, a32.half(), b32.half()),
               "fp16_bf16v": (4, a32.bfloat16().half(), b32.bfloat16().half()),
               "bf16_zero": (1, torch.zeros(M, K, device="cuda", dtype=torch.bfloat16),
                             torch.zeros(N, K, device="cuda", dtype=torch.bfloat16))}
        del a32, b32
        outs = {k: torch.empty(M, N, device="cuda", dtype=torch.bfloat16 if v[0] == 1 else torch.float16)
                for k, v in ops.items()}
        best = {k: 1e30 for k in ops}
        it = 10 if M * N * K < 1e12 else 4
        if pmc:   # 5 launches per kind, in KINDS order (the clocks() grouping)
            for k in KINDS:
                code, a, b = ops[k]
                for _i in range(5):
                    gemm(code, a, b, bias, outs[k], M, N, K, act, z)
            torch.cuda.synchronize()
            del ops, outs
            torch.cuda.empty_cache()
            continue
        for _ in range(rounds):
            for k, (code, a, b) in ops.items():
                for _w in range(2):
                    gemm(code, a, b, bias, outs[k], M, N, K, act, z)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _i in range(it):
                    gemm(code, a, b, bias, outs[k], M, N, K, act, z)
                e1.record()
                torch.cuda.synchronize()
                best[k] = min(best[k], e0.elapsed_time(e1) / it)
        tf = 2.0 * M * N * K / 1e12
        res[name] = {k: {"us": round(v * 1e3, 1), "tflops": round(tf / (v * 1e-3), 1)} for k, v in best.items()}
        print(name, f"M={M} N={N} K={K} act={act}", "  ".join(f"{k} {v*1e3:.1f} us ({tf/(v*1e-3):.0f} TF/s)"
                                                          for k, v in best.items()), flush=True)
        del ops, outs
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
