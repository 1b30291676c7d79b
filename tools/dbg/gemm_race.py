"""Debug: persistent vs non-persistent bf16 GEMM bit-equality on the WavLM shapes, repeated."""
import importlib, sys, os
sys.path.insert(0, os.getcwd())
import torch
importlib.import_module("stuttering-speech-representation_amd")
from ssr_amd import _lib
from ssr_amd.model import gemm
torch.manual_seed(0)
for (M, N, K, act) in [(40704, 2560, 768, None), (40704, 3072, 768, "gelu_fast"), (11448, 2560, 768, None),
                       (40704, 512, 1536, "gelu_fast")]:
    a = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
    b = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    bias = torch.randn(N, device="cuda") * 0.1
    with _lib.option("gemm_nonpersist", 1):
        ref = gemm(a, b, bias=bias, act=act, out_dtype=torch.bfloat16)
    bad = 0
    for it in range(6):
        got = gemm(a, b, bias=bias, act=act, out_dtype=torch.bfloat16)
        ne = (got.view(torch.int16) != ref.view(torch.int16))
        n = int(ne.sum())
        if n:
            bad += 1
            rows = ne.any(1).nonzero().flatten()
            cols = ne.any(0).nonzero().flatten()
            print("MISMATCH", (M, N, K, act), "iter", it, "n", n, "rows", rows[:8].tolist(), "tiles_m",
                  sorted(set((rows // 256).tolist()))[:10], "cols", cols[:8].tolist(),
                  "maxdiff", float((got.float() - ref.float()).abs().max()), flush=True)
    print((M, N, K, act), "mismatching iterations", bad, flush=True)
