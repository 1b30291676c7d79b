"""Debug: the folded-LN persistent GEMM (sse_gemm_lnfold) vs non-persistent, and position invariance."""
import importlib, sys, os, ctypes
sys.path.insert(0, os.getcwd())
import numpy as np, torch
importlib.import_module("stuttering-speech-representation_amd")
from ssr_amd import _lib
L = _lib.lib()
torch.manual_seed(0)
z = torch.zeros(64, device="cuda")
def run(a, b, bias, acol, part, act, nonpersist=0):
    M, K = a.shape; N = b.shape[0]
    ct = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    with _lib.option("gemm_nonpersist", nonpersist):
        rc = L.sse_gemm_lnfold(a.data_ptr(), b.data_ptr(), bias.data_ptr(), acol.data_ptr(), part.data_ptr(), ct.data_ptr(),
                               M, N, K, act, ctypes.c_float(1e-5), z.data_ptr(), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, rc
    torch.cuda.synchronize()
    return ct
for (M, N, act) in [(40704, 2560, 0), (40704, 3072, 2), (11448, 2560, 0)]:
    K = 768
    a = (torch.randn(M, K, device="cuda") * 2 + 0.3).bfloat16()
    b = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    bias = torch.randn(N, device="cuda") * 0.1
    acol = b.float().sum(1)
    af = a.float().view(M, 3, 256)
    mean = af.mean(2); m2 = ((af - mean[..., None]) ** 2).sum(2)
    part = torch.stack([mean, m2], -1).contiguous()          # [M][3][2]
    p = run(a, b, bias, acol, part, act)
    q = run(a, b, bias, acol, part, act, 1)
    ne = (p.view(torch.int16) != q.view(torch.int16))
    r = ne.any(1).nonzero().flatten()
    print((M, N, act), "persist vs nonpersist mismatches", int(ne.sum()), "rows", r[:10].tolist(), flush=True)
    # position invariance: roll rows by 256*k and recompute persistent
    for sh in (256, 256 * 43, 128):
        a2 = torch.roll(a, sh, 0); part2 = torch.roll(part, sh, 0)
        p2 = torch.roll(run(a2, b, bias, acol, part2, act), -sh, 0)
        ne2 = (p2.view(torch.int16) != p.view(torch.int16))
        print("  roll", sh, "mismatches vs unrolled persistent", int(ne2.sum()), flush=True)
