"""Debug: persistent (folded LN) vs non-persistent GEMMs through the full bf16 WavLM-base forward."""
import importlib, sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
importlib.import_module("stuttering-speech-representation_amd")
from ssr_amd import config as C, synth, _lib
from ssr_amd.model import SSEModel
spec = C.WAVLM_BASE
m = SSEModel(spec, synth.synth_wavlm_state_dict(spec, seed=7), device="cuda:0", dtype="bf16")
idx = list(range(13))
for seed in (1234, 77, 5):
    for B, L in ((256, 48000), (72, 50976)):
        w = torch.from_numpy(synth.synth_clips(B, L, seed=seed)).cuda()
        a = m.embed(w, idx).cpu().numpy()
        with _lib.option("gemm_nonpersist", 1):
            b = m.embed(w, idx).cpu().numpy()
        d = [(c, l) for c in range(B) for l in range(13) if not np.array_equal(a[c, l], b[c, l])]
        first = sorted(set(c for c, _ in d))
        print(seed, B, L, "clips differing", len(first), first[:10], "first layers", sorted(set(l for c, l in d if c == (first[0] if first else -1)))[:4], flush=True)
