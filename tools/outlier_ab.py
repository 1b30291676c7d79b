#!/usr/bin/env python3
"""bf16 WavLM-base on the outlier-weight fixture under A/B kernel switches (sse_set_option):
prints max rel-L2 / min cosine against the reference fixture for each setting."""
import importlib, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
importlib.import_module("stuttering-speech-representation_amd")
from ssr_amd import _lib, config as C, synth
from ssr_amd.model import SSEModel

g = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "outlier.npz"))
sd = synth.outlier_weights(synth.synth_wavlm_state_dict(C.WAVLM_BASE, seed=7))
m = SSEModel(C.WAVLM_BASE, sd, device="cuda:0", dtype="bf16")
clips = torch.from_numpy(synth.synth_clips(4, 48000, seed=1234)).cuda()
idx = [int(i) for i in g["wavlm_layer_indices"]]
ref = g["wavlm_emb"]
for opts in ([], [("gelu_exact", 1)], [("no_lnfold", 1)], [("conv0_valu", 1)], [("posconv_gemm", 1)]):
    for k, v in opts:
        _lib.lib().sse_set_option(k.encode(), v)
    got = m.embed(clips, idx).cpu().numpy()
    rel = np.linalg.norm(got - ref, axis=-1) / np.linalg.norm(ref, axis=-1)
    cos = (got * ref).sum(-1) / (np.linalg.norm(got, axis=-1) * np.linalg.norm(ref, axis=-1))
    print(opts, "rel-L2 max %.4f cos min %.5f" % (rel.max(), cos.min()), flush=True)
    for k, v in opts:
        _lib.lib().sse_set_option(k.encode(), 0)
