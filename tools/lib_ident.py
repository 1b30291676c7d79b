#!/usr/bin/env python3
"""Whole-model embeddings of the in-tree libsse.so saved / compared against another build's (bit identity of a
schedule-only change).  Usage: python tools/lib_ident.py save out.pt [--lib other.so]; python tools/lib_ident.py
check out.pt"""
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

importlib.import_module("stuttering-speech-representation_amd")
from ssr_amd import _lib, config as C, synth  # noqa: E402
from ssr_amd.model import SSEModel  # noqa: E402

mode, path = sys.argv[1], sys.argv[2]
if "--lib" in sys.argv:
    _lib.use_library(sys.argv[sys.argv.index("--lib") + 1])
out = {}
for spec, dtype, B, L in ((C.WAVLM_BASE, "bf16", 7, 48000), (C.WAVLM_BASE, "bf16", 256, 48000),
                          (C.WAVLM_BASE, "fp16", 5, 48000), (C.WAVLM_LARGE, "bf16", 3, 48000),
                          (C.WHISPER_SMALL, "bf16", 2, 480000)):
    m = SSEModel(spec, synth.synth_state_dict(spec), device="cuda:0", dtype=dtype)
    w = torch.from_numpy(synth.synth_clips(B, L, seed=B)).cuda()
    out[f"{spec.name}/{dtype}/{B}"] = m.embed(w, spec.default_layer_indices()).cpu()
    del m
    torch.cuda.empty_cache()
if mode == "save":
    torch.save(out, path)
else:
    ref = torch.load(path, weights_only=True)
    bad = [k for k in out if not torch.equal(out[k], ref[k])]
    for k in out:
        print(k, "bit-identical" if k not in bad else "DIFFERENT")
    sys.exit(1 if bad else 0)
