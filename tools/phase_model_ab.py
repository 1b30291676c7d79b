#!/usr/bin/env python3
"""Whole-model bit-identity of the default GEMM K-tile schedules against option gemm_4phase = 1 / 2: WavLM-base and
-large bf16, WavLM-base fp16, Whisper-small bf16 / fp8, Whisper-large-v2 fp8 at small batches.  Exit 1 on a difference."""
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

importlib.import_module("stuttering-speech-representation_amd")
from ssr_amd import _lib, config as C, synth  # noqa: E402
from ssr_amd.model import SSEModel  # noqa: E402

ok = True
for spec, dtype, B, L in ((C.WAVLM_BASE, "bf16", 7, 48000), (C.WAVLM_BASE, "fp16", 5, 48000),
                          (C.WAVLM_LARGE, "bf16", 3, 48000), (C.WHISPER_SMALL, "bf16", 2, 480000),
                          (C.WHISPER_SMALL, "fp8", 3, 480000), (C.WHISPER_LARGE_V2, "fp8", 2, 480000)):
    m = SSEModel(spec, synth.synth_state_dict(spec), device="cuda:0", dtype=dtype)
    w = torch.from_numpy(synth.synth_clips(B, L, seed=B)).cuda()
    idx = spec.default_layer_indices()
    a = m.embed(w, idx)
    for v in (1,):
        with _lib.option("gemm_4phase", v):
            b = m.embed(w, idx)
        same = bool(torch.equal(a, b))
        ok &= same
        print(spec.name, dtype, f"gemm_4phase={v}", "bit-identical" if same else
              f"DIFFERENT max {float((a - b).abs().max()):.3e}", flush=True)
    del m
    torch.cuda.empty_cache()
sys.exit(0 if ok else 1)
