"""ORACLE (test infrastructure only): operand-format emulation of the reference's WavLM forward.

Runs ``oracle.wavlm_aten.WavLMAten`` (the reference's own ATen call sequence, bit-exact with its
fixtures) with every dense GEMM / strided conv (feature-encoder convs 1..6, feature projection,
Q/K/V/out projections, the gate linear, FFN1/FFN2) fed operands rounded to a GEMM operand format,
products accumulated in fp32 -- the arithmetic of an ideal kernel in that format, independent of
any HIP code.  It answers "how much of a GPU path's error does the FORMAT alone force on these
inputs?", which is how the per-dtype bars of the outlier-weight stress test are derived
(tests/test_gpu_outlier.py, DESIGN.md "Parity bars"):

  bf16      operands bf16(x), bf16(w)                               (the bf16 path's GEMMs)
  fp16      operands f16(x), f16(w 2^e) 2^-e                          (per-tensor power-of-two scale)
  bf16x3    hi + lo bf16 split, hi*hi + lo*hi + hi*lo                 (round-2 split-bf16 scheme)
  fp16x3    hi + lo' f16 split of common.h x3_split4, weights 2^e-scaled, subnormals flushed
            (the worst case for the fp16 MFMA) -- the SSE_DTYPE_FP16X3 path's scheme

conv0 (a VALU / exact-f32 kernel in every path), the positional conv, the attention core and the
LayerNorms stay fp32 as in the fp16x3 path.  Usage:

  python oracle/emulate.py --fixture outlier --formats bf16,fp16,bf16x3,fp16x3
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
importlib.import_module("stuttering-speech-representation_amd")   # registers ssr_amd

from oracle.wavlm_aten import WavLMAten   # noqa: E402

_LIN, _CONV = F.linear, F.conv1d


def _ftz16(t: torch.Tensor) -> torch.Tensor:
    return torch.where(t.abs() < 2.0 ** -14, torch.zeros_like(t), t)


def _f16(t: torch.Tensor) -> torch.Tensor:
    r = t.half().float()
    if not torch.isfinite(r).all():
        raise OverflowError("operand outside the fp16 range")
    return r


def _pow2_scale(w: torch.Tensor) -> float:
    m = float(w.abs().max())
    return float(2.0 ** np.floor(np.log2(16384.0 / m))) if m > 0 else 1.0


def emulated_product(fn, x: torch.Tensor, w: torch.Tensor, fmt: str) -> torch.Tensor:
    """fn(a, b) = the fp32 linear / conv of already-rounded operands."""
    if fmt == "bf16":
        return fn(x.bfloat16().float(), w.bfloat16().float())
    if fmt == "fp16":
        s = _pow2_scale(w)
        return fn(_f16(x), _f16(w * s)) / s
    if fmt == "bf16x3":
        xh = x.bfloat16().float()
        xl = (x - xh).bfloat16().float()
        wh = w.bfloat16().float()
        wl = (w - wh).bfloat16().float()
        return fn(xh, wh) + fn(xl, wh) + fn(xh, wl)
    if fmt == "fp16x3":   # common.h x3_split4 + Arena::put_x3
        s = _pow2_scale(w)
        ws = w * s
        xh = _ftz16(_f16(x))
        xl = _ftz16(_f16((x - xh) * 2048.0))
        wh = _ftz16(_f16(ws))
        wm = _ftz16(_f16(wh / 2048.0))
        wl = _ftz16(_f16(ws - wh))
        return (fn(xh, wh) + fn(xl, wm) + fn(xh, wl)) / s
    raise ValueError(fmt)


class _Patch:
    def __init__(self, fmt: str):
        self.fmt = fmt

    def __enter__(self):
        fmt = self.fmt

        def lin(x, w, b=None):
            y = emulated_product(_LIN, x, w, fmt)
            return y if b is None else y + b

        def conv(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
            if groups != 1 or w.shape[1] == 1:      # positional conv / conv0: fp32 in every path
                return _CONV(x, w, b, stride, padding, dilation, groups)
            y = emulated_product(lambda a, c: _CONV(a, c, None, stride, padding, dilation), x, w, fmt)
            return y if b is None else y + b[None, :, None]

        F.linear, F.conv1d = lin, conv
        return self

    def __exit__(self, *exc):
        F.linear, F.conv1d = _LIN, _CONV


def _rel_cos(got: np.ndarray, ref: np.ndarray):
    rel = np.linalg.norm(got - ref, axis=-1) / np.linalg.norm(ref, axis=-1)
    cos = (got * ref).sum(-1) / (np.linalg.norm(got, axis=-1) * np.linalg.norm(ref, axis=-1))
    return rel, cos


def emulate(spec, sd: dict, clips: np.ndarray, layer_indices, fmt: str) -> np.ndarray:
    with torch.no_grad(), _Patch(fmt):
        return WavLMAten(spec, sd).embed(clips, layer_indices)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--fixture", default="outlier", choices=["outlier", "wavlm_base"])
    ap.add_argument("--formats", default="bf16,fp16,bf16x3,fp16x3")
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    from ssr_amd import config as C, synth
    g = np.load(os.path.join(ROOT, "tests", "golden", f"{a.fixture}.npz"))
    if a.fixture == "outlier":   # tests/golden/make_golden.py outlier_golden
        sd = synth.outlier_weights(synth.synth_wavlm_state_dict(C.WAVLM_BASE, seed=7))
        clips = synth.synth_clips(4, 48000, seed=1234)
        idx, ref = [int(i) for i in g["wavlm_layer_indices"]], g["wavlm_emb"]
    else:                        # tests/conftest.py wavlm_sd / wavlm_clips
        sd = synth.synth_wavlm_state_dict(C.WAVLM_BASE, seed=7)
        clips = synth.synth_clips(16, 48000, seed=1234)[:4]
        idx, ref = [int(i) for i in g["layer_indices"]], g["emb_norm0"][:4]
    res = {}
    for fmt in a.formats.split(","):
        rel, cos = _rel_cos(emulate(C.WAVLM_BASE, sd, clips, idx, fmt), ref)
        res[fmt] = {"rel_l2_max": float(rel.max()), "cos_min": float(cos.min())}
        print(fmt, json.dumps(res[fmt]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"fixture": a.fixture, "formats": res}, f, indent=1)


if __name__ == "__main__":
    main()
