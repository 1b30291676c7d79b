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


def _mx8(t: torch.Tensor, dim: int) -> torch.Tensor:
    """MX-fp8 quantise-dequantise along `dim` (blocks of 32, E8M0 scale = smallest 2^E with
    max|x| <= 448 2^E, e4m3 RNE; oracle/mx.py's rule)."""
    x = t.movedim(dim, -1)
    K = x.shape[-1]
    pad = (-K) % 32
    xp = torch.nn.functional.pad(x, (0, pad))
    b = xp.reshape(*xp.shape[:-1], -1, 32)
    amax = b.abs().amax(-1, keepdim=True)
    e = torch.ceil(torch.log2(torch.clamp(amax, min=1e-38) / 448.0)).clamp(-127, 127)
    sc = torch.exp2(e)
    q = (b / sc).to(torch.float8_e4m3fn).float() * sc
    q = q.reshape(xp.shape)[..., :K]
    return q.movedim(-1, dim)


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
    if fmt == "fp16x3f8":   # hi x hi in fp16, the two cross terms as MX-fp8 products (probe, not a GPU path)
        s = _pow2_scale(w)
        ws = w * s
        xh = _ftz16(_f16(x))
        xl = _ftz16(_f16((x - xh) * 2048.0))
        wh = _ftz16(_f16(ws))
        wl = _ftz16(_f16(ws - wh))
        return (fn(xh, wh) + fn(_mx8(xl, 1 if x.dim() == 3 else -1), _mx8(wh, 1 if w.dim() == 3 else -1)) / 2048.0
                + fn(_mx8(xh, 1 if x.dim() == 3 else -1), _mx8(wl, 1 if w.dim() == 3 else -1))) / s
    if fmt in ("fp16x2a", "fp16x2w"):   # two products: split activations (a) or split weights (w)
        s = _pow2_scale(w)
        ws = w * s
        xh = _ftz16(_f16(x))
        wh = _ftz16(_f16(ws))
        if fmt == "fp16x2a":
            xl = _ftz16(_f16((x - xh) * 2048.0))
            return (fn(xh, wh) + fn(xl, _ftz16(_f16(wh / 2048.0)))) / s
        return (fn(xh, wh) + fn(xh, _ftz16(_f16(ws - wh)))) / s
    raise ValueError(fmt)


_SDPA = F.scaled_dot_product_attention

# pipeline stages a per-stage format assignment can name (the GEMM roles of the GPU path)
STAGES = ("conv", "proj", "posconv", "qkv", "attn", "oproj", "ffn1", "ffn2")


def stage_of(key: str) -> str | None:
    """Weight key of the WavLM state dict -> pipeline stage."""
    if key.startswith("feature_extractor.conv_layers.") and ".conv.weight" in key:
        return None if key.startswith("feature_extractor.conv_layers.0.") else "conv"
    if key == "feature_projection.projection.weight":
        return "proj"
    if key == "encoder.pos_conv_embed.conv.parametrizations.weight.original1":
        return "posconv"
    for frag, st in ((".q_proj.", "qkv"), (".k_proj.", "qkv"), (".v_proj.", "qkv"), ("gru_rel_pos_linear", "qkv"),
                     (".out_proj.", "oproj"), ("intermediate_dense", "ffn1"), ("output_dense", "ffn2")):
        if frag in key and key.endswith("weight"):
            return st
    return None


class _Patch:
    """fmt: one format for every GEMM (the historical mode), or a dict stage -> format (missing
    stages stay exact fp32).  Stage of a call: looked up from the weight tensor's identity (``ids``);
    the positional conv's weight is recomputed by weight norm every forward, so grouped convs are
    the "posconv" stage; the attention core ("attn": Q.K^T and P.V operands) is emulated by patching
    scaled_dot_product_attention."""

    def __init__(self, fmt, ids: dict | None = None):
        self.fmt = fmt
        self.ids = ids or {}

    def _f(self, w, default_stage=None):
        if isinstance(self.fmt, str):
            return self.fmt
        st = self.ids.get(id(w), default_stage)
        return self.fmt.get(st, "fp32") if st else "fp32"

    def __enter__(self):
        def lin(x, w, b=None):
            f = self._f(w)
            y = _LIN(x, w) if f == "fp32" else emulated_product(_LIN, x, w, f)
            return y if b is None else y + b

        def conv(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
            if w.shape[1] == 1:                      # conv0: fp32 in every path
                return _CONV(x, w, b, stride, padding, dilation, groups)
            if groups != 1:                          # positional conv
                f = "fp32" if isinstance(self.fmt, str) else self.fmt.get("posconv", "fp32")
            else:
                f = self._f(w)
            if f == "fp32":
                return _CONV(x, w, b, stride, padding, dilation, groups)
            y = emulated_product(lambda a, c: _CONV(a, c, None, stride, padding, dilation, groups), x, w, f)
            return y if b is None else y + b[None, :, None]

        def sdpa(q, k, v, attn_mask=None, dropout_p=0.0, is_causal=False, scale=None, **kw):
            f = "fp32" if isinstance(self.fmt, str) else self.fmt.get("attn", "fp32")
            if f == "fp32":
                return _SDPA(q, k, v, attn_mask=attn_mask, dropout_p=dropout_p, is_causal=is_causal, scale=scale)
            sc = (q.shape[-1] ** -0.5) if scale is None else scale
            s_ = emulated_product(lambda a, c: a @ c.transpose(-2, -1), q, k, f) * sc
            if attn_mask is not None:
                s_ = s_ + attn_mask
            p_ = torch.softmax(s_, dim=-1)
            return emulated_product(lambda a, c: a @ c.transpose(-2, -1), p_, v.transpose(-2, -1).contiguous(), f)

        F.linear, F.conv1d, F.scaled_dot_product_attention = lin, conv, sdpa
        return self

    def __exit__(self, *exc):
        F.linear, F.conv1d, F.scaled_dot_product_attention = _LIN, _CONV, _SDPA


def _rel_cos(got: np.ndarray, ref: np.ndarray):
    rel = np.linalg.norm(got - ref, axis=-1) / np.linalg.norm(ref, axis=-1)
    cos = (got * ref).sum(-1) / (np.linalg.norm(got, axis=-1) * np.linalg.norm(ref, axis=-1))
    return rel, cos


def emulate(spec, sd: dict, clips: np.ndarray, layer_indices, fmt) -> np.ndarray:
    """fmt: a format name for every GEMM, or a dict stage -> format (others exact fp32)."""
    o = WavLMAten(spec, sd)
    ids = {id(v): stage_of(k) for k, v in o.w.items() if stage_of(k)}
    with torch.no_grad(), _Patch(fmt, ids):
        return o.embed(clips, layer_indices)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--fixture", default="outlier", choices=["outlier", "wavlm_base"])
    ap.add_argument("--formats", default="bf16,fp16,bf16x3,fp16x3")
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--out", default="")
    ap.add_argument("--stages", action="store_true", help="per-stage sensitivity table (STAGES)")
    ap.add_argument("--assign", action="append", default=[], help="stage=fmt,... assignment to evaluate")
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
    if a.stages:
        # per-stage sensitivity: each stage alone in the format (others exact fp32), then the
        # assignment given by --assign (stage=fmt,...)
        for fmt in a.formats.split(","):
            for st in STAGES:
                rel, cos = _rel_cos(emulate(C.WAVLM_BASE, sd, clips, idx, {st: fmt}), ref)
                res[f"{st}:{fmt}"] = {"rel_l2_max": float(rel.max()), "cos_min": float(cos.min())}
                print(st, fmt, json.dumps(res[f"{st}:{fmt}"]), flush=True)
        for asg in a.assign:
            d = dict(kv.split("=") for kv in asg.split(","))
            rel, cos = _rel_cos(emulate(C.WAVLM_BASE, sd, clips, idx, d), ref)
            res["assign:" + asg] = {"rel_l2_max": float(rel.max()), "cos_min": float(cos.min())}
            print("assign", asg, json.dumps(res["assign:" + asg]), flush=True)
        if a.out:
            with open(a.out, "w") as f:
                json.dump({"fixture": a.fixture, "per_stage": res}, f, indent=1)
        return
    for fmt in a.formats.split(","):
        rel, cos = _rel_cos(emulate(C.WAVLM_BASE, sd, clips, idx, fmt), ref)
        res[fmt] = {"rel_l2_max": float(rel.max()), "cos_min": float(cos.min())}
        print(fmt, json.dumps(res[fmt]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"fixture": a.fixture, "formats": res}, f, indent=1)


if __name__ == "__main__":
    main()
