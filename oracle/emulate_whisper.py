"""ORACLE (test infrastructure only): operand-format emulation of the Whisper encoder's fp8 path.

The restated encoder (oracle/whisper.py ``WhisperOracle.hidden_states``, REF
whisper_embeddings_large.py:242-254 through HF ``WhisperEncoder``) in torch fp32 with the GEMM /
attention operands rounded the way a GPU path stores them, products accumulated in fp32.  It answers
"what does a given operand format cost on the large-v2 fixture?" before a kernel is written for it:

  gemm mx8     qkv / fc1 / fc2: both operands MX-fp8 along K (blocks of 32, E8M0 scale, e4m3 RNE;
               oracle/mx.py's rule), out-projection and convs bf16 -- the SSE_DTYPE_FP8 path
  oproj        bf16 (default) | mx8: the out-projection's operands MX-fp8 too (option f8_oproj = 1, round 6)
  stream bf16  residual stream and the qkv / context outputs rounded to bf16 where the path stores them
               (--stream res32: the residual stream kept fp32, the others bf16; fp32: nothing rounded)
  attn         bf16     Q, K, V, P bf16 (the shipped attention)
               qk8      Q.K^T on MX-fp8 operands (blocks of 32 along the head dim), P.V bf16
               qk8pv8t  + P e4m3 (unscaled, p <= 1) and V MX-fp8 along the KEY axis (blocks of 32 keys)
               qk8pv8   + P e4m3 and V e4m3 with one power-of-two scale per (head, dim) column
               qk8pv8x  qk8pv8 with the row sum l over the UNrounded p (the fp8 kernel's fp32 VALU sum)
               qk8pv8h  qk8pv8x with one V scale per head (max over the head's dims and the clip's tokens)

Usage: python oracle/emulate_whisper.py --attn bf16,qk8,qk8pv8t,qk8pv8
"""
from __future__ import annotations

import argparse
import importlib
import json
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
importlib.import_module("stuttering-speech-representation_amd")   # registers ssr_amd

from oracle.emulate import _mx8   # noqa: E402


def _bf(t):
    return t.bfloat16().float()


def _e4m3(t):
    return t.to(torch.float8_e4m3fn).float()


def _ln(x, w, b, eps):
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * w + b


def _gelu(x):
    return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))


def _conv(x, w, b, stride, fmt):
    """k = 3, pad 1 on channels-last x [T, C] as an im2col GEMM; w [out, in, 3]."""
    T, C = x.shape
    xp = torch.nn.functional.pad(x, (0, 0, 1, 1))
    t_out = (T + 2 - 3) // stride + 1
    cols = xp.unfold(0, 3, stride)[:t_out]                  # [t_out, C, 3]
    cols = cols.permute(0, 2, 1).reshape(t_out, 3 * C)
    wk = w.permute(2, 1, 0).reshape(3 * C, -1)
    if fmt == "bf16":
        cols, wk = _bf(cols), _bf(wk)
    return cols @ wk + b


def _lin(x, w, fmt):
    if fmt == "mx8":
        return _mx8(x, -1) @ _mx8(w, -1).T
    if fmt == "bf16":
        return _bf(x) @ _bf(w).T
    return x @ w.T


def _attn(q, k, v, attn):
    """q, k, v [heads, T, hd] (q pre-scaled) -> context [heads, T, hd]."""
    if attn == "fp32":
        s = q @ k.transpose(1, 2)
        return torch.softmax(s, -1) @ v
    if attn == "bf16":
        s = _bf(q) @ _bf(k).transpose(1, 2)
    else:
        s = _mx8(q, -1) @ _mx8(k, -1).transpose(1, 2)
    m = s.amax(-1, keepdim=True)
    p = torch.exp(s - m)
    if attn in ("bf16", "qk8"):
        pq, vq = _bf(p), _bf(v)
    elif attn == "qk8pv8t":
        pq, vq = _e4m3(p), _mx8(v, 1)                        # V blocks of 32 keys per (head, dim)
    elif attn in ("qk8pv8", "qk8pv8x", "qk8pv8h"):
        amax = v.abs().amax(1, keepdim=True).clamp(min=1e-30)
        if attn == "qk8pv8h":
            amax = amax.amax(-1, keepdim=True)
        sc = torch.exp2(torch.ceil(torch.log2(amax / 448.0)))
        pq, vq = _e4m3(p), _e4m3(v / sc) * sc
    else:
        raise ValueError(attn)
    l = p.sum(-1, keepdim=True) if attn in ("bf16", "qk8", "qk8pv8x", "qk8pv8h") else pq.sum(-1, keepdim=True)
    return (pq @ vq) / l


def _gelu_poly(x, c, coef):
    """the kernels' clamped odd-polynomial GELU (common.h gelu_fp8out2 form): x (1/2 + xc R(xc^2))"""
    xc = x.clamp(-c, c)
    s = xc * xc
    pp = torch.full_like(x, coef[0])
    for a in coef[1:]:
        pp = pp * s + a
    return x * (xc * pp + 0.5)


GELU_FP8 = {   # tools/fit_gelu.py fits: (clamp, coefficients highest degree first)
    "deg5": (3.5, (-3.503167250e-07, 2.229058919e-05, -5.630472442e-04, 7.574830670e-03, -6.208017841e-02,
                   3.963519037e-01)),
    "deg3": (3.0, (-0.00015428909682668746, 0.004529666155576706, -0.05285683274269104, 0.38795197010040283)),
    "deg2": (3.0, (0.0018274825997650623, -0.03881775215268135, 0.3680003583431244)),
}


def hidden_states(spec, p, mel, gemm="mx8", attn="bf16", stream="bf16", gelu_fc1="exact", oproj="bf16"):
    eps, nh, hd = spec.ln_eps, spec.heads, spec.head_dim
    rnd = _bf if stream in ("bf16", "res32") else (lambda t: t)     # qkv / context outputs
    rx = _bf if stream == "bf16" else (lambda t: t)                  # the residual stream (res32: fp32)
    cf = "bf16" if gemm != "fp32" else "fp32"
    x = mel.T
    x = _gelu(_conv(x, p["encoder.conv1.weight"], p["encoder.conv1.bias"], 1, cf))
    x = _gelu(_conv(x, p["encoder.conv2.weight"], p["encoder.conv2.bias"], 2, cf))
    x = rx(x + p["encoder.embed_positions.weight"][: x.shape[0]])
    hs = [x]
    T = x.shape[0]
    for l in range(spec.layers):
        a = f"encoder.layers.{l}"
        s_ = f"{a}.self_attn"
        h = _ln(x, p[f"{a}.self_attn_layer_norm.weight"], p[f"{a}.self_attn_layer_norm.bias"], eps)
        q = rnd((_lin(h, p[f"{s_}.q_proj.weight"], gemm) + p[f"{s_}.q_proj.bias"]) * hd ** -0.5)
        k = rnd(_lin(h, p[f"{s_}.k_proj.weight"], gemm))
        v = rnd(_lin(h, p[f"{s_}.v_proj.weight"], gemm) + p[f"{s_}.v_proj.bias"])
        qh, kh, vh = (t.reshape(T, nh, hd).transpose(0, 1) for t in (q, k, v))
        ctx = rnd(_attn(qh, kh, vh, attn).transpose(0, 1).reshape(T, nh * hd))
        x = rx(x + _lin(ctx, p[f"{s_}.out_proj.weight"], oproj if gemm == "mx8" else cf) + p[f"{s_}.out_proj.bias"])
        h = _ln(x, p[f"{a}.final_layer_norm.weight"], p[f"{a}.final_layer_norm.bias"], eps)
        h = _lin(h, p[f"{a}.fc1.weight"], gemm) + p[f"{a}.fc1.bias"]
        h = _gelu(h) if gelu_fc1 == "exact" else _gelu_poly(h, *GELU_FP8[gelu_fc1])
        x = rx(x + _lin(h, p[f"{a}.fc2.weight"], gemm) + p[f"{a}.fc2.bias"])
        hs.append(x)
    hs[-1] = _ln(x, p["encoder.layer_norm.weight"], p["encoder.layer_norm.bias"], eps)
    return hs


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--attn", default="bf16,qk8,qk8pv8t,qk8pv8")
    ap.add_argument("--gemm", default="mx8")
    ap.add_argument("--gelu", default="exact", help="fc1 GELU: exact | deg5 | deg3 | deg2 (the fp8-out polynomials)")
    ap.add_argument("--oproj", default="bf16", help="out-projection operands with --gemm mx8: bf16 | mx8")
    ap.add_argument("--stream", default="bf16", help="bf16 | res32 | fp32 (see the module docstring)")
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    from ssr_amd import config as C, synth
    g = np.load(os.path.join(ROOT, "tests", "golden", "whisper_large_v2.npz"))
    spec = C.WHISPER_LARGE_V2
    p = {k: torch.from_numpy(np.asarray(v, np.float32)) for k, v in synth.synth_whisper_state_dict(spec, seed=11).items()}
    mel = torch.from_numpy(g["mel"][0])
    idx = [int(i) for i in g["layer_indices"]]
    ref = g["emb"][0]
    res = {}
    with torch.no_grad():
        for attn in a.attn.split(","):
            hs = hidden_states(spec, p, mel, a.gemm, attn, stream=a.stream, gelu_fc1=a.gelu, oproj=a.oproj)
            got = np.stack([hs[i].mean(0).numpy() for i in idx])
            rel = np.linalg.norm(got - ref, axis=-1) / np.linalg.norm(ref, axis=-1)
            cos = (got * ref).sum(-1) / (np.linalg.norm(got, axis=-1) * np.linalg.norm(ref, axis=-1))
            key = f"{a.gemm}/{attn}/{a.gelu}/oproj-{a.oproj}/stream-{a.stream}"
            res[key] = {"rel_l2_max": float(rel.max()), "cos_min": float(cos.min())}
            print(key, json.dumps(res[key]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
