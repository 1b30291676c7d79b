"""Deterministic synthetic clips and weights (counter-based splitmix64, numpy only).

There is no dataset or hub checkpoint offline, so every input
the oracle, the golden fixtures, the GPU tests and ``bench.py`` use comes from here.
``np.random`` is avoided on purpose: its Generator streams are not guaranteed stable
across numpy versions, while this counter hash is (it is plain uint64 arithmetic).

* clips: white Gaussian (sigma 0.1, Box-Muller) + a 3-tone sum, clipped to +-1
  (SURVEY.md §8(d) "Inputs").
* weights: uniform in [-a, a) per tensor with per-kind scales chosen so the random
  network keeps O(1) activations (softmax and the gated relative-position bias are both
  exercised, not saturated).  Throughput does not depend on weight values.
"""
from __future__ import annotations

import math
import zlib

import numpy as np

from .config import WavLMSpec, WhisperSpec, param_specs

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _base(seed: int, stream: int) -> np.uint64:
    s = np.array([(seed * 0x100000001B3 + stream * 0x9E3779B1 + 0x632BE59BD9B4E019) & 0xFFFFFFFFFFFFFFFF],
                 dtype=np.uint64)
    return _splitmix64(s)[0]


def uniform01(seed: int, stream: int, n: int, offset: int = 0) -> np.ndarray:
    """float64 uniforms in [0, 1) with 53 random bits, element i = hash(seed, stream, offset+i)."""
    idx = np.arange(offset, offset + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = _splitmix64(idx + _base(seed, stream))
    return (h >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def uniform_pm1_f32(seed: int, stream: int, n: int, chunk: int = 1 << 24) -> np.ndarray:
    """float32 uniforms in [-1, 1) (24-bit grid, exact in fp32); chunked for 1e9-element tensors."""
    out = np.empty(n, dtype=np.float32)
    b = _base(seed, stream)
    for o in range(0, n, chunk):
        m = min(chunk, n - o)
        idx = np.arange(o, o + m, dtype=np.uint64)
        with np.errstate(over="ignore"):
            h = _splitmix64(idx + b)
        out[o:o + m] = ((h >> np.uint64(40)).astype(np.int64) - (1 << 23)).astype(np.float32) * np.float32(2.0 ** -23)
    return out


def gaussian(seed: int, stream: int, n: int) -> np.ndarray:
    """float64 standard normals (Box-Muller on two independent uniform streams)."""
    u1 = uniform01(seed, 2 * stream, n)
    u2 = uniform01(seed, 2 * stream + 1, n)
    return np.sqrt(-2.0 * np.log1p(-u1)) * np.cos(2.0 * math.pi * u2)


def synth_clips(n_clips: int, n_samples: int, seed: int = 1234, sigma: float = 0.1,
                tones: bool = True, first_clip: int = 0, sample_rate: int = 16000) -> np.ndarray:
    """``[n_clips, n_samples]`` float32 clips; clip ``c`` depends only on (seed, first_clip + c)."""
    out = np.empty((n_clips, n_samples), dtype=np.float32)
    t = np.arange(n_samples, dtype=np.float64) / sample_rate
    for i in range(n_clips):
        c = first_clip + i
        x = sigma * gaussian(seed, 1000 + c, n_samples)
        if tones:
            fr = uniform01(seed, 500000 + c, 6)
            for k in range(3):
                f = 120.0 + 3000.0 * fr[k]
                x += 0.08 * np.sin(2.0 * math.pi * f * t + 2.0 * math.pi * fr[3 + k])
        out[i] = np.clip(x, -1.0, 1.0).astype(np.float32)
    return out


def _stream_of(key: str) -> int:
    return zlib.crc32(key.encode()) & 0x7FFFFFFF


def _wavlm_init(key: str, shape: tuple, spec: WavLMSpec, u: np.ndarray) -> np.ndarray:
    fan = int(np.prod(shape[1:])) if len(shape) > 1 else 1
    if key.endswith("parametrizations.weight.original0"):           # weight-norm g
        g = math.sqrt(spec.hidden * spec.hidden // spec.pos_groups / (shape[-1] * spec.hidden // spec.pos_groups))
        return (g * (1.0 + 0.1 * u)).astype(np.float32)
    if key.endswith("parametrizations.weight.original1"):           # weight-norm v
        return u
    if "layer_norm.weight" in key:
        return (1.0 + 0.1 * u).astype(np.float32)
    if "layer_norm.bias" in key:
        return (0.1 * u).astype(np.float32)
    if key.endswith("rel_attn_embed.weight"):
        return u
    if key.endswith("gru_rel_pos_const"):
        return (1.0 + 0.2 * u).astype(np.float32)
    if key.endswith("gru_rel_pos_linear.bias"):
        return (0.2 * u).astype(np.float32)
    if key.endswith(".bias"):
        return (0.02 * u).astype(np.float32)
    if "conv_layers" in key:                                         # conv + GELU: He-like gain
        return (math.sqrt(6.0 / fan) * u).astype(np.float32)
    return (math.sqrt(3.0 / fan) * u).astype(np.float32)


def synth_wavlm_state_dict(spec: WavLMSpec, seed: int = 7) -> dict[str, np.ndarray]:
    sd = {}
    for key, shape in param_specs(spec):
        n = int(np.prod(shape))
        u = uniform_pm1_f32(seed, _stream_of(key), n)
        sd[key] = _wavlm_init(key, shape, spec, u).reshape(shape)
    return sd


def sinusoids(length: int, channels: int, max_timescale: float = 10000.0) -> np.ndarray:
    """Whisper's fixed position table (HF/models/whisper/modeling_whisper.py:55-65), float32."""
    inc = np.float32(math.log(max_timescale) / (channels // 2 - 1))
    inv = np.exp(-inc * np.arange(channels // 2, dtype=np.float32)).astype(np.float32)
    st = np.arange(length, dtype=np.float32)[:, None] * inv[None, :]
    return np.concatenate([np.sin(st), np.cos(st)], axis=1).astype(np.float32)


def _whisper_hf_extra(spec: WhisperSpec) -> list[tuple[str, tuple]]:
    """Decoder tensors an HF WhisperModel holds but the 1-token pass never reads (full embedding
    tables and the self-attention q/k projections): synthesised so a HF model can be loaded."""
    D = spec.d_model
    out = [("decoder.embed_tokens.weight", (spec.vocab_size, D)),
           ("decoder.embed_positions.weight", (spec.max_target_positions, D))]
    for l in range(spec.decoder_layers):
        p = f"decoder.layers.{l}.self_attn"
        out += [(f"{p}.q_proj.weight", (D, D)), (f"{p}.q_proj.bias", (D,)), (f"{p}.k_proj.weight", (D, D))]
    return out


def synth_whisper_state_dict(spec: WhisperSpec, seed: int = 11, full_hf: bool = False) -> dict[str, np.ndarray]:
    """Synthetic Whisper weights.  Decoder rows that the path reads through "[0]" keys are row 0
    of the full synthetic tables, so ``full_hf=True`` (HF-loadable) and the packed blob agree."""
    sd = {}
    specs = [(k, s) for k, s in param_specs(spec) if not k.endswith("[0]")]
    if spec.decoder_layers:
        specs += _whisper_hf_extra(spec)
    for key, shape in specs:
        n = int(np.prod(shape))
        if key == "encoder.embed_positions.weight":
            sd[key] = sinusoids(shape[0], shape[1])
            continue
        if key in ("decoder.embed_tokens.weight", "decoder.embed_positions.weight"):
            if not full_hf:                              # only row 0 is read (input id 0, position 0)
                sd[key + "[0]"] = (0.5 * uniform_pm1_f32(seed, _stream_of(key), shape[1])).astype(np.float32)
                continue
            t = (0.5 * uniform_pm1_f32(seed, _stream_of(key), n)).reshape(shape).astype(np.float32)
            t[0] = (0.5 * uniform_pm1_f32(seed, _stream_of(key), shape[1])).astype(np.float32)
            sd[key] = t
            continue
        u = uniform_pm1_f32(seed, _stream_of(key), n)
        fan = int(np.prod(shape[1:])) if len(shape) > 1 else 1
        if "layer_norm.weight" in key:
            v = 1.0 + 0.1 * u
        elif "layer_norm.bias" in key:
            v = 0.1 * u
        elif key.endswith(".bias"):
            v = 0.02 * u
        elif ".conv" in key or "fc1" in key:
            v = math.sqrt(6.0 / fan) * u
        else:
            v = math.sqrt(3.0 / fan) * u
        sd[key] = np.asarray(v, dtype=np.float32).reshape(shape)
    return sd


def synth_state_dict(spec, seed: int | None = None) -> dict[str, np.ndarray]:
    if isinstance(spec, WavLMSpec):
        return synth_wavlm_state_dict(spec, 7 if seed is None else seed)
    return synth_whisper_state_dict(spec, 11 if seed is None else seed)


def outlier_weights(sd: dict, seed: int = 3, n_out: int = 4, gain: float = 30.0, dof: int = 3) -> dict:
    """A heavy-tailed variant of a synthetic state dict, shaped like real checkpoints' outlier
    features (stress fixtures for the bf16 / fp8 bars):

    * every LayerNorm / GroupNorm gain gets ``n_out`` channels (picked per tensor by the counter
      hash) multiplied by ``gain`` -- a few feature dimensions an order of magnitude above the rest;
    * every projection / conv weight (not biases, embeddings, positions or the positional conv's
      weight-norm factors) is redrawn Student-t with ``dof`` degrees of freedom, rescaled to the
      uniform tensor's standard deviation (same scale, far heavier tails).

    Deterministic per key (same transform for the HF-loadable and the packed dictionaries)."""
    out = {}
    for key, v in sd.items():
        v = np.asarray(v)
        if "layer_norm.weight" in key:
            w = v.astype(np.float32).copy().reshape(-1)
            u = uniform01(seed, _stream_of(key + "#out"), n_out)
            ch = np.unique((u * w.size).astype(np.int64))
            w[ch] *= np.float32(gain)
            out[key] = w.reshape(v.shape)
            continue
        skip = (v.ndim < 2 or key.endswith(".bias") or "embed" in key or "parametrizations" in key
                or key.endswith("[0]") or "rel_attn" in key or "gru_rel_pos" in key)
        if skip:
            out[key] = v
            continue
        n = v.size
        st = _stream_of(key + "#t")
        z = gaussian(seed, st, n)
        chi = np.zeros(n)
        for k in range(dof):
            chi += gaussian(seed, st + 1 + k, n) ** 2
        t = z / np.sqrt(chi / dof)                       # Student-t(dof), variance dof / (dof - 2)
        t *= float(np.std(v)) / math.sqrt(dof / (dof - 2.0))
        out[key] = t.astype(np.float32).reshape(v.shape)
    return out
