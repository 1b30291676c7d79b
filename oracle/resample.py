"""ORACLE (test infrastructure only): numpy restatement of the reference's ingest transforms.

The reference resamples with ``torchaudio.transforms.Resample(sample_rate, 16000)`` and mixes
to mono with ``torch.mean(waveform, dim=0, keepdim=True)`` (REF/WavLM_embeddings.py:101-110,
REF/whisper_embeddings_large.py:78-96, REF/model_training_1.py:216-233).  torchaudio is a
third-party dependency that is ABSENT from this image and unpinned by the reference (no
requirements file); this file restates its published default algorithm
(``torchaudio.functional.functional._get_sinc_resample_kernel`` /
``_apply_sinc_resample_kernel``, torchaudio 2.x: method "sinc_interp_hann",
lowpass_filter_width 6, rolloff 0.99, kernel built in float64 and cast to float32, conv1d in
float32).  PARITY UNPINNED against torchaudio itself (no fixture of it exists offline); the
restatement is checked by properties (identity at equal rates, output length, band-limited
tone preservation, linearity) in tests/test_ingest_cpu.py.
"""
from __future__ import annotations

import math

import numpy as np


def resample_kernel(orig_freq: int, new_freq: int, lowpass_filter_width: int = 6, rolloff: float = 0.99,
                    rows=None):
    """-> (kernel float32 [new, 2*width + orig], width, orig, new) after dividing by the gcd.
    ``rows = (p0, p1)`` builds only phases p0..p1-1 (large co-prime rate pairs, e.g. pitch shift's
    int(16000/rate) -> 16000, have a 16000 x 17000 filter bank)."""
    g = math.gcd(int(orig_freq), int(new_freq))
    orig, new = int(orig_freq) // g, int(new_freq) // g
    base = min(orig, new) * rolloff
    width = math.ceil(lowpass_filter_width * orig / base)
    p0, p1 = (0, new) if rows is None else rows
    idx = np.arange(-width, width + orig, dtype=np.float64)[None, :] / orig
    # torch.arange(0, -new, -1) is int64; "/ new" promotes to the default float32, then "+ idx"
    # (float64) promotes to float64
    t = (np.arange(-p0, -p1, -1, dtype=np.int64)[:, None] / np.float32(new)).astype(np.float32).astype(np.float64)
    t = t + idx
    t = t * base
    t = np.clip(t, -lowpass_filter_width, lowpass_filter_width)
    window = np.cos(t * math.pi / lowpass_filter_width / 2) ** 2
    t = t * math.pi
    scale = base / orig
    with np.errstate(invalid="ignore", divide="ignore"):
        k = np.where(t == 0, 1.0, np.sin(t) / t)
    k = k * (window * scale)
    return k.astype(np.float32), width, orig, new


def _plan(orig_freq: int, new_freq: int, lowpass_filter_width: int = 6, rolloff: float = 0.99):
    g = math.gcd(int(orig_freq), int(new_freq))
    orig, new = int(orig_freq) // g, int(new_freq) // g
    return math.ceil(lowpass_filter_width * orig / (min(orig, new) * rolloff)), orig, new


def resample(wave: np.ndarray, orig_freq: int, new_freq: int) -> np.ndarray:
    """[..., L] float32 -> [..., ceil(new*L/orig)] float32 (torchaudio Resample default)."""
    if orig_freq == new_freq:
        return np.asarray(wave, dtype=np.float32).copy()
    width, orig, new = _plan(orig_freq, new_freq)
    x = np.asarray(wave, dtype=np.float32)
    shape = x.shape
    x = x.reshape(-1, shape[-1])
    n, L = x.shape
    xp = np.pad(x, ((0, 0), (width, width + orig)))
    K = 2 * width + orig
    n_blk = (xp.shape[1] - K) // orig + 1
    frames = np.lib.stride_tricks.as_strided(xp, shape=(n, n_blk, K), strides=(xp.strides[0], orig * 4, 4))
    frames = frames.astype(np.float64)
    out = np.empty((n, n_blk, new), dtype=np.float64)
    step = max(1, (1 << 22) // K)
    for p0 in range(0, new, step):
        k = resample_kernel(orig_freq, new_freq, rows=(p0, min(new, p0 + step)))[0]
        out[:, :, p0:p0 + k.shape[0]] = frames @ k.astype(np.float64).T
    out = out.reshape(n, -1)
    target = int(math.ceil(new * L / orig))
    return out[:, :target].astype(np.float32).reshape(shape[:-1] + (target,))


def mono(wave: np.ndarray) -> np.ndarray:
    """[C, L] -> [L]: torch.mean over channels (sum then divide, float32)."""
    x = np.asarray(wave, dtype=np.float32)
    if x.ndim == 1 or x.shape[0] == 1:
        return x.reshape(-1).copy()
    s = x[0].copy()
    for c in range(1, x.shape[0]):
        s = s + x[c]
    return (s / np.float32(x.shape[0])).astype(np.float32)
