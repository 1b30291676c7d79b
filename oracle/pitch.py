"""ORACLE (test infrastructure only): numpy restatement of the pitch branch of model_training_01's
augment_audio (REF/model_training_01.py:172-177):
``torchaudio.transforms.PitchShift(sample_rate, n_steps=n_steps)(waveform)``.

torchaudio is a third-party dependency ABSENT from this image and unpinned by the reference (no
requirements file).  Restated from its published 2.x algorithm with the transform's defaults
(bins_per_octave 12, n_fft 512, win_length 512, hop 128, torch.hann_window periodic):

  rate = 2.0 ** (-n_steps / 12)
  _stretch_waveform:
    X  = torch.stft(x, 512, 128, 512, hann, center=True, pad_mode="reflect", onesided=True)
    pa = torch.linspace(0, pi * 128, 257)[:, None]
    Y  = phase_vocoder(X, rate, pa):
           ts = arange(0, T, rate); alpha = ts % 1; X padded with 2 zero frames
           X0 = X[:, ts.long()], X1 = X[:, ts.long() + 1]
           ph = angle(X1) - angle(X0) - pa; ph -= 2pi * round(ph / 2pi); ph += pa
           ph = cat([angle(X[:, :1]), ph[:, :-1]]); acc = cumsum(ph)
           Y  = polar(alpha * |X1| + (1 - alpha) * |X0|, acc)
    xs = torch.istft(Y, 512, 128, 512, hann, length=round(L / rate))
  resample(xs, int(sample_rate / rate), sample_rate)  (oracle/resample.py)
  _fix_waveform_shape: truncate or zero-pad to L

The element-wise chain is evaluated in float32 op by op (torch's CPU tensor ops), the cumsum in
float64 (ATen's CPU cumsum accumulates in acc_type<float> = double), the FFTs in float64 and
rounded to float32 (torch: pocketfft in float32; last-ulp differences).  The arange / linspace
tables follow ATen's CPU kernels (RangeFactoriesKernel.cpp) on an AVX2 build: 2 x 8-lane vectors
per step, each vector = base + i*step from its first index, the scalar formula on the tail (an
AVX-512 build differs in the last ulp of some entries).  PARITY UNPINNED against torchaudio
itself (no offline fixture of it exists); the restatement is checked by properties in
tests/test_ingest_cpu.py (n_steps = 0 reconstructs the clip, a tone moves by 2^(n/12), length).
"""
from __future__ import annotations

import math

import numpy as np

from .resample import resample

N_FFT, HOP, BINS = 512, 128, 257


def hann512() -> np.ndarray:
    n = np.arange(N_FFT + 1, dtype=np.float32)
    c = np.cos(n * np.float32(math.pi * 2.0 / N_FFT))
    return (c * np.float32(-0.5) + np.float32(0.5))[:N_FFT].astype(np.float32)


def _vec_chunks(n: int):
    """(first index, lane) of each element under cpu_serial_kernel_vec, or (-1, -1) on the tail."""
    i = np.arange(n)
    nv = (n // 16) * 16
    k0 = np.where(i < nv, i & ~7, -1)
    return i, k0, nv


def arange_ts(n: int, rate: float) -> np.ndarray:
    i, k0, nv = _vec_chunks(n)
    base = (rate * np.maximum(k0, 0).astype(np.float64)).astype(np.float32).astype(np.float64)
    vec = (base + (i - np.maximum(k0, 0)).astype(np.float64) * rate).astype(np.float32)
    tail = (rate * i.astype(np.float64)).astype(np.float32)
    return np.where(i < nv, vec, tail).astype(np.float32)


def linspace_pa() -> np.ndarray:
    end = np.float32(math.pi * HOP)
    step = np.float32(end / np.float32(256.0))
    i, k0, nv = _vec_chunks(BINS)
    k0c = np.maximum(k0, 0)
    base = np.where(k0c < 128, np.float32(0.0) + step * k0c.astype(np.float32),
                    end - step * (BINS - k0c - 1).astype(np.float32)).astype(np.float32)
    vec = (base + (i - k0c).astype(np.float32) * step).astype(np.float32)
    return np.where(i < nv, vec, end).astype(np.float32)


def stft(x: np.ndarray) -> np.ndarray:
    """[L] -> complex64 [T][257] (frames x bins)."""
    w = hann512()
    xp = np.pad(np.asarray(x, dtype=np.float32), N_FFT // 2, mode="reflect")
    T = 1 + (xp.size - N_FFT) // HOP
    fr = np.lib.stride_tricks.as_strided(xp, shape=(T, N_FFT), strides=(HOP * 4, 4))
    return np.fft.rfft((fr * w).astype(np.float64), axis=1).astype(np.complex64)


def phase_vocoder(X: np.ndarray, rate: float) -> np.ndarray:
    """complex64 [T][257] -> complex64 [ceil(T/rate)][257]."""
    if rate == 1.0:
        return X.copy()
    T = X.shape[0]
    n = int(math.ceil(T / rate))
    ts = arange_ts(n, rate)
    i0 = ts.astype(np.int64)
    alpha = (ts - np.floor(ts)).astype(np.float32)[:, None]
    pa = linspace_pa()[None, :]
    Xp = np.concatenate([X, np.zeros((2, X.shape[1]), np.complex64)])
    c0, c1 = Xp[i0], Xp[i0 + 1]
    a0, a1 = np.angle(c0).astype(np.float32), np.angle(c1).astype(np.float32)
    n0, n1 = np.abs(c0).astype(np.float32), np.abs(c1).astype(np.float32)
    tp = np.float32(2 * math.pi)
    ph = (a1 - a0 - pa).astype(np.float32)
    ph = (ph - tp * np.rint(ph / tp)).astype(np.float32)
    ph = (ph + pa).astype(np.float32)
    ph = np.concatenate([np.angle(X[:1]).astype(np.float32), ph[:-1]])
    acc = np.cumsum(ph.astype(np.float64), axis=0).astype(np.float32)
    mag = (alpha * n1 + (np.float32(1.0) - alpha) * n0).astype(np.float32)
    return (mag * np.cos(acc) + 1j * (mag * np.sin(acc))).astype(np.complex64)


def istft(Y: np.ndarray, length: int) -> np.ndarray:
    """complex64 [n][257] -> float32 [length] (center trim, window-envelope normalised)."""
    w = hann512()
    n = Y.shape[0]
    fr = (np.fft.irfft(Y.astype(np.complex128), n=N_FFT, axis=1).astype(np.float32) * w).astype(np.float32)
    exp_len = N_FFT + HOP * (n - 1)
    y = np.zeros(exp_len, np.float64)
    env = np.zeros(exp_len, np.float64)
    for t in range(n):
        y[t * HOP:t * HOP + N_FFT] += fr[t]
        env[t * HOP:t * HOP + N_FFT] += (w * w).astype(np.float32)
    s = N_FFT // 2
    y, env = y[s:s + length], env[s:s + length]
    out = np.zeros(length, np.float32)
    out[:y.size] = (y / env).astype(np.float32)
    return out


def pitch_shift(x: np.ndarray, sample_rate: int, n_steps: int) -> np.ndarray:
    """[L] float32 -> [L] float32 (no clamp: augment_audio clamps afterwards)."""
    x = np.asarray(x, dtype=np.float32).reshape(-1)
    L = x.size
    if L <= N_FFT // 2:
        raise ValueError("reflect padding needs more than n_fft/2 samples (torch.stft raises)")
    rate = 2.0 ** (-float(n_steps) / 12)
    xs = istft(phase_vocoder(stft(x), rate), int(round(L / rate)))
    y = resample(xs, int(sample_rate / rate), sample_rate)
    out = np.zeros(L, np.float32)
    m = min(L, y.size)
    out[:m] = y[:m]
    return out
