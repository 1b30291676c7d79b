"""Ingest on the GPU: mono mix and torchaudio-compatible resampling.

Restates the transform half of the reference's ``load_audio`` (REF/WavLM_embeddings.py:87-125,
REF/whisper_embeddings_large.py:78-96, REF/model_training_1.py:216-233):
``torch.mean(waveform, dim=0)`` for multi-channel files, then
``torchaudio.transforms.Resample(sample_rate, 16000)`` (sinc_interp_hann, width 6, rolloff
0.99).  Both run in libsse.so (``sse_mono`` / ``sse_resample``); there is no CPU fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def mono(x: torch.Tensor) -> torch.Tensor:
    """[C, L] or [B, C, L] fp32 on a GPU -> [L] / [B, L] channel mean."""
    if x.device.type != "cuda":
        raise ValueError("ingest runs on a GPU device (no CPU fallback)")
    squeeze = x.dim() == 2
    x = (x[None] if squeeze else x).to(torch.float32).contiguous()
    B, C, L = x.shape
    y = torch.empty((B, L), dtype=torch.float32, device=x.device)
    _lib.check(_lib.lib().sse_mono(x.data_ptr(), B, C, L, y.data_ptr(), _stream(x.device)), "sse_mono")
    return y[0] if squeeze else y


def resampled_length(n: int, orig_freq: int, new_freq: int) -> int:
    return int(_lib.lib().sse_resample_length(int(n), int(orig_freq), int(new_freq)))


def resample(x: torch.Tensor, orig_freq: int, new_freq: int) -> torch.Tensor:
    """[L] or [B, L] fp32 on a GPU -> [..., ceil(new*L/orig)] (torchaudio Resample default)."""
    if x.device.type != "cuda":
        raise ValueError("ingest runs on a GPU device (no CPU fallback)")
    squeeze = x.dim() == 1
    x = (x[None] if squeeze else x).to(torch.float32).contiguous()
    B, L = x.shape
    L_ = _lib.lib()
    Lo = resampled_length(L, orig_freq, new_freq)
    n = L_.sse_resample_workspace_bytes(B, L, int(orig_freq), int(new_freq))
    ws = torch.empty(max(n, 256), dtype=torch.uint8, device=x.device)
    y = torch.empty((B, Lo), dtype=torch.float32, device=x.device)
    _lib.check(L_.sse_resample(x.data_ptr(), B, L, int(orig_freq), int(new_freq), y.data_ptr(), ws.data_ptr(),
                               ws.numel(), _stream(x.device)), "sse_resample")
    return y[0] if squeeze else y


def to_16k_mono(wav: np.ndarray, sr: int, target_sr: int = 16000, device=None) -> torch.Tensor:
    """[C, L] host samples (read_wav layout) -> [L'] fp32 on ``device``: mono mix then resample,
    the order of the reference's load_audio."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    x = torch.from_numpy(np.ascontiguousarray(np.asarray(wav, dtype=np.float32))).to(dev)
    if x.dim() == 1:
        x = x[None]
    x = mono(x) if x.shape[0] > 1 else x[0]
    if sr != target_sr:
        x = resample(x, sr, target_sr)
    return x
