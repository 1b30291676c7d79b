"""WAV ingest used by the drop-in load_audio (REF/WavLM_embeddings.py:87-125), CPU only."""
import struct

import numpy as np
import pytest


def write_wav(path, x, sr=16000, fmt="pcm16"):
    """Test helper: mono/multichannel RIFF writer ([n] or [ch, n])."""
    x = np.atleast_2d(np.asarray(x, np.float32))
    ch, n = x.shape
    inter = x.T.reshape(-1)
    if fmt == "pcm16":
        data = np.clip(np.round(inter * 32768.0), -32768, 32767).astype("<i2").tobytes()
        code, bits = 1, 16
    else:
        data = inter.astype("<f4").tobytes()
        code, bits = 3, 32
    fmt_chunk = struct.pack("<HHIIHH", code, ch, sr, sr * ch * bits // 8, ch * bits // 8, bits)
    body = b"WAVE" + b"fmt " + struct.pack("<I", 16) + fmt_chunk + b"data" + struct.pack("<I", len(data)) + data
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", len(body)) + body)


def test_float_roundtrip(tmp_path):
    from ssr_amd.extract import load_audio
    x = np.linspace(-0.5, 0.5, 1000, dtype=np.float32)
    p = str(tmp_path / "f.wav")
    write_wav(p, x, fmt="float")
    assert np.array_equal(load_audio(p), x)


def test_pcm16_mono_trim_no_gpu_needed(tmp_path):
    """A 16 kHz mono file needs no transform, so load_audio works without a GPU."""
    from ssr_amd.extract import load_audio
    a = np.full(32000, 0.25, np.float32)
    p = str(tmp_path / "m.wav")
    write_wav(p, a, fmt="pcm16")
    y = load_audio(p, max_length=1.0)
    assert y.shape == (16000,)
    assert np.allclose(y, 0.25, atol=1e-4)


def test_bad_files_return_none(tmp_path):
    from ssr_amd.extract import load_audio
    p = tmp_path / "bad.wav"
    p.write_bytes(b"not a wav file")
    assert load_audio(str(p)) is None
    q = tmp_path / "trunc.wav"
    q.write_bytes(b"RIFF\x10\x00\x00\x00WAVEfmt ")
    assert load_audio(str(q)) is None        # missing data chunk
