"""CPU checks of the ingest row: the resampling oracle's properties
(torchaudio is absent: parity against torchaudio itself is UNPINNED, see oracle/resample.py)
and the on-disk embedding format (writer.py) against the reference's reader logic."""
import math
import os

import numpy as np
import pandas as pd
import pytest


def test_resample_identity_and_length():
    from oracle.resample import resample
    x = np.random.default_rng(0).standard_normal(1000).astype(np.float32)
    assert np.array_equal(resample(x, 16000, 16000), x)
    for sr in (8000, 22050, 32000, 44100, 48000):
        for L in (1, 7, 441, 1000, 44101):
            y = resample(np.zeros(L, np.float32), sr, 16000)
            assert y.shape == (math.ceil(16000 * L / sr),)


def test_resample_preserves_band_limited_tone():
    from oracle.resample import resample
    for sr in (22050, 44100, 48000, 8000):
        n = sr * 2
        t = np.arange(n) / sr
        f = 440.0 if sr > 8000 else 300.0
        x = (0.5 * np.sin(2 * np.pi * f * t)).astype(np.float32)
        y = resample(x, sr, 16000)
        ty = np.arange(y.shape[0]) / 16000
        ref = 0.5 * np.sin(2 * np.pi * f * ty)
        mid = slice(200, y.shape[0] - 200)               # away from the zero-padded edges
        assert np.abs(y[mid] - ref[mid]).max() < 2e-3, sr


def test_resample_linear_and_close_to_scipy_polyphase():
    from oracle.resample import resample
    from scipy.signal import resample_poly
    rng = np.random.default_rng(1)
    a, b = rng.standard_normal((2, 8820)).astype(np.float32)
    ya, yb, yab = resample(a, 44100, 16000), resample(b, 44100, 16000), resample(a + 2 * b, 44100, 16000)
    assert np.abs(yab - (ya + 2 * yb)).max() < 1e-5
    # an independent polyphase design agrees on low-pass content (different filter, same ideal)
    t = np.arange(44100) / 44100
    x = (np.sin(2 * np.pi * 1000 * t) + 0.3 * np.sin(2 * np.pi * 3100 * t)).astype(np.float32)
    y1 = resample(x, 44100, 16000)
    y2 = resample_poly(x, 160, 441)
    assert np.abs(y1[300:-300] - y2[300:-300]).max() < 5e-3


def test_kernel_rows_are_normalised():
    from oracle.resample import resample_kernel
    k, width, orig, new = resample_kernel(44100, 16000)
    assert (orig, new, width) == (441, 160, 17) and k.shape == (160, 2 * 17 + 441)
    assert np.allclose(k.sum(axis=1), 1.0, atol=2e-2)    # DC gain ~1 (rolloff 0.99, Hann window)


def test_mono_is_channel_mean():
    from oracle.resample import mono
    x = np.random.default_rng(2).standard_normal((3, 50)).astype(np.float32)
    assert np.array_equal(mono(x), ((x[0] + x[1]) + x[2]) / np.float32(3))


def _df(n, H, rng):
    return pd.DataFrame({"filename": [f"f{i}" for i in range(n)], "path": [f"/d/f{i}.wav" for i in range(n)],
                         "label": rng.integers(0, 2, n), "split": ["train"] * n,
                         "layer_12": list(rng.standard_normal((n, H)).astype(np.float32)),
                         "layer_6": list(rng.standard_normal((n, H)).astype(np.float32))})


def test_save_embeddings_reference_layout(tmp_path):
    from ssr_amd.writer import load_split, save_embeddings, write_split
    rng = np.random.default_rng(3)
    df = _df(5, 8, rng)
    save_embeddings(df, str(tmp_path / "a"), split="train", expected_dim=8)
    d = tmp_path / "a" / "train"
    assert sorted(os.listdir(d)) == ["embedding_metadata.csv", "layer_12_embeddings.npy", "layer_6_embeddings.npy"]
    meta = pd.read_csv(d / "embedding_metadata.csv")
    assert list(meta.columns) == ["filename", "path", "label", "split"]
    arr = np.load(d / "layer_12_embeddings.npy")
    assert arr.dtype == np.float32 and arr.shape == (5, 8) and np.array_equal(arr, np.stack(df["layer_12"]))
    # the reference reader's globbing (REF/model_training_1.py:128-139)
    m2, emb = load_split(str(tmp_path / "a"), "train")
    assert sorted(emb) == ["layer_12", "layer_6"] and m2.equals(meta)
    # the batched writer produces byte-identical files
    write_split(str(tmp_path / "b"), "train", df[["filename", "path", "label", "split"]],
                {"layer_12": np.stack(df["layer_12"]), "layer_6": np.stack(df["layer_6"])})
    for f in os.listdir(d):
        assert (d / f).read_bytes() == (tmp_path / "b" / "train" / f).read_bytes()


def test_whisper_columns_and_split_all(tmp_path):
    from ssr_amd.writer import save_embeddings
    df = pd.DataFrame({"filename": ["a", "b"], "encoder_layer_32": [np.ones(4, np.float32)] * 2,
                       "decoder_layer_30": [np.zeros(4, np.float32)] * 2})
    save_embeddings(df, str(tmp_path), split="all")
    assert sorted(os.listdir(tmp_path)) == ["decoder_layer_30_embeddings.npy", "embedding_metadata.csv",
                                            "encoder_layer_32_embeddings.npy"]


def test_shards_merge_in_corpus_order_and_resume(tmp_path):
    from ssr_amd.writer import ShardWriter, load_split, merge_shards, write_split
    rng = np.random.default_rng(4)
    N, H = 23, 6
    meta = pd.DataFrame({"filename": [f"f{i}" for i in range(N)], "label": rng.integers(0, 3, N)})
    emb = {"layer_12": rng.standard_normal((N, H)).astype(np.float32)}
    # two ranks, out-of-order writes, rank 1 "crashes" and re-writes a range after resume
    w0, w1 = ShardWriter(str(tmp_path), "devel", 0), ShardWriter(str(tmp_path), "devel", 1)
    for lo, hi, w in ((12, 18, w1), (0, 6, w0), (6, 12, w0), (18, 23, w1)):
        w.write(lo, meta.iloc[lo:hi], {k: v[lo:hi] for k, v in emb.items()})
    w1b = ShardWriter(str(tmp_path), "devel", 1)
    assert sorted(w1b.done()) == [(12, 6), (18, 5)]
    w1b.write(18, meta.iloc[18:23], {k: v[18:23] for k, v in emb.items()})
    assert merge_shards(str(tmp_path), "devel", expected_dim=H) == N
    m, e = load_split(str(tmp_path), "devel")
    assert np.array_equal(e["layer_12"], emb["layer_12"]) and list(m["filename"]) == list(meta["filename"])
    write_split(str(tmp_path / "ref"), "devel", meta, emb)
    assert (tmp_path / "devel" / "layer_12_embeddings.npy").read_bytes() == \
        (tmp_path / "ref" / "devel" / "layer_12_embeddings.npy").read_bytes()


def test_merge_detects_gap(tmp_path):
    from ssr_amd.writer import ShardWriter, merge_shards
    w = ShardWriter(str(tmp_path), None, 0)
    w.write(0, [{"filename": "a"}], {"layer_1": np.zeros((1, 2), np.float32)})
    w.write(2, [{"filename": "c"}], {"layer_1": np.zeros((1, 2), np.float32)})
    with pytest.raises(ValueError):
        merge_shards(str(tmp_path))


def _ref_draws(rng, n, variant):
    """The random calls of the reference's augment_audio, restated line by line
    (REF/model_training_1.py:179-200; REF/model_training_01.py:153-181)."""
    out = []
    for _ in range(n):
        if variant == "1":
            t = rng.choice(['speed', 'noise', 'volume', 'none'])
            if t == 'speed':
                f = rng.uniform(0.95, 1.05)
                out.append((t, f, int(16000 * f)))
            elif t == 'noise':
                out.append((t, rng.uniform(0.001, 0.005), 0))
            elif t == 'volume':
                out.append((t, rng.uniform(0.9, 1.1), 0))
            else:
                out.append((t, 1.0, 0))
        else:
            t = rng.choice(['speed', 'noise', 'pitch', 'volume'])
            if t == 'speed':
                f = rng.uniform(0.9, 1.1)
                out.append((t, f, int(16000 * f)))
            elif t == 'noise':
                out.append((t, rng.uniform(0.005, 0.02), 0))
            elif t == 'pitch':
                out.append((t, float(rng.randint(-2, 2)), 0))
            else:
                out.append((t, rng.uniform(0.8, 1.2), 0))
    return out


@pytest.mark.parametrize("variant", ["1", "01"])
def test_augmentation_draws_follow_reference_rng_order(variant):
    import random
    from ssr_amd.augment import draw
    ref = _ref_draws(random.Random(123), 200, variant)
    rng = random.Random(123)
    got = []
    for _ in range(200):
        s = draw(rng, variant)
        got.append((s.kind, float(s.n_steps) if s.kind == "pitch" else s.factor, s.new_sr))
    assert got == ref
    assert {k for k, _, _ in got} == set(["speed", "noise", "volume", "none"] if variant == "1"
                                         else ["speed", "noise", "pitch", "volume"])


def test_augment_oracle_ops():
    from oracle.augment import augment
    from ssr_amd import synth
    x = synth.synth_clips(1, 16000, seed=9)[0] * 8          # exceeds +-1 -> clamp matters
    assert np.abs(augment(x, "none")).max() <= 1.0
    v = augment(x, "volume", 0.5)
    assert np.array_equal(v, np.clip(x * np.float32(0.5), -1, 1))
    z = np.zeros(200000, np.float32)
    n = augment(z, "noise", 0.004, seed=1, stream=3)
    assert abs(n.std() - 0.004) < 1e-4 and abs(n.mean()) < 5e-5
    s = augment(synth.synth_clips(1, 48000, seed=2)[0], "speed", new_sr=int(16000 * 0.97))
    assert s.shape == (48000,)


def test_pitch_oracle_round_trip_and_tone():
    """oracle/pitch.py (torchaudio PitchShift restated, parity unpinned): n_steps = 0 is an
    STFT -> iSTFT round trip (Hann^2 envelope at hop n_fft/4 is exact), a tone moves to
    f * 2^(n/12), the length is kept, and the clamp of augment() follows."""
    from oracle.augment import augment
    from oracle.pitch import pitch_shift
    sr = 4000                                   # small co-prime resampling banks: seconds of CPU
    t = np.arange(8000) / sr
    x = (0.3 * np.sin(2 * np.pi * 200 * t)).astype(np.float32)
    assert np.abs(pitch_shift(x, sr, 0) - x).max() < 1e-6
    for n in (-2, -1, 1, 2):
        y = pitch_shift(x, sr, n)
        assert y.shape == x.shape
        seg = y[1000:7000]
        spec = np.abs(np.fft.rfft(seg * np.hanning(seg.size), n=8 * seg.size))
        f = np.argmax(spec) * sr / (8 * seg.size)
        assert abs(f / (200 * 2 ** (n / 12)) - 1) < 2e-3, (n, f)
    loud = x * 8
    assert np.abs(augment(loud, "pitch", sample_rate=sr, n_steps=1)).max() <= 1.0
    assert np.array_equal(augment(loud, "pitch", sample_rate=sr, n_steps=0), np.clip(loud, -1, 1))


def test_pitch_tables_follow_aten_cpu_kernels():
    from oracle.pitch import arange_ts, hann512, linspace_pa
    pa = linspace_pa()
    assert pa.dtype == np.float32 and pa.shape == (257,) and pa[0] == 0 and pa[-1] == np.float32(np.pi * 128)
    assert np.abs(pa - np.pi / 2 * np.arange(257)).max() < 1e-4
    rate = 2.0 ** (1 / 6)
    ts = arange_ts(37, rate)
    assert ts.shape == (37,) and np.abs(ts - rate * np.arange(37)).max() < 1e-5
    assert ts[-1] == np.float32(rate * 36)      # the tail (37 = 2*16 + 5) uses the scalar formula
    w = hann512()
    assert w[0] == 0 and w[256] == 1 and np.allclose(w, 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(512) / 512), atol=1e-7)


def test_pitch_short_clip_and_abi_sizes():
    from oracle.pitch import pitch_shift
    from ssr_amd import _lib
    with pytest.raises(ValueError):
        pitch_shift(np.zeros(256, np.float32), 16000, 1)
    L = _lib.lib()
    assert L.sse_pitch_shift_workspace_bytes(1, 256, 16000, 1) == 0      # reflect pad needs L > 256
    assert L.sse_pitch_shift_workspace_bytes(1, 16000, 16000, 99) == 0
    # 16 kHz, +2 semitones: the 17959 -> 16000 polyphase bank (16000 x 17973 fp32) dominates
    assert L.sse_pitch_shift_workspace_bytes(1, 16000, 16000, 2) > 16000 * 17973 * 4
