"""Synthetic generator determinism and HF state-dict packing (host logic, CPU only)."""
import numpy as np
import pytest


def test_clips_deterministic_and_independent():
    from ssr_amd import synth
    a = synth.synth_clips(4, 1000, seed=3)
    b = synth.synth_clips(2, 1000, seed=3, first_clip=2)
    assert np.array_equal(a[2:], b)
    assert a.dtype == np.float32 and np.abs(a).max() <= 1.0
    assert not np.array_equal(a[0], a[1])
    assert abs(float(a.std()) - np.sqrt(0.1 ** 2 + 3 * 0.08 ** 2 / 2)) < 0.02


def test_uniform_grid_and_range():
    from ssr_amd import synth
    u = synth.uniform_pm1_f32(1, 2, 100000)
    assert u.min() >= -1.0 and u.max() < 1.0
    assert np.all(u * 2 ** 23 == np.round(u * 2 ** 23))
    assert abs(float(u.mean())) < 0.01


def test_pack_weights_roundtrip_hf_model(wavlm_sd):
    import torch
    from transformers import WavLMConfig, WavLMModel
    from ssr_amd import config as C
    from ssr_amd.model import pack_weights
    m = WavLMModel(WavLMConfig())
    m.load_state_dict({k: torch.from_numpy(v) for k, v in wavlm_sd.items()}, strict=False)
    blob_hf = pack_weights(C.WAVLM_BASE, m.state_dict())
    blob_np = pack_weights(C.WAVLM_BASE, wavlm_sd)
    assert blob_hf.size == C.weight_floats(C.WAVLM_BASE)
    assert np.array_equal(blob_hf, blob_np)


def test_pack_weights_legacy_weight_norm_names(wavlm_sd):
    from ssr_amd import config as C
    from ssr_amd.model import pack_weights
    sd = dict(wavlm_sd)
    p = "encoder.pos_conv_embed.conv."
    sd[p + "weight_g"] = sd.pop(p + "parametrizations.weight.original0")
    sd[p + "weight_v"] = sd.pop(p + "parametrizations.weight.original1")
    assert np.array_equal(pack_weights(C.WAVLM_BASE, sd), pack_weights(C.WAVLM_BASE, wavlm_sd))


def test_pack_weights_rejects_bad_shapes(wavlm_sd):
    from ssr_amd import config as C
    from ssr_amd.model import pack_weights
    sd = dict(wavlm_sd)
    sd["feature_projection.projection.bias"] = np.zeros(5, np.float32)
    with pytest.raises(ValueError):
        pack_weights(C.WAVLM_BASE, sd)
    del sd["feature_projection.projection.bias"]
    with pytest.raises(KeyError):
        pack_weights(C.WAVLM_BASE, sd)


def test_frames_match_hf():
    from ssr_amd import config as C
    for L, T in ((48000, 149), (16000, 49), (400, 1), (160000, 499)):
        assert C.WAVLM_BASE.frames(L) == T
    assert C.WAVLM_BASE.default_layer_indices() == [12, 11, 10, 6]
    assert C.WAVLM_LARGE.default_layer_indices() == [24, 23, 22, 12]
    assert C.WHISPER_LARGE_V2.default_layer_indices() == [32, 31, 30]


def test_whisper_decoder_compact_and_hf_tables_pack_identically():
    """The compact "[0]"-row decoder dict and the HF-loadable full tables pack to the same blob."""
    from ssr_amd import config as C, synth
    from ssr_amd.model import pack_weights
    sd = synth.synth_whisper_state_dict(C.WHISPER_TINY_DEC)
    full = synth.synth_whisper_state_dict(C.WHISPER_TINY_DEC, full_hf=True)
    assert full["decoder.embed_tokens.weight"].shape == (51865, 384)
    assert np.array_equal(full["decoder.embed_tokens.weight"][0], sd["decoder.embed_tokens.weight[0]"])
    a, b = pack_weights(C.WHISPER_TINY_DEC, sd), pack_weights(C.WHISPER_TINY_DEC, full)
    assert a.size == C.weight_floats(C.WHISPER_TINY_DEC) and np.array_equal(a, b)
    # the encoder part of the blob is unchanged by adding the decoder
    enc = pack_weights(C.WHISPER_TINY, synth.synth_whisper_state_dict(C.WHISPER_TINY))
    assert np.array_equal(a[:enc.size], enc)
