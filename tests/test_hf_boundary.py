"""The zero-line-change boundary of INTEGRATION.md §1 on CPU: ``hf.WavLMModel.from_hf`` /
``hf.WhisperModel.from_hf`` read a real transformers model (REF/WavLM_embeddings.py:482-483,
REF/whisper_embeddings_large.py:437-438 load exactly such models) into a spec and the C-ABI
weight blob.  Checked here without a GPU:

* the config -> spec mapping (``wavlm_spec_from_config`` / ``whisper_spec_from_config``) gives
  the named specs the kernels and fixtures are built for, field by field (feat_extract_norm,
  do_stable_layer_norm, the relative-position buckets, the decoder tables);
* ``pack_weights(spec, hf_model.state_dict())`` is bit-identical to the blob of the synthetic state
  dict ``tests/golden/make_golden.py`` loaded into the same HF model (its sha256 is the manifest's),
  including the legacy ``weight_g`` / ``weight_v`` names and the full decoder embedding tables;
* ``from_hf`` itself hands ``SSEModel`` exactly that spec and state dict (SSEModel replaced by a
  recorder: the device half is the GPU suite's).
"""
import dataclasses
import hashlib

import numpy as np
import pytest
import torch


def _sd_sha(sd: dict) -> str:   # tests/golden/make_golden.py::_sd_sha
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(np.ascontiguousarray(sd[k]).tobytes())
    return h.hexdigest()


def _wavlm_large_config():
    from transformers import WavLMConfig
    # the config make_golden.py builds the wavlm-large fixture with (manifest "wavlm_large".config)
    return WavLMConfig(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16, intermediate_size=4096,
                       feat_extract_norm="layer", do_stable_layer_norm=True, conv_bias=False)


def _whisper_config(spec):
    from transformers import WhisperConfig
    # the config make_golden.py::whisper_golden builds for spec
    return WhisperConfig(d_model=spec.d_model, encoder_layers=spec.layers, encoder_attention_heads=spec.heads,
                         decoder_layers=spec.decoder_layers, decoder_attention_heads=spec.heads,
                         encoder_ffn_dim=spec.ffn, decoder_ffn_dim=spec.dec_ffn_dim, num_mel_bins=spec.n_mels,
                         vocab_size=spec.vocab_size, max_target_positions=spec.max_target_positions)


def test_wavlm_base_config_maps_to_base_spec():
    from transformers import WavLMConfig
    from ssr_amd import config as C, hf
    spec = hf.wavlm_spec_from_config(WavLMConfig())
    assert spec is C.WAVLM_BASE
    # the fields the kernels branch on, spelled out
    assert (spec.feat_norm_layer, spec.stable_layer_norm, spec.conv_bias) == (False, False, False)
    assert (spec.num_buckets, spec.max_distance, spec.pos_kernel, spec.pos_groups) == (320, 800, 128, 16)
    assert spec.conv_kernel == (10, 3, 3, 3, 3, 2, 2) and spec.conv_stride == (5, 2, 2, 2, 2, 2, 2)


def test_wavlm_large_config_maps_to_large_spec():
    from ssr_amd import config as C, hf
    spec = hf.wavlm_spec_from_config(_wavlm_large_config())
    assert spec is C.WAVLM_LARGE
    assert spec.feat_norm_layer and spec.stable_layer_norm


def test_wavlm_unknown_shape_keeps_its_fields():
    from transformers import WavLMConfig
    from ssr_amd import config as C, hf
    spec = hf.wavlm_spec_from_config(WavLMConfig(num_hidden_layers=6, num_buckets=160, max_bucket_distance=400))
    assert spec.layers == 6 and spec.num_buckets == 160 and spec.max_distance == 400
    assert dataclasses.replace(spec, layers=12, num_buckets=320, max_distance=800, name=C.WAVLM_BASE.name) == C.WAVLM_BASE
    with pytest.raises(NotImplementedError):
        hf.wavlm_spec_from_config(WavLMConfig(feat_extract_norm="batch"))


@pytest.mark.parametrize("name", ["WHISPER_TINY", "WHISPER_SMALL", "WHISPER_LARGE_V2"])
def test_whisper_configs_map_to_named_specs(name):
    from ssr_amd import config as C, hf
    dec = getattr(C, name + "_DEC")
    cfg = _whisper_config(dec)
    assert hf.whisper_spec_from_config(cfg) is dec
    assert hf.whisper_spec_from_config(cfg, with_decoder=False) is getattr(C, name)
    s = hf.whisper_spec_from_config(cfg)
    assert (s.vocab_size, s.max_target_positions, s.max_positions, s.n_mels) == (51865, 448, 1500, 80)


def test_whisper_head_mismatch_rejected():
    from transformers import WhisperConfig
    from ssr_amd import hf
    with pytest.raises(NotImplementedError):
        hf.whisper_spec_from_config(WhisperConfig(encoder_attention_heads=4, decoder_attention_heads=8))


def _hf_wavlm(cfg, sd):
    from transformers import WavLMModel
    m = WavLMModel(cfg)
    missing, unexpected = m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    assert not unexpected and set(missing) == {"masked_spec_embed"}, (missing, unexpected)
    return m


def test_wavlm_large_pack_from_hf_state_dict(golden_manifest):
    """The blob packed from the HF model's own state_dict() equals the fixture's synthetic weights."""
    from ssr_amd import config as C, hf, synth
    from ssr_amd.model import pack_weights
    sd = synth.synth_wavlm_state_dict(C.WAVLM_LARGE, seed=9)
    assert _sd_sha(sd) == golden_manifest["wavlm_large"]["weights_sha256"]
    m = _hf_wavlm(_wavlm_large_config(), sd)
    spec = hf.wavlm_spec_from_config(m.config)
    blob = pack_weights(spec, m.state_dict())
    assert blob.size == C.weight_floats(C.WAVLM_LARGE)
    assert np.array_equal(blob, pack_weights(C.WAVLM_LARGE, sd))


def test_wavlm_base_pack_from_hf_legacy_weight_norm(wavlm_sd, golden_manifest):
    """An HF state dict whose pos-conv weight norm carries the legacy weight_g / weight_v names."""
    from transformers import WavLMConfig
    from ssr_amd import config as C
    from ssr_amd.model import pack_weights
    assert _sd_sha(wavlm_sd) == golden_manifest["wavlm_base"]["weights_sha256"]
    sd = dict(_hf_wavlm(WavLMConfig(), wavlm_sd).state_dict())
    p = "encoder.pos_conv_embed.conv."
    assert p + "parametrizations.weight.original0" in sd
    sd[p + "weight_g"] = sd.pop(p + "parametrizations.weight.original0")
    sd[p + "weight_v"] = sd.pop(p + "parametrizations.weight.original1")
    assert np.array_equal(pack_weights(C.WAVLM_BASE, sd), pack_weights(C.WAVLM_BASE, wavlm_sd))


@pytest.mark.parametrize("name", ["WHISPER_TINY", "WHISPER_SMALL"])
def test_whisper_pack_from_hf_state_dict_full_decoder_tables(name, golden_manifest):
    """Encoder + 1-token decoder from the HF model's state_dict(): the full embed_tokens /
    embed_positions tables are reduced to the row 0 the reference's decoder pass reads."""
    from transformers import WhisperModel
    from ssr_amd import config as C, hf, synth
    from ssr_amd.model import pack_weights
    dec = getattr(C, name + "_DEC")
    full = synth.synth_whisper_state_dict(dec, seed=11, full_hf=True)
    tag = name.lower()
    assert _sd_sha(synth.synth_whisper_state_dict(dec, seed=11)) == golden_manifest[tag]["decoder_weights_sha256"]
    m = WhisperModel(_whisper_config(dec))
    missing, unexpected = m.load_state_dict({k: torch.from_numpy(v) for k, v in full.items()}, strict=False)
    assert not missing and not unexpected, (missing, unexpected)
    sd = m.state_dict()
    assert tuple(sd["decoder.embed_tokens.weight"].shape) == (dec.vocab_size, dec.d_model)
    spec = hf.whisper_spec_from_config(m.config)
    blob = pack_weights(spec, sd)
    assert blob.size == C.weight_floats(dec)
    assert np.array_equal(blob, pack_weights(dec, synth.synth_whisper_state_dict(dec, seed=11)))
    # encoder-only: the blob is the decoder blob's prefix
    enc = pack_weights(hf.whisper_spec_from_config(m.config, with_decoder=False), sd)
    assert np.array_equal(enc, blob[:enc.size])


def test_from_hf_hands_spec_and_state_dict_to_sse_model(monkeypatch, wavlm_sd):
    """from_hf -> SSEModel(spec, hf_model.state_dict(), device, dtype), with SSEModel recorded."""
    from transformers import WavLMConfig, WhisperModel as HFWhisper
    from ssr_amd import config as C, hf, synth
    from ssr_amd.model import pack_weights
    seen = []

    class Recorder:
        def __init__(self, spec, state_dict, device="cuda:0", dtype="bf16", **kw):
            seen.append((spec, state_dict, device, dtype))
            self.spec, self.device = spec, torch.device("cpu")

    monkeypatch.setattr(hf, "SSEModel", Recorder)
    hf.WavLMModel.from_hf(_hf_wavlm(WavLMConfig(), wavlm_sd), device="cuda:3", dtype="bf16")
    spec, sd, dev, dt = seen[-1]
    assert spec is C.WAVLM_BASE and (dev, dt) == ("cuda:3", "bf16")
    assert np.array_equal(pack_weights(spec, sd), pack_weights(C.WAVLM_BASE, wavlm_sd))

    dec = C.WHISPER_TINY_DEC
    m = HFWhisper(_whisper_config(dec))
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synth.synth_whisper_state_dict(dec, full_hf=True).items()})
    w = hf.WhisperModel.from_hf(m, dtype="fp32")
    assert seen[-1][0] is dec and w.config.hidden_size == dec.d_model
    hf.WhisperModel.from_hf(m, with_decoder=False)
    assert seen[-1][0] is C.WHISPER_TINY
