"""The reference's call surface on the HIP path: WAV file in -> {"layer_<i>": float32[H]} out
(REF/WavLM_embeddings.py:267-341, REF/whisper_embeddings_large.py:234-299,
REF/model_training_1.py:235-316), checked against the golden outputs of the reference."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from test_wavio import write_wav

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return np.linalg.norm(a - b) / np.linalg.norm(b)


@pytest.fixture(scope="module")
def wavlm_pair(wavlm_sd):
    from ssr_amd import config as C
    from ssr_amd.hf import Wav2Vec2FeatureExtractor, WavLMModel
    return (WavLMModel.from_state_dict(C.WAVLM_BASE, wavlm_sd, device="cuda:0", dtype="fp32"),
            Wav2Vec2FeatureExtractor(do_normalize=False, device="cuda:0"))


def test_extract_wavlm_embeddings_files(tmp_path, wavlm_pair, wavlm_clips, golden_wavlm):
    from ssr_amd.extract import extract_wavlm_embeddings
    model, fe = wavlm_pair
    idx = [int(i) for i in golden_wavlm["layer_indices"]]
    for i in range(3):
        p = str(tmp_path / f"c{i}.wav")
        write_wav(p, wavlm_clips[i], fmt="float")
        d = extract_wavlm_embeddings(p, model, fe, "cuda:0", idx)
        assert list(d) == [f"layer_{j}" for j in idx]
        for j, k in enumerate(idx):
            v = d[f"layer_{k}"]
            assert v.dtype == np.float32 and v.shape == (768,)
            assert _rel(v, golden_wavlm["emb_norm0"][i, j]) <= 1e-4


def test_generic_hf_route_matches_fused(wavlm_pair, wavlm_clips, golden_wavlm):
    """The reference's own loop (model(...).hidden_states then torch.mean) on the duck model."""
    model, fe = wavlm_pair
    inputs = fe(wavlm_clips[0], sampling_rate=16000, return_tensors="pt").to("cuda:0")
    out = model(inputs.input_values, output_hidden_states=True, return_dict=True)
    assert len(out.hidden_states) == 13 and out.hidden_states[0].shape == (1, 149, 768)
    assert next(model.parameters()).device.type == "cuda" and model.config.hidden_size == 768
    for j, k in enumerate(golden_wavlm["layer_indices"]):
        v = torch.mean(out.hidden_states[int(k)], dim=1).cpu().numpy().flatten()
        assert _rel(v, golden_wavlm["emb_norm0"][0, j]) <= 1e-4


def test_errors_return_none(tmp_path, wavlm_pair):
    from ssr_amd.extract import extract_embeddings_from_audio_wavlm, extract_wavlm_embeddings
    model, fe = wavlm_pair
    assert extract_wavlm_embeddings(str(tmp_path / "missing.wav"), model, fe, "cuda:0", [12]) is None
    assert extract_embeddings_from_audio_wavlm(np.zeros(100, np.float32), model, fe, "cuda:0", [12]) is None
    d = extract_embeddings_from_audio_wavlm(np.zeros(16000, np.float32), model, fe, "cuda:0", [12, 40])
    assert list(d) == ["layer_12"]                  # out-of-range index warned and skipped (REF :324-325)


def test_normalizing_feature_extractor(wavlm_sd, wavlm_clips, golden_wavlm):
    from ssr_amd import config as C
    from ssr_amd.extract import extract_embeddings_from_audio_wavlm
    from ssr_amd.hf import Wav2Vec2FeatureExtractor, WavLMModel
    model = WavLMModel.from_state_dict(C.WAVLM_BASE, wavlm_sd, device="cuda:0", dtype="fp32")
    fe = Wav2Vec2FeatureExtractor(do_normalize=True, device="cuda:0")
    idx = [int(i) for i in golden_wavlm["layer_indices"]]
    d = extract_embeddings_from_audio_wavlm(wavlm_clips[1], model, fe, "cuda:0", idx)
    for j, k in enumerate(idx):
        assert _rel(d[f"layer_{k}"], golden_wavlm["emb_norm1"][1, j]) <= 1e-4


def test_extract_whisper_embeddings_fixed_files(tmp_path, golden_manifest):
    """Encoder AND decoder embeddings through the drop-in glue and through the reference's own
    generic route (processor -> model.encoder -> model.decoder), against the reference fixture."""
    from ssr_amd import config as C, synth
    from ssr_amd.extract import extract_whisper_embeddings_fixed
    from ssr_amd.hf import WhisperModel, WhisperProcessor
    g = np.load(os.path.join(GOLDEN, "whisper_tiny.npz"))
    model = WhisperModel.from_state_dict(C.WHISPER_TINY_DEC,
                                         synth.synth_whisper_state_dict(C.WHISPER_TINY_DEC, seed=11),
                                         device="cuda:0", dtype="fp32")
    proc = WhisperProcessor(feature_size=80, device="cuda:0")
    enc = [int(i) for i in g["layer_indices"]]
    dec = [int(i) for i in g["decoder_indices"]]
    clip = synth.synth_clips(1, 48000, seed=4321, first_clip=0)[0]
    p = str(tmp_path / "w.wav")
    write_wav(p, clip, fmt="float")
    d = extract_whisper_embeddings_fixed(p, model, proc, "cuda:0", enc, dec)
    assert list(d) == [f"encoder_layer_{i}" for i in enc] + [f"decoder_layer_{i}" for i in dec]
    for j, k in enumerate(enc):
        assert _rel(d[f"encoder_layer_{k}"], g["emb"][0, j]) <= 1e-4
    for j, k in enumerate(dec):
        assert d[f"decoder_layer_{k}"].shape == (384,)
        assert _rel(d[f"decoder_layer_{k}"], g["dec_emb"][0, j]) <= 1e-4
    # out-of-range indices are skipped (REF :274-297 logs a warning and moves on)
    d2 = extract_whisper_embeddings_fixed(p, model, proc, "cuda:0", [enc[0], 99], [dec[0], 99])
    assert list(d2) == [f"encoder_layer_{enc[0]}", f"decoder_layer_{dec[0]}"]
    # generic HF route through the processor + model.encoder + model.decoder (REF :242-262)
    feats = proc(clip, sampling_rate=16000, return_tensors="pt").input_features.to("cuda:0")
    out = model.encoder(feats, output_hidden_states=True, return_dict=True)
    v = torch.mean(out.hidden_states[enc[0]], dim=1).cpu().numpy().flatten()
    assert _rel(v, g["emb"][0, 0]) <= 1e-4
    do = model.decoder(input_ids=torch.zeros((1, 1), dtype=torch.long).to("cuda:0"),
                       encoder_hidden_states=out.last_hidden_state, output_hidden_states=True, return_dict=True)
    assert len(do.hidden_states) == C.WHISPER_TINY_DEC.decoder_layers + 1
    for j, k in enumerate(dec):
        u = do.hidden_states[k].squeeze(1).cpu().numpy().flatten()
        assert _rel(u, g["dec_emb"][0, j]) <= 1e-4
    with pytest.raises(NotImplementedError):
        model.decoder(input_ids=torch.ones((1, 1), dtype=torch.long), encoder_hidden_states=out.last_hidden_state)
