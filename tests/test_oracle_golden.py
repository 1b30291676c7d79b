"""Pins the oracle (oracle/*.py) to the reference: fixtures in tests/golden/ were produced by
running REF/WavLM_embeddings.py:extract_wavlm_embeddings and
REF/whisper_embeddings_large.py:extract_whisper_embeddings_fixed themselves
(tests/golden/make_golden.py).  Inputs are regenerated from seeds and checked by SHA-256."""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN

ORACLE_TOL = 1e-5     # fp32 restatement vs fp32 reference (observed ~1e-6)


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _rel(a, b):
    return np.linalg.norm(a - b, axis=-1) / np.linalg.norm(b, axis=-1)


def test_inputs_match_manifest(wavlm_clips, wavlm_sd, golden_manifest):
    m = golden_manifest["wavlm_base"]
    assert _sha(wavlm_clips) == m["clips_sha256"]
    h = hashlib.sha256()
    for k in sorted(wavlm_sd):
        h.update(k.encode())
        h.update(np.ascontiguousarray(wavlm_sd[k]).tobytes())
    assert h.hexdigest() == m["weights_sha256"]


def test_wavlm_oracle_vs_reference(wavlm_clips, wavlm_sd, golden_wavlm):
    from oracle.wavlm import WavLMOracle
    from ssr_amd import config as C
    o = WavLMOracle(C.WAVLM_BASE, wavlm_sd)
    idx = [int(i) for i in golden_wavlm["layer_indices"]]
    got = o.embed(wavlm_clips[:3], idx)
    assert _rel(got, golden_wavlm["emb_norm0"][:3]).max() <= ORACLE_TOL
    got1 = o.embed(wavlm_clips[:2], idx, do_normalize=True)
    assert _rel(got1, golden_wavlm["emb_norm1"][:2]).max() <= ORACLE_TOL


def test_wavlm_oracle_intermediates(wavlm_clips, wavlm_sd, golden_wavlm):
    from oracle.wavlm import WavLMOracle
    from ssr_amd import config as C
    o = WavLMOracle(C.WAVLM_BASE, wavlm_sd)
    fe = o.feature_encoder(wavlm_clips[0])
    ref = golden_wavlm["frontend_clip0"]
    assert np.linalg.norm(fe - ref) / np.linalg.norm(ref) <= ORACLE_TOL
    hs = o.hidden_states(wavlm_clips[0])
    for k, i in (("hs0_clip0", 0), ("hs1_clip0", 1)):
        assert np.linalg.norm(hs[i] - golden_wavlm[k]) / np.linalg.norm(golden_wavlm[k]) <= ORACLE_TOL
    pooled = np.stack([h.mean(0) for h in hs])
    assert _rel(pooled, golden_wavlm["emb_all_layers"][0]).max() <= ORACLE_TOL


def test_whisper_oracle_vs_reference(golden_manifest):
    from oracle.whisper import WhisperOracle, log_mel
    from ssr_amd import config as C, synth
    g = np.load(os.path.join(GOLDEN, "whisper_tiny.npz"))
    man = golden_manifest["whisper_tiny"]
    clips = [synth.synth_clips(1, int(16000 * d), seed=4321, first_clip=i)[0] for i, d in enumerate(man["durations_s"])]
    assert [_sha(c) for c in clips] == man["clips_sha256"]
    for i, c in enumerate(clips):
        assert np.abs(log_mel(c) - g["mel"][i]).max() <= 2e-5
    o = WhisperOracle(C.WHISPER_TINY, synth.synth_whisper_state_dict(C.WHISPER_TINY, seed=11))
    got = np.concatenate([o.embed(c[None], [int(i) for i in g["layer_indices"]]) for c in clips])
    assert _rel(got, g["emb"]).max() <= ORACLE_TOL


def test_mel_filters_match_hf():
    from oracle.whisper import mel_filters
    from transformers.audio_utils import mel_filter_bank
    hf = mel_filter_bank(201, 80, 0.0, 8000.0, 16000, norm="slaney", mel_scale="slaney")
    assert np.abs(mel_filters(80) - hf).max() <= 1e-12


def test_rel_buckets_match_hf():
    import torch
    from oracle.wavlm import rel_position_buckets
    from transformers.models.wavlm.modeling_wavlm import WavLMAttention
    att = WavLMAttention(768, 12)
    T = 600
    ctx = torch.arange(T)[:, None]
    mem = torch.arange(T)[None, :]
    ref = att._relative_positions_bucket(mem - ctx).numpy()
    assert np.array_equal(rel_position_buckets(T, T), ref)


def test_wavlm_large_oracle_vs_reference(golden_manifest):
    """WavLM-large shape: layer-norm conv frontend + stable-LN encoder."""
    from oracle.wavlm import WavLMOracle
    from ssr_amd import config as C, synth
    g = np.load(os.path.join(GOLDEN, "wavlm_large.npz"))
    man = golden_manifest["wavlm_large"]
    clips = synth.synth_clips(3, 48000, seed=77)
    assert _sha(clips) == man["clips_sha256"]
    o = WavLMOracle(C.WAVLM_LARGE, synth.synth_wavlm_state_dict(C.WAVLM_LARGE, seed=9))
    fe = o.feature_encoder(clips[0])
    assert np.linalg.norm(fe - g["frontend_clip0"]) / np.linalg.norm(g["frontend_clip0"]) <= ORACLE_TOL
    got = o.embed(clips[:2], [int(i) for i in g["layer_indices"]], do_normalize=True)
    assert _rel(got, g["emb"][:2]).max() <= ORACLE_TOL


def test_whisper_decoder_oracle_vs_reference(golden_manifest):
    """1-token decoder pass: decoder_layer_* embeddings of
    REF/whisper_embeddings_large.py:283-297 with the pinned synthetic decoder weights."""
    from oracle.whisper import WhisperOracle
    from ssr_amd import config as C, synth
    g = np.load(os.path.join(GOLDEN, "whisper_tiny.npz"))
    man = golden_manifest["whisper_tiny"]
    sd = synth.synth_whisper_state_dict(C.WHISPER_TINY_DEC, seed=11)
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(np.ascontiguousarray(sd[k]).tobytes())
    assert h.hexdigest() == man["decoder_weights_sha256"]
    clips = [synth.synth_clips(1, int(16000 * d), seed=4321, first_clip=i)[0] for i, d in enumerate(man["durations_s"])]
    o = WhisperOracle(C.WHISPER_TINY_DEC, sd)
    enc_idx = [int(i) for i in g["layer_indices"]]
    dec_idx = [int(i) for i in g["decoder_indices"]]
    for i, c in enumerate(clips):
        enc, dec = o.embed_both(c[None], enc_idx, dec_idx)
        assert _rel(enc[0], g["emb"][i]).max() <= ORACLE_TOL
        assert _rel(dec[0], g["dec_emb"][i]).max() <= ORACLE_TOL


def test_aten_restatement_matches_reference(wavlm_clips, wavlm_sd, golden_wavlm):
    """bench.py's cpu_baseline (oracle/wavlm_aten.py: the reference's batch-1 loop on the same ATen
    ops) reproduces the reference's own fixture, with and without do_normalize."""
    from oracle.wavlm_aten import WavLMAten
    from ssr_amd import config as C
    o = WavLMAten(C.WAVLM_BASE, wavlm_sd)
    idx = [int(i) for i in golden_wavlm["layer_indices"]]
    for norm, n in ((0, 4), (1, 4)):
        got = o.embed(wavlm_clips[:n], idx, do_normalize=bool(norm))
        ref = golden_wavlm[f"emb_norm{norm}"][:n]
        rel = np.linalg.norm(got - ref, axis=-1) / np.linalg.norm(ref, axis=-1)
        assert rel.max() <= 1e-5, (norm, rel.max())


def test_oracles_vs_outlier_fixtures():
    """The stress fixtures (heavy-tailed weights with outlier LayerNorm channels, synth.outlier_weights,
    run through the reference's own glue): the numpy oracles reproduce them within fp32 round-off.
    The outlier channels make the network ill-conditioned enough that two fp32 evaluations in
    different summation orders (numpy BLAS vs torch/MKL) differ by ~2e-5 in rel-L2 (1e-6 on the
    benign weights), so the pin here is the north star's fp32 bar, 1e-4."""
    from oracle.wavlm import WavLMOracle
    from oracle.whisper import WhisperOracle
    from ssr_amd import config as C, synth
    g = np.load(os.path.join(GOLDEN, "outlier.npz"))
    sd = synth.outlier_weights(synth.synth_wavlm_state_dict(C.WAVLM_BASE, seed=7))
    clips = synth.synth_clips(4, 48000, seed=1234)
    got = WavLMOracle(C.WAVLM_BASE, sd).embed(clips[:2], [int(i) for i in g["wavlm_layer_indices"]])
    ref = g["wavlm_emb"][:2]
    assert (np.linalg.norm(got - ref, axis=-1) / np.linalg.norm(ref, axis=-1)).max() <= 1e-4
    spec = C.WhisperSpec(d_model=512, layers=3, heads=8, ffn=2048, name="whisper-mx-test")
    sdw = synth.outlier_weights(synth.synth_whisper_state_dict(spec, seed=21))
    wc = synth.synth_clips(2, 48000, seed=99)
    got = WhisperOracle(spec, sdw).embed(wc[:1], [int(i) for i in g["whisper_layer_indices"]])
    ref = g["whisper_emb"][:1]
    assert (np.linalg.norm(got - ref, axis=-1) / np.linalg.norm(ref, axis=-1)).max() <= 1e-4


def test_whisper_aten_restatement_matches_reference(golden_manifest):
    """bench.py's Whisper cpu_baseline (oracle/whisper_aten.py: the reference's batch-1 loop on the
    same ATen ops, encoder + 1-token decoder) reproduces the reference's own whisper_tiny fixture:
    log-mel, encoder and decoder keys (observed bit-equal)."""
    from oracle.whisper_aten import WhisperAten
    from ssr_amd import config as C, synth
    g = np.load(os.path.join(GOLDEN, "whisper_tiny.npz"))
    man = golden_manifest["whisper_tiny"]
    clips = [synth.synth_clips(1, int(16000 * d), seed=4321, first_clip=i)[0] for i, d in enumerate(man["durations_s"])]
    o = WhisperAten(C.WHISPER_TINY_DEC, synth.synth_whisper_state_dict(C.WHISPER_TINY_DEC, seed=11))
    ei = [int(i) for i in g["layer_indices"]]
    di = [int(i) for i in g["decoder_indices"]]
    for i, c in enumerate(clips):
        assert np.abs(o.log_mel(c)[0].numpy() - g["mel"][i]).max() <= 1e-5
        d = o.extract(c, ei, di)
        assert _rel(np.stack([d[f"encoder_layer_{k}"] for k in ei]), g["emb"][i]).max() <= 1e-5
        assert _rel(np.stack([d[f"decoder_layer_{k}"] for k in di]), g["dec_emb"][i]).max() <= 1e-5


def test_whisper_small_oracle_vs_reference(golden_manifest):
    """openai/whisper-small shape (the reference's default Whisper, REF/whisper_embeddings_large.py:34):
    encoder and 1-token decoder embeddings of the reference's own glue, one clip (the second clip is
    covered by the GPU test), plus the fixture's input hashes."""
    from oracle.whisper import WhisperOracle
    from ssr_amd import config as C, synth
    g = np.load(os.path.join(GOLDEN, "whisper_small.npz"))
    man = golden_manifest["whisper_small"]
    clips = [synth.synth_clips(1, int(16000 * d), seed=4321, first_clip=i)[0] for i, d in enumerate(man["durations_s"])]
    assert [_sha(c) for c in clips] == man["clips_sha256"]
    o = WhisperOracle(C.WHISPER_SMALL_DEC, synth.synth_whisper_state_dict(C.WHISPER_SMALL_DEC, seed=11))
    enc, dec = o.embed_both(clips[0][None], [int(i) for i in g["layer_indices"]], [int(i) for i in g["decoder_indices"]])
    assert _rel(enc[0], g["emb"][0]).max() <= ORACLE_TOL
    assert _rel(dec[0], g["dec_emb"][0]).max() <= ORACLE_TOL
