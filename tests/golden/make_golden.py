#!/usr/bin/env python3
"""Generate the golden fixtures by running the REFERENCE's own glue (container only).

Runs ``extract_wavlm_embeddings`` (REF/WavLM_embeddings.py:267-341) and
``extract_whisper_embeddings_fixed`` (REF/whisper_embeddings_large.py:234-299) exactly as
the reference calls them, on HF models (transformers, third-party, version recorded in
the manifest) built offline and loaded with the deterministic synthetic weights of
``synth.py`` (no hub access: SURVEY.md §8(c)).

* ``torchaudio`` is absent here; a stub whose ``load(path)`` returns the synthetic clip
  registered for that path is installed AFTER ``import transformers``.
* The reference is imported by path from a temp cwd (it creates ``logs/`` at import) with
  ``sys.dont_write_bytecode = True`` so nothing is written under /root/reference.
* Only inputs and outputs are written (small .npz files + manifest.json); nothing from the
  reference travels with them.

Usage: python tests/golden/make_golden.py [--skip-large]
"""
from __future__ import annotations

import argparse
import dataclasses
import hashlib
import importlib
import importlib.util
import json
import os
import sys
import tempfile
import time
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import transformers  # noqa: E402  (must precede the torchaudio stub)

ssr = importlib.import_module("stuttering-speech-representation_amd")
from ssr_amd import config as C, synth  # noqa: E402

REF = "/root/reference"
_CLIPS: dict[str, np.ndarray] = {}


def _install_torchaudio_stub():
    ta = types.ModuleType("torchaudio")

    def load(path):
        return torch.from_numpy(_CLIPS[path][None, :].copy()), 16000

    ta.load = load
    tr = types.ModuleType("torchaudio.transforms")

    class Resample:  # never used: every synthetic clip is already 16 kHz
        def __init__(self, *a, **k):
            raise RuntimeError("resample not expected")

    tr.Resample = Resample
    ta.transforms = tr
    sys.modules["torchaudio"] = ta
    sys.modules["torchaudio.transforms"] = tr


def _import_ref(name, fname):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, fname))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _sd_sha(sd: dict) -> str:
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(np.ascontiguousarray(sd[k]).tobytes())
    return h.hexdigest()


def _register(prefix, clips):
    paths = []
    for i, c in enumerate(clips):
        p = f"/synthetic/{prefix}_{i:03d}.wav"
        _CLIPS[p] = c
        paths.append(p)
    return paths


def wavlm_golden(ref_w, manifest):
    from transformers import Wav2Vec2FeatureExtractor, WavLMConfig, WavLMModel
    spec = C.WAVLM_BASE
    sd = synth.synth_wavlm_state_dict(spec, seed=7)
    model = WavLMModel(WavLMConfig())
    missing, unexpected = model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    assert not unexpected and set(missing) == {"masked_spec_embed"}, (missing, unexpected)
    model.eval()
    clips = synth.synth_clips(16, 48000, seed=1234)
    paths = _register("wavlm", clips)
    out = {}
    idx = spec.default_layer_indices()                  # [12, 11, 10, 6] (REF :506)
    for do_norm in (False, True):
        fe = Wav2Vec2FeatureExtractor(do_normalize=do_norm)
        n = 16 if not do_norm else 4
        t0 = time.time()
        embs = []
        for p in paths[:n]:
            d = ref_w.extract_wavlm_embeddings(p, model, fe, "cpu", idx)
            embs.append(np.stack([d[f"layer_{i}"] for i in idx]))
        out[f"emb_norm{int(do_norm)}"] = np.stack(embs).astype(np.float32)
        manifest[f"wavlm_emb_norm{int(do_norm)}_s"] = time.time() - t0
    # all 13 pooled layers for 2 clips through the same reference function
    fe = Wav2Vec2FeatureExtractor(do_normalize=False)
    all_idx = list(range(spec.num_hidden_states))
    out["emb_all_layers"] = np.stack([
        np.stack([ref_w.extract_wavlm_embeddings(p, model, fe, "cpu", all_idx)[f"layer_{i}"] for i in all_idx])
        for p in paths[:2]]).astype(np.float32)
    # intermediates of clip 0 for kernel-level tests
    with torch.no_grad():
        x = torch.from_numpy(clips[:1])
        feats = model.feature_extractor(x)                          # [1, 512, 149]
        hs = model(x, output_hidden_states=True).hidden_states
    out["frontend_clip0"] = feats[0].numpy().T.copy()           # [149, 512] channels-last
    out["hs0_clip0"] = hs[0][0].numpy().copy()
    out["hs1_clip0"] = hs[1][0].numpy().copy()
    out["layer_indices"] = np.array(idx, dtype=np.int32)
    np.savez_compressed(os.path.join(HERE, "wavlm_base.npz"), **out)
    manifest["wavlm_base"] = {
        "spec": spec.name, "weight_seed": 7, "clip_seed": 1234, "n_clips": 16, "n_samples": 48000,
        "weights_sha256": _sd_sha(sd), "clips_sha256": _sha(clips), "layer_indices": idx,
        "reference_fn": "REF/WavLM_embeddings.py:extract_wavlm_embeddings",
        "feature_extractor": "Wav2Vec2FeatureExtractor(do_normalize=False|True)",
    }


def wavlm_large_golden(ref_w, manifest):
    """WavLM-large shape (layer-norm conv frontend, stable-LN encoder)."""
    from transformers import Wav2Vec2FeatureExtractor, WavLMConfig, WavLMModel
    spec = C.WAVLM_LARGE
    sd = synth.synth_wavlm_state_dict(spec, seed=9)
    cfg = WavLMConfig(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16, intermediate_size=4096,
                      feat_extract_norm="layer", do_stable_layer_norm=True, conv_bias=False)
    model = WavLMModel(cfg)
    missing, unexpected = model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    assert not unexpected and set(missing) == {"masked_spec_embed"}, (missing, unexpected)
    model.eval()
    clips = synth.synth_clips(3, 48000, seed=77)
    paths = _register("wavlm_large", clips)
    idx = spec.default_layer_indices()                  # [24, 23, 22, 12]
    fe = Wav2Vec2FeatureExtractor(do_normalize=True)    # wavlm-large normalises its input
    t0 = time.time()
    emb = np.stack([np.stack([ref_w.extract_wavlm_embeddings(p, model, fe, "cpu", idx)[f"layer_{i}"] for i in idx])
                    for p in paths]).astype(np.float32)
    manifest["wavlm_large_s"] = time.time() - t0
    with torch.no_grad():
        feats = model.feature_extractor(torch.from_numpy(clips[:1]))
    np.savez_compressed(os.path.join(HERE, "wavlm_large.npz"), emb=emb, layer_indices=np.array(idx, np.int32),
                        frontend_clip0=feats[0].numpy().T.copy())
    manifest["wavlm_large"] = {"spec": spec.name, "weight_seed": 9, "clip_seed": 77, "n_clips": 3, "n_samples": 48000,
                               "weights_sha256": _sd_sha(sd), "clips_sha256": _sha(clips), "layer_indices": idx,
                               "reference_fn": "REF/WavLM_embeddings.py:extract_wavlm_embeddings",
                               "feature_extractor": "Wav2Vec2FeatureExtractor(do_normalize=True)",
                               "config": "WavLMConfig(1024/24/16/4096, feat_extract_norm=layer, "
                                         "do_stable_layer_norm=True, conv_bias=False)"}


def whisper_golden(ref_h, manifest, spec, tag, n_clips, seed, durations):
    """Encoder AND decoder embeddings from the reference glue.  ``spec`` carries decoder_layers;
    the decoder weights are the synthetic ``full_hf`` tables (row 0 == the compact blob's "[0]"
    rows), so the decoder fixture is pinned and reproducible anywhere."""
    from transformers import WhisperConfig, WhisperFeatureExtractor, WhisperModel
    enc_spec = dataclasses.replace(spec, decoder_layers=0, name=spec.name.split("+")[0])
    sd = synth.synth_whisper_state_dict(spec, seed=seed, full_hf=True)
    cfg = WhisperConfig(d_model=spec.d_model, encoder_layers=spec.layers, encoder_attention_heads=spec.heads,
                        decoder_layers=spec.decoder_layers, decoder_attention_heads=spec.heads,
                        encoder_ffn_dim=spec.ffn, decoder_ffn_dim=spec.dec_ffn_dim, num_mel_bins=spec.n_mels,
                        vocab_size=spec.vocab_size, max_target_positions=spec.max_target_positions)
    model = WhisperModel(cfg)
    missing, unexpected = model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    assert not unexpected and not missing, (missing, unexpected)
    model.eval()
    del sd
    clips = [synth.synth_clips(1, int(16000 * d), seed=4321, first_clip=i)[0] for i, d in enumerate(durations)]
    paths = _register(tag, clips)
    proc = WhisperFeatureExtractor(feature_size=spec.n_mels)
    enc_idx = spec.default_layer_indices()
    dec_idx = spec.default_decoder_indices() + [0]
    t0 = time.time()
    embs, decs = [], []
    for p in paths[:n_clips]:
        d = ref_h.extract_whisper_embeddings_fixed(p, model, proc, "cpu", enc_idx, dec_idx)
        embs.append(np.stack([d[f"encoder_layer_{i}"] for i in enc_idx]))
        decs.append(np.stack([d[f"decoder_layer_{i}"] for i in dec_idx]))
    manifest[f"{tag}_s"] = time.time() - t0
    mels = np.stack([proc(c, sampling_rate=16000, return_tensors="np").input_features[0] for c in clips[:n_clips]])
    out = {"emb": np.stack(embs).astype(np.float32), "layer_indices": np.array(enc_idx, np.int32),
           "mel": mels.astype(np.float32), "dec_emb": np.stack(decs).astype(np.float32),
           "decoder_indices": np.array(dec_idx, np.int32)}
    np.savez_compressed(os.path.join(HERE, f"{tag}.npz"), **out)
    manifest[tag] = {"spec": enc_spec.name, "decoder_spec": spec.name, "weight_seed": seed, "clip_seed": 4321,
                     "durations_s": durations[:n_clips], "clips_sha256": [_sha(c) for c in clips[:n_clips]],
                     "weights_sha256": _sd_sha(synth.synth_whisper_state_dict(enc_spec, seed=seed)),
                     "decoder_weights_sha256": _sd_sha(synth.synth_whisper_state_dict(spec, seed=seed)),
                     "layer_indices": enc_idx, "decoder_indices": dec_idx,
                     "reference_fn": "REF/whisper_embeddings_large.py:extract_whisper_embeddings_fixed",
                     "note": "decoder: input id 0 at position 0 (REF :257-262); synthetic full_hf decoder tables"}


# the fp8 (MX) GEMMs need d_model and ffn multiples of 256: the smallest Whisper shape of the MX tests
WHISPER_MX_DEC = C.WhisperSpec(d_model=512, layers=3, heads=8, ffn=2048, decoder_layers=1,
                               name="whisper-mx-test+decoder")


def outlier_golden(ref_w, ref_h, manifest):
    """Stress fixtures: heavy-tailed weights with outlier feature channels (synth.outlier_weights)
    through the reference's own glue -- WavLM-base (4 clips) and the MX-test Whisper shape (2 clips)."""
    from transformers import Wav2Vec2FeatureExtractor, WavLMConfig, WavLMModel
    from transformers import WhisperConfig, WhisperFeatureExtractor, WhisperModel
    spec = C.WAVLM_BASE
    sd = synth.outlier_weights(synth.synth_wavlm_state_dict(spec, seed=7))
    model = WavLMModel(WavLMConfig())
    missing, unexpected = model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    assert not unexpected and set(missing) == {"masked_spec_embed"}, (missing, unexpected)
    model.eval()
    clips = synth.synth_clips(4, 48000, seed=1234)
    paths = _register("wavlm_outlier", clips)
    idx = spec.default_layer_indices()
    fe = Wav2Vec2FeatureExtractor(do_normalize=False)
    t0 = time.time()
    emb = np.stack([np.stack([ref_w.extract_wavlm_embeddings(p, model, fe, "cpu", idx)[f"layer_{i}"] for i in idx])
                    for p in paths]).astype(np.float32)
    manifest["wavlm_outlier_s"] = time.time() - t0
    spec_w = WHISPER_MX_DEC
    sdw = synth.outlier_weights(synth.synth_whisper_state_dict(spec_w, seed=21, full_hf=True))
    cfg = WhisperConfig(d_model=spec_w.d_model, encoder_layers=spec_w.layers, encoder_attention_heads=spec_w.heads,
                        decoder_layers=spec_w.decoder_layers, decoder_attention_heads=spec_w.heads,
                        encoder_ffn_dim=spec_w.ffn, decoder_ffn_dim=spec_w.dec_ffn_dim, num_mel_bins=spec_w.n_mels,
                        vocab_size=spec_w.vocab_size, max_target_positions=spec_w.max_target_positions)
    wm = WhisperModel(cfg)
    missing, unexpected = wm.load_state_dict({k: torch.from_numpy(v) for k, v in sdw.items()}, strict=False)
    assert not unexpected and not missing, (missing, unexpected)
    wm.eval()
    wclips = synth.synth_clips(2, 48000, seed=99)
    wpaths = _register("whisper_outlier", wclips)
    proc = WhisperFeatureExtractor(feature_size=spec_w.n_mels)
    eidx = spec_w.default_layer_indices()
    t0 = time.time()
    wemb = np.stack([np.stack([ref_h.extract_whisper_embeddings_fixed(p, wm, proc, "cpu", eidx, [1, 0])[f"encoder_layer_{i}"]
                               for i in eidx]) for p in wpaths]).astype(np.float32)
    manifest["whisper_outlier_s"] = time.time() - t0
    np.savez_compressed(os.path.join(HERE, "outlier.npz"), wavlm_emb=emb, wavlm_layer_indices=np.array(idx, np.int32),
                        whisper_emb=wemb, whisper_layer_indices=np.array(eidx, np.int32))
    manifest["outlier"] = {"transform": "synth.outlier_weights(seed=3, n_out=4, gain=30, dof=3)",
                           "wavlm": {"spec": spec.name, "weight_seed": 7, "clip_seed": 1234, "n_clips": 4,
                                     "weights_sha256": _sd_sha(sd), "clips_sha256": _sha(clips)},
                           "whisper": {"spec": "d512/3 layers/8 heads/ffn 2048 (+1 decoder layer)", "weight_seed": 21,
                                       "clip_seed": 99, "n_clips": 2, "clips_sha256": _sha(wclips)},
                           "reference_fn": ["REF/WavLM_embeddings.py:extract_wavlm_embeddings",
                                            "REF/whisper_embeddings_large.py:extract_whisper_embeddings_fixed"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-large", action="store_true")
    ap.add_argument("--only", default=None, help="wavlm | wavlm_large | whisper_tiny | whisper_small | outlier | whisper_large_v2")
    args = ap.parse_args()
    torch.set_num_threads(os.cpu_count())
    manifest = {"transformers": transformers.__version__, "torch": torch.__version__, "numpy": np.__version__}
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as td:
        os.chdir(td)
        try:
            _install_torchaudio_stub()
            ref_w = _import_ref("ref_wavlm_embeddings", "WavLM_embeddings.py")
            ref_h = _import_ref("ref_whisper_embeddings_large", "whisper_embeddings_large.py")
            only = args.only
            if only in (None, "wavlm"):
                wavlm_golden(ref_w, manifest)
            if only in (None, "wavlm_large"):
                wavlm_large_golden(ref_w, manifest)
            if only in (None, "whisper_tiny"):
                whisper_golden(ref_h, manifest, C.WHISPER_TINY_DEC, "whisper_tiny", 2, 11, [3.0, 30.0])
            if only in (None, "outlier"):
                outlier_golden(ref_w, ref_h, manifest)
            if only in (None, "whisper_small"):   # the reference's default Whisper (REF :34)
                whisper_golden(ref_h, manifest, C.WHISPER_SMALL_DEC, "whisper_small", 2, 11, [3.0, 12.0])
            if not args.skip_large and only in (None, "whisper_large_v2"):
                whisper_golden(ref_h, manifest, C.WHISPER_LARGE_V2_DEC, "whisper_large_v2", 1, 11, [3.0])
        finally:
            os.chdir(cwd)
    old = {}
    mp = os.path.join(HERE, "manifest.json")
    if os.path.exists(mp):
        old = json.load(open(mp))
    old.update(manifest)
    with open(mp, "w") as f:
        json.dump(old, f, indent=1, sort_keys=True)
    print(json.dumps(manifest, indent=1))


if __name__ == "__main__":
    main()
