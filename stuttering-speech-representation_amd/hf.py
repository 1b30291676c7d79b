"""HF-duck-typed objects over the HIP path (the reference's operator API).

The reference's glue only touches a narrow surface of the HF objects it is handed:
  model(input_values, output_hidden_states=True, return_dict=True).hidden_states / .last_hidden_state
                                               REF/WavLM_embeddings.py:76, 257, 302-310
  model.config.hidden_size, next(model.parameters()).device     REF/WavLM_embeddings.py:66, 83
  model.encoder(input_features, output_hidden_states=True, return_dict=True)
                                               REF/whisper_embeddings_large.py:64, 250-254
  feature_extractor(audio, sampling_rate=16000, return_tensors="pt").to(device).input_values
                                               REF/WavLM_embeddings.py:289-293
  processor(audio, sampling_rate=16000, return_tensors="pt").input_features
                                               REF/whisper_embeddings_large.py:242-246
These classes provide exactly that surface, so the reference's own functions (and
model_training_*.py) run unchanged on them, with every tensor op in libsse.so on the GPU.
  model.decoder(input_ids=zeros((1, 1)), encoder_hidden_states=..., output_hidden_states=True)
                                               REF/whisper_embeddings_large.py:257-262
The decoder twin supports exactly that call (one token, id 0, position 0); other ids raise.
"""
from __future__ import annotations

from dataclasses import dataclass
from types import SimpleNamespace

import numpy as np
import torch

from . import config as C
from .model import SSEModel, logmel, normalize


@dataclass
class BaseModelOutput:
    last_hidden_state: torch.Tensor
    hidden_states: tuple | None = None
    attentions: tuple | None = None

    def __getitem__(self, i):
        return (self.last_hidden_state, self.hidden_states)[i]


class BatchFeature(dict):
    """Minimal transformers.BatchFeature: attribute access + .to(device)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def to(self, device):
        return BatchFeature({k: (v.to(device) if isinstance(v, torch.Tensor) else v) for k, v in self.items()})


def _to_batch(raw, device) -> torch.Tensor:
    if isinstance(raw, (list, tuple)) and raw and not np.isscalar(raw[0]):
        arrs = [np.asarray(r, dtype=np.float32) for r in raw]
        if len({a.shape[-1] for a in arrs}) != 1:
            raise ValueError("ragged batches are not supported: pass one clip or equal lengths")
        raw = np.stack(arrs)
    if isinstance(raw, torch.Tensor):
        t = raw.to(torch.float32)
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(raw, dtype=np.float32)))
    if t.dim() == 1:
        t = t[None]
    return t.to(device)


class Wav2Vec2FeatureExtractor:
    """Wav2Vec2FeatureExtractor twin (HF feature_extraction_wav2vec2.py:99-236): float32 cast,
    optional zero-mean/unit-variance normalisation on the GPU (sse_normalize)."""

    def __init__(self, do_normalize: bool = False, sampling_rate: int = 16000, device="cuda:0", **_):
        self.do_normalize = do_normalize
        self.sampling_rate = sampling_rate
        self.device = torch.device(device)

    def __call__(self, raw_speech, sampling_rate=None, return_tensors="pt", **_):
        if sampling_rate is not None and sampling_rate != self.sampling_rate:
            raise ValueError(f"expected sampling_rate={self.sampling_rate}, got {sampling_rate}")
        x = _to_batch(raw_speech, self.device)
        if self.do_normalize:
            x = normalize(x)
        return BatchFeature(input_values=x)


class WhisperFeatureExtractor:
    """WhisperFeatureExtractor / WhisperProcessor twin: pad/truncate to 30 s and log-mel on the
    GPU (sse_logmel, HF feature_extraction_whisper.py:135-168, 300-307)."""

    def __init__(self, feature_size: int = 80, sampling_rate: int = 16000, device="cuda:0", **_):
        self.feature_size = feature_size
        self.sampling_rate = sampling_rate
        self.device = torch.device(device)

    def __call__(self, raw_speech, sampling_rate=None, return_tensors="pt", **_):
        if sampling_rate is not None and sampling_rate != self.sampling_rate:
            raise ValueError(f"expected sampling_rate={self.sampling_rate}, got {sampling_rate}")
        return BatchFeature(input_features=logmel(_to_batch(raw_speech, self.device), self.feature_size))


WhisperProcessor = WhisperFeatureExtractor


def _shape_key(spec):
    """A spec with the name dropped and the decoder FFN width made explicit (0 without a decoder)."""
    import dataclasses
    if isinstance(spec, C.WhisperSpec):
        spec = dataclasses.replace(spec, dec_ffn=spec.dec_ffn_dim if spec.decoder_layers else 0)
    return dataclasses.replace(spec, name="")


def _canonical(spec, known):
    """The named spec of ``known`` with the same shape as ``spec`` (else ``spec`` itself)."""
    return next((k for k in known if _shape_key(k) == _shape_key(spec)), spec)


def wavlm_spec_from_config(c) -> C.WavLMSpec:
    """transformers ``WavLMConfig`` -> ``WavLMSpec`` (host only, no GPU): the shape fields the
    reference's hub checkpoints set (HF/models/wavlm/configuration_wavlm.py:159-213), read by
    ``WavLMModel.from_hf`` (REF/WavLM_embeddings.py:482-483 loads the HF model this maps).
    ``WavLMConfig()`` maps to ``C.WAVLM_BASE``, the wavlm-large shape to ``C.WAVLM_LARGE``."""
    if c.feat_extract_norm not in ("group", "layer"):
        raise NotImplementedError(f"feat_extract_norm={c.feat_extract_norm!r}")
    spec = C.WavLMSpec(hidden=c.hidden_size, layers=c.num_hidden_layers, heads=c.num_attention_heads,
                       ffn=c.intermediate_size, conv_dim=tuple(c.conv_dim), conv_kernel=tuple(c.conv_kernel),
                       conv_stride=tuple(c.conv_stride), conv_bias=bool(c.conv_bias),
                       feat_norm_layer=c.feat_extract_norm == "layer",
                       stable_layer_norm=bool(c.do_stable_layer_norm), pos_kernel=c.num_conv_pos_embeddings,
                       pos_groups=c.num_conv_pos_embedding_groups, num_buckets=c.num_buckets,
                       max_distance=c.max_bucket_distance, ln_eps=c.layer_norm_eps,
                       name=getattr(c, "_name_or_path", "") or "wavlm")
    return _canonical(spec, (C.WAVLM_BASE, C.WAVLM_LARGE))


def whisper_spec_from_config(c, with_decoder: bool = True) -> C.WhisperSpec:
    """transformers ``WhisperConfig`` -> ``WhisperSpec`` (host only, no GPU), read by
    ``WhisperModel.from_hf`` (REF/whisper_embeddings_large.py:437-438 loads the HF model this maps).
    The whisper-tiny / -small / -large-v2 shapes map to the named ``C.WHISPER_*`` specs (``*_DEC``
    with the decoder)."""
    if c.decoder_attention_heads != c.encoder_attention_heads:
        raise NotImplementedError("decoder and encoder head counts differ")
    spec = C.WhisperSpec(d_model=c.d_model, layers=c.encoder_layers, heads=c.encoder_attention_heads,
                         ffn=c.encoder_ffn_dim, n_mels=c.num_mel_bins, max_positions=c.max_source_positions,
                         decoder_layers=c.decoder_layers if with_decoder else 0, dec_ffn=c.decoder_ffn_dim,
                         vocab_size=c.vocab_size, max_target_positions=c.max_target_positions,
                         name=getattr(c, "_name_or_path", "") or "whisper")
    known = ((C.WHISPER_TINY_DEC, C.WHISPER_SMALL_DEC, C.WHISPER_LARGE_V2_DEC) if with_decoder
             else (C.WHISPER_TINY, C.WHISPER_SMALL, C.WHISPER_LARGE_V2))
    return _canonical(spec, known)


class _DuckModel:
    def __init__(self, sse: SSEModel):
        self.sse = sse
        self.config = SimpleNamespace(hidden_size=sse.spec.hidden, d_model=sse.spec.hidden,
                                      num_hidden_layers=sse.spec.layers, model_type=sse.spec.name)
        self._p = torch.zeros(1, device=sse.device)

    def parameters(self):
        yield self._p

    @property
    def device(self):
        return self.sse.device

    def to(self, device):
        if torch.device(device) != self.sse.device and not (torch.device(device).type == "cuda"
                                                             and torch.device(device).index is None):
            raise ValueError(f"model lives on {self.sse.device}; build a new one for {device}")
        return self

    def eval(self):
        return self

    def embed(self, wave, layer_indices):
        return self.sse.embed(wave, layer_indices)


class WavLMModel(_DuckModel):
    """WavLMModel twin.  ``WavLMModel.from_hf(hf_model)`` takes the weights of a real
    transformers WavLMModel (e.g. a hub checkpoint loaded elsewhere)."""

    @classmethod
    def from_state_dict(cls, spec, state_dict, device="cuda:0", dtype="fp32"):
        return cls(SSEModel(spec, state_dict, device=device, dtype=dtype))

    @classmethod
    def from_hf(cls, hf_model, device="cuda:0", dtype="fp32"):
        return cls.from_state_dict(wavlm_spec_from_config(hf_model.config), hf_model.state_dict(), device, dtype)

    def __call__(self, input_values, attention_mask=None, output_hidden_states=None, return_dict=True, **_):
        if attention_mask is not None:
            raise NotImplementedError("padded batches (attention_mask) are not supported")
        hs = self.sse.hidden_states(_to_batch(input_values, self.sse.device))
        return BaseModelOutput(last_hidden_state=hs[-1], hidden_states=hs if output_hidden_states else None)

    forward = __call__


class _WhisperEncoder:
    def __init__(self, sse: SSEModel):
        self.sse = sse

    def __call__(self, input_features, attention_mask=None, output_hidden_states=None, return_dict=True, **_):
        hs = self.sse.hidden_states_from_mel(input_features.to(self.sse.device))
        return BaseModelOutput(last_hidden_state=hs[-1], hidden_states=hs if output_hidden_states else None)


class _WhisperDecoder:
    """The reference's decoder call: one start token (id 0) per clip at position 0."""

    def __init__(self, sse: SSEModel):
        self.sse = sse

    def __call__(self, input_ids=None, encoder_hidden_states=None, output_hidden_states=None, return_dict=True,
                 attention_mask=None, past_key_values=None, **_):
        if not self.sse.spec.decoder_layers:
            raise NotImplementedError(f"{self.sse.spec.name} was built without the decoder (decoder_layers=0)")
        if encoder_hidden_states is None or input_ids is None:
            raise ValueError("the decoder twin needs input_ids and encoder_hidden_states")
        if attention_mask is not None or past_key_values is not None:
            raise NotImplementedError("only the 1-token pass of REF/whisper_embeddings_large.py:257-262")
        ids = torch.as_tensor(input_ids)
        if ids.dim() != 2 or ids.shape[1] != 1 or bool((ids != 0).any()):
            raise NotImplementedError("only input_ids == zeros((B, 1)) (the reference's start token) is built")
        enc = encoder_hidden_states.to(self.sse.device)
        if enc.shape[0] != ids.shape[0]:
            raise ValueError(f"batch mismatch: input_ids {tuple(ids.shape)} vs encoder states {tuple(enc.shape)}")
        hs = self.sse.decoder_hidden_states(enc)
        return BaseModelOutput(last_hidden_state=hs[-1], hidden_states=hs if output_hidden_states else None)


class WhisperModel(_DuckModel):
    """WhisperModel twin: ``.encoder`` and the 1-token ``.decoder`` pass run on the HIP path."""

    def __init__(self, sse: SSEModel):
        super().__init__(sse)
        self.encoder = _WhisperEncoder(sse)
        self.decoder = _WhisperDecoder(sse)

    @classmethod
    def from_state_dict(cls, spec, state_dict, device="cuda:0", dtype="fp32"):
        return cls(SSEModel(spec, state_dict, device=device, dtype=dtype))

    @classmethod
    def from_hf(cls, hf_model, device="cuda:0", dtype="fp32", with_decoder=True):
        spec = whisper_spec_from_config(hf_model.config, with_decoder=with_decoder)
        return cls.from_state_dict(spec, hf_model.state_dict(), device, dtype)
