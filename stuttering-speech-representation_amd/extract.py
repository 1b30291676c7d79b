"""Drop-in replacements for the reference's embedding glue.

Same names, arguments, return values and error behaviour as:
  extract_wavlm_embeddings              REF/WavLM_embeddings.py:267-341
  extract_whisper_embeddings_fixed      REF/whisper_embeddings_large.py:234-299
  extract_embeddings_from_audio_wavlm   REF/model_training_1.py:235-266   (in-memory twin)
  extract_embeddings_from_audio_whisper REF/model_training_1.py:268-316   (in-memory twin)
  load_audio                            REF/WavLM_embeddings.py:87-125
Return ``{"layer_<i>": float32[H]}`` (or ``encoder_layer_<i>``); ``None`` plus a log line on
any error, never raise; OOM is recognised by exception type (``torch.OutOfMemoryError`` /
``SSEOutOfMemoryError``), not by the "CUDA out of memory" string the reference matches.

When ``model`` is one of this package's objects (hf.WavLMModel / hf.WhisperModel) the
hidden states are never materialised: the fused ``sse_embed`` path pools them on the GPU.
Any other HF-compatible model object takes the reference's generic route.
"""
from __future__ import annotations

import logging
import struct

import numpy as np
import torch

from ._lib import SSEOutOfMemoryError
from .hf import WavLMModel, WhisperModel

logger = logging.getLogger(__name__)


# --------------------------------------------------------------------------------------------
def read_wav(path: str) -> tuple[np.ndarray, int]:
    """Minimal RIFF/WAVE reader (PCM 8/16/24/32-bit, IEEE float 32/64) -> ([channels, n], sr),
    scaled like torchaudio.load (integer PCM divided by 2^(bits-1))."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise ValueError(f"{path}: not a RIFF/WAVE file")
    pos, fmt, pcm = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack("<I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            fmt = struct.unpack("<HHIIHH", body[:16])
            if fmt[0] == 0xFFFE and len(body) >= 26:        # WAVE_FORMAT_EXTENSIBLE: subformat code
                fmt = (struct.unpack("<H", body[24:26])[0],) + fmt[1:]
        elif cid == b"data":
            pcm = body
        pos += 8 + size + (size & 1)
    if fmt is None or pcm is None:
        raise ValueError(f"{path}: missing fmt/data chunk")
    code, ch, sr, _, _, bits = fmt
    if code == 1:
        if bits == 8:
            x = (np.frombuffer(pcm, np.uint8).astype(np.float32) - 128.0) / 128.0
        elif bits == 16:
            x = np.frombuffer(pcm, "<i2").astype(np.float32) / 32768.0
        elif bits == 24:
            b = np.frombuffer(pcm, np.uint8).reshape(-1, 3).astype(np.int32)
            v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
            x = (np.where(v >= 1 << 23, v - (1 << 24), v)).astype(np.float32) / float(1 << 23)
        elif bits == 32:
            x = np.frombuffer(pcm, "<i4").astype(np.float64).astype(np.float32) / float(1 << 31)
        else:
            raise ValueError(f"{path}: {bits}-bit PCM unsupported")
    elif code == 3:
        x = np.frombuffer(pcm, "<f4" if bits == 32 else "<f8").astype(np.float32)
    else:
        raise ValueError(f"{path}: wave format {code} unsupported")
    n = x.size // ch
    return x[:n * ch].reshape(n, ch).T.copy(), sr


def load_audio(file_path, target_sr=16000, max_length=None, device=None):
    """REF/WavLM_embeddings.py:87-125: mono mean, resample, trim; float32[n] or None.
    Mono mixing and resampling run on the GPU (ingest.py); a 16 kHz mono file needs no GPU."""
    try:
        wav, sr = read_wav(file_path)
        if wav.shape[0] > 1 or sr != target_sr:
            from .ingest import to_16k_mono
            wav = to_16k_mono(wav, sr, target_sr, device).cpu().numpy()[None]
        if max_length is not None:
            m = int(max_length * target_sr)
            if wav.shape[1] > m:
                logger.info(f"Trimming audio from {wav.shape[1] / target_sr:.2f}s to {max_length:.2f}s")
                wav = wav[:, :m]
        return wav.squeeze().astype(np.float32)
    except Exception as e:
        logger.error(f"Error loading {file_path}: {e}")
        return None


def _is_oom(e: BaseException) -> bool:
    return isinstance(e, (torch.OutOfMemoryError, SSEOutOfMemoryError))


def _pool_generic(hidden_states, layer_indices, prefix):
    out = {}
    for idx in layer_indices:
        if idx < len(hidden_states):
            out[f"{prefix}{idx}"] = torch.mean(hidden_states[idx], dim=1).cpu().numpy().flatten()
        else:
            logger.warning(f"Layer {idx} is out of range (max: {len(hidden_states) - 1})")
    return out


def extract_embeddings_from_audio_wavlm(audio_array, model, feature_extractor, device, layer_indices):
    """REF/model_training_1.py:235-266 (in-memory twin)."""
    try:
        inputs = feature_extractor(audio_array, sampling_rate=16000, return_tensors="pt").to(device)
        with torch.no_grad():
            if isinstance(model, WavLMModel):
                n_hs = model.sse.spec.layers + 1
                valid = [i for i in layer_indices if i < n_hs]
                for i in layer_indices:
                    if i >= n_hs:
                        logger.warning(f"Layer {i} is out of range (max: {n_hs - 1})")
                if not valid:
                    return {}
                emb = model.embed(inputs.input_values, valid).cpu().numpy()
                return {f"layer_{i}": emb[0, j].copy() for j, i in enumerate(valid)}
            outputs = model(inputs.input_values, output_hidden_states=True, return_dict=True)
            return _pool_generic(outputs.hidden_states, layer_indices, "layer_")
    except Exception as e:
        if _is_oom(e):
            logger.error("HIP out of memory while extracting WavLM embeddings")
            torch.cuda.empty_cache()
        else:
            logger.error(f"Error extracting WavLM embeddings: {e}")
        return None


def extract_wavlm_embeddings(audio_file, model, feature_extractor, device, layer_indices, max_length=None,
                             sample_rate=16000):
    """REF/WavLM_embeddings.py:267-341."""
    audio = load_audio(audio_file, target_sr=sample_rate, max_length=max_length, device=device)
    if audio is None:
        return None
    if audio.shape[-1] > 500000:
        logger.warning(f"Very long input ({audio.shape[-1]} samples, ~{audio.shape[-1] / sample_rate:.2f}s). "
                       "This may cause memory issues.")
    out = extract_embeddings_from_audio_wavlm(audio, model, feature_extractor, device, layer_indices)
    if out is None:
        logger.error(f"Error extracting embeddings for {audio_file}")
    return out


def extract_embeddings_from_audio_whisper(audio_array, model, processor, device, layer_names):
    """REF/model_training_1.py:268-316 (in-memory twin): ``encoder_layer_<i>`` time-means and
    ``decoder_layer_<i>`` states of the 1-token decoder pass, in ``layer_names`` order.  A model
    built without the decoder (decoder_layers=0) reports and skips decoder names."""
    try:
        wanted = []
        for n in layer_names:
            if n.startswith("encoder_layer_") or n.startswith("decoder_layer_"):
                wanted.append((n.startswith("decoder_"), int(n.split("_")[-1]), n))
        with torch.no_grad():
            if isinstance(model, WhisperModel):
                spec = model.sse.spec
                if any(d for d, _, _ in wanted) and not spec.decoder_layers:
                    logger.warning(f"{spec.name} was built without the decoder; decoder_layer_* skipped")
                    wanted = [w for w in wanted if not w[0]]
                enc = [i for d, i, _ in wanted if not d and i < spec.layers + 1]
                dec = [i for d, i, _ in wanted if d and i < spec.decoder_layers + 1]
                if not enc and not dec:
                    return {}
                wave = torch.from_numpy(np.ascontiguousarray(np.asarray(audio_array, np.float32)))
                e, dd = model.sse.whisper_embed(wave.to(model.sse.device), enc, dec)
                e, dd = e.cpu().numpy(), dd.cpu().numpy()
                out = {}
                for d, i, n in wanted:
                    if d and i in dec:
                        out[n] = dd[0, dec.index(i)].copy()
                    elif not d and i in enc:
                        out[n] = e[0, enc.index(i)].copy()
                return out
            feats = processor(audio_array, sampling_rate=16000, return_tensors="pt").input_features.to(device)
            eo = model.encoder(feats, output_hidden_states=True, return_dict=True)
            do = None
            if any(d for d, _, _ in wanted):
                do = model.decoder(input_ids=torch.zeros((1, 1), dtype=torch.long).to(device),
                                   encoder_hidden_states=eo.last_hidden_state, output_hidden_states=True,
                                   return_dict=True)
            out = {}
            for d, i, n in wanted:
                states = do.hidden_states if d else eo.hidden_states
                if i < len(states):
                    h = states[i]
                    out[n] = (h.squeeze(1) if d else torch.mean(h, dim=1)).cpu().numpy().flatten()
            return out
    except Exception as e:
        if _is_oom(e):
            logger.error("HIP out of memory while extracting Whisper embeddings")
            torch.cuda.empty_cache()
        else:
            logger.error(f"Error extracting Whisper embeddings: {e}")
        return None


def extract_whisper_embeddings_fixed(audio_file, model, processor, device, encoder_indices, decoder_indices):
    """REF/whisper_embeddings_large.py:234-299: encoder time-means + 1-token decoder states."""
    audio = load_audio(audio_file, device=device)
    if audio is None:
        return None
    if isinstance(model, WhisperModel):
        for i in encoder_indices:
            if i >= model.sse.spec.layers + 1:
                logger.warning(f"Encoder layer {i} is out of range (max: {model.sse.spec.layers})")
        for i in decoder_indices:
            if model.sse.spec.decoder_layers and i >= model.sse.spec.decoder_layers + 1:
                logger.warning(f"Decoder layer {i} is out of range (max: {model.sse.spec.decoder_layers})")
    names = [f"encoder_layer_{i}" for i in encoder_indices] + [f"decoder_layer_{i}" for i in decoder_indices]
    return extract_embeddings_from_audio_whisper(audio, model, processor, device, names)
