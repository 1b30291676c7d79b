"""ORACLE (test infrastructure only): numpy restatement of the Whisper embedding path.

Follows:
  WhisperFeatureExtractor.__call__ pad/truncate   HF/models/whisper/feature_extraction_whisper.py:300-307
  _torch_extract_fbank_features                   HF/models/whisper/feature_extraction_whisper.py:135-168
  mel_filter_bank (slaney scale + slaney norm)    HF/audio_utils.py:448-538, 541-560, 638-740
  WhisperEncoder.forward                          HF/models/whisper/modeling_whisper.py:592-646
  WhisperEncoderLayer / WhisperAttention          HF/models/whisper/modeling_whisper.py:215-413
  output capture (hs[-1] = post-LN)               HF/utils/output_capturing.py:105-117, 268-279
  encoder pooling                                 REF/whisper_embeddings_large.py:264-281
  1-token decoder pass (input id 0, position 0)   REF/whisper_embeddings_large.py:257-262,
                                                  HF/models/whisper/modeling_whisper.py:448-506, 689-790
  decoder "pooling" (squeeze the single token)    REF/whisper_embeddings_large.py:283-297
"""
from __future__ import annotations

import math

import numpy as np

from .wavlm import gelu, layer_norm

N_FFT, HOP, N_SAMPLES = 400, 160, 480000


def _hz_to_mel_slaney(f):
    f = np.asarray(f, dtype=np.float64)
    mels = 3.0 * f / 200.0
    logstep = 27.0 / np.log(6.4)
    return np.where(f >= 1000.0, 15.0 + np.log(np.maximum(f, 1e-12) / 1000.0) * logstep, mels)


def _mel_to_hz_slaney(m):
    m = np.asarray(m, dtype=np.float64)
    f = 200.0 * m / 3.0
    logstep = np.log(6.4) / 27.0
    return np.where(m >= 15.0, 1000.0 * np.exp(logstep * (m - 15.0)), f)


def mel_filters(n_mels: int = 80, n_freq: int = N_FFT // 2 + 1, sr: int = 16000) -> np.ndarray:
    """[n_freq, n_mels] float64 (HF mel_filter_bank(..., norm="slaney", mel_scale="slaney"))."""
    mel_freqs = np.linspace(_hz_to_mel_slaney(0.0), _hz_to_mel_slaney(8000.0), n_mels + 2)
    ff = _mel_to_hz_slaney(mel_freqs)
    fft_freqs = np.linspace(0, sr // 2, n_freq)
    diff = np.diff(ff)
    slopes = ff[None, :] - fft_freqs[:, None]
    down = -slopes[:, :-2] / diff[:-1]
    up = slopes[:, 2:] / diff[1:]
    fb = np.maximum(0.0, np.minimum(down, up))
    return fb * (2.0 / (ff[2:n_mels + 2] - ff[:n_mels]))[None, :]


def pad_or_trim(wave: np.ndarray, n: int = N_SAMPLES) -> np.ndarray:
    w = np.zeros(n, dtype=np.float32)
    m = min(n, wave.shape[-1])
    w[:m] = wave[:m]
    return w


def log_mel(wave: np.ndarray, n_mels: int = 80) -> np.ndarray:
    """One clip -> [n_mels, 3000] float32 (HF :135-168, torch.stft center=True reflect, periodic Hann)."""
    x = pad_or_trim(wave).astype(np.float64)
    xp = np.pad(x, (N_FFT // 2, N_FFT // 2), mode="reflect")
    n_frames = 1 + (xp.shape[0] - N_FFT) // HOP                      # 3001
    fr = np.lib.stride_tricks.as_strided(xp, shape=(n_frames, N_FFT), strides=(HOP * 8, 8))
    win = 0.5 - 0.5 * np.cos(2.0 * math.pi * np.arange(N_FFT) / N_FFT)
    spec = np.fft.rfft(fr * win, axis=-1)[:-1]                         # drop last frame -> [3000, 201]
    power = (spec.real ** 2 + spec.imag ** 2)
    mel = power @ mel_filters(n_mels).astype(np.float32).astype(np.float64)   # filters cast to fp32 (HF :157)
    lg = np.log10(np.maximum(mel, 1e-10))
    lg = np.maximum(lg, lg.max() - 8.0)
    return ((lg + 4.0) / 4.0).T.astype(np.float32)


class WhisperOracle:
    def __init__(self, spec, sd: dict, dtype=np.float32):
        self.spec, self.dt = spec, dtype
        self.p = {k: np.asarray(v, dtype=dtype) for k, v in sd.items()}

    def _conv(self, x, w, b, stride):
        """Conv1d k=3 pad=1 on channels-last x [T, C]; w [out, in, 3]."""
        T, C = x.shape
        xp = np.zeros((T + 2, C), dtype=self.dt)
        xp[1:T + 1] = x
        t_out = (T + 2 - 3) // stride + 1
        cols = np.ascontiguousarray(np.lib.stride_tricks.as_strided(
            np.ascontiguousarray(xp), shape=(t_out, 3 * C), strides=(stride * C * xp.itemsize, xp.itemsize)))
        wk = np.ascontiguousarray(w.transpose(2, 1, 0).reshape(3 * C, -1))
        return (cols @ wk + b).astype(self.dt)

    def attention(self, x, l):
        s, p = self.spec, self.p
        q_ = f"encoder.layers.{l}.self_attn"
        T, D = x.shape
        nh, hd = s.heads, s.head_dim
        q = (x @ p[f"{q_}.q_proj.weight"].T + p[f"{q_}.q_proj.bias"]) * np.asarray(hd ** -0.5, self.dt)
        k = x @ p[f"{q_}.k_proj.weight"].T
        v = x @ p[f"{q_}.v_proj.weight"].T + p[f"{q_}.v_proj.bias"]
        qh, kh, vh = (a.reshape(T, nh, hd).transpose(1, 0, 2) for a in (q, k, v))
        sc = qh @ kh.transpose(0, 2, 1)
        sc = sc - sc.max(-1, keepdims=True)
        e = np.exp(sc)
        pr = e / e.sum(-1, keepdims=True)
        ctx = (pr @ vh).transpose(1, 0, 2).reshape(T, D).astype(self.dt)
        return (ctx @ p[f"{q_}.out_proj.weight"].T + p[f"{q_}.out_proj.bias"]).astype(self.dt)

    def hidden_states(self, mel):
        """mel [n_mels, 3000] -> layers+1 hidden states [1500, D]; last one post final LN."""
        s, p, eps = self.spec, self.p, self.spec.ln_eps
        x = mel.T.astype(self.dt)
        x = gelu(self._conv(x, p["encoder.conv1.weight"], p["encoder.conv1.bias"], 1))
        x = gelu(self._conv(x, p["encoder.conv2.weight"], p["encoder.conv2.bias"], 2))
        x = (x + p["encoder.embed_positions.weight"][: x.shape[0]]).astype(self.dt)
        hs = [x]
        for l in range(s.layers):
            q_ = f"encoder.layers.{l}"
            h = layer_norm(x, p[f"{q_}.self_attn_layer_norm.weight"], p[f"{q_}.self_attn_layer_norm.bias"], eps)
            x = (x + self.attention(h, l)).astype(self.dt)
            h = layer_norm(x, p[f"{q_}.final_layer_norm.weight"], p[f"{q_}.final_layer_norm.bias"], eps)
            h = gelu((h @ p[f"{q_}.fc1.weight"].T + p[f"{q_}.fc1.bias"]).astype(self.dt))
            x = (x + h @ p[f"{q_}.fc2.weight"].T + p[f"{q_}.fc2.bias"]).astype(self.dt)
            hs.append(x)
        hs[-1] = layer_norm(x, p["encoder.layer_norm.weight"], p["encoder.layer_norm.bias"], eps)
        return hs

    def _row0(self, key):
        p = self.p
        return p[key + "[0]"] if key + "[0]" in p else p[key][0]

    def decoder_hidden_states(self, enc):
        """enc [1500, D] (encoder last_hidden_state) -> decoder_layers+1 states [D] for input id 0.

        Self-attention of one query over its own single key: softmax == 1 exactly, so the block
        is out_proj(v_proj(LN(x))) (q_proj / k_proj do not influence the result)."""
        s, p, eps = self.spec, self.p, self.spec.ln_eps
        nh, hd = s.heads, s.head_dim
        x = (self._row0("decoder.embed_tokens.weight") + self._row0("decoder.embed_positions.weight")).astype(self.dt)
        hs = [x]
        for l in range(s.decoder_layers):
            q_ = f"decoder.layers.{l}"
            h = layer_norm(x[None], p[f"{q_}.self_attn_layer_norm.weight"], p[f"{q_}.self_attn_layer_norm.bias"], eps)[0]
            v = h @ p[f"{q_}.self_attn.v_proj.weight"].T + p[f"{q_}.self_attn.v_proj.bias"]
            x = (x + v @ p[f"{q_}.self_attn.out_proj.weight"].T + p[f"{q_}.self_attn.out_proj.bias"]).astype(self.dt)
            a = f"{q_}.encoder_attn"
            h = layer_norm(x[None], p[f"{q_}.encoder_attn_layer_norm.weight"],
                           p[f"{q_}.encoder_attn_layer_norm.bias"], eps)[0]
            q = (h @ p[f"{a}.q_proj.weight"].T + p[f"{a}.q_proj.bias"]) * np.asarray(hd ** -0.5, self.dt)
            k = enc @ p[f"{a}.k_proj.weight"].T
            v = enc @ p[f"{a}.v_proj.weight"].T + p[f"{a}.v_proj.bias"]
            qh = q.reshape(nh, hd)
            kh = k.reshape(-1, nh, hd).transpose(1, 0, 2)
            vh = v.reshape(-1, nh, hd).transpose(1, 0, 2)
            sc = np.einsum("hd,htd->ht", qh, kh)
            sc = sc - sc.max(-1, keepdims=True)
            e = np.exp(sc)
            pr = e / e.sum(-1, keepdims=True)
            ctx = np.einsum("ht,htd->hd", pr, vh).reshape(-1).astype(self.dt)
            x = (x + ctx @ p[f"{a}.out_proj.weight"].T + p[f"{a}.out_proj.bias"]).astype(self.dt)
            h = layer_norm(x[None], p[f"{q_}.final_layer_norm.weight"], p[f"{q_}.final_layer_norm.bias"], eps)[0]
            h = gelu((h @ p[f"{q_}.fc1.weight"].T + p[f"{q_}.fc1.bias"]).astype(self.dt))
            x = (x + h @ p[f"{q_}.fc2.weight"].T + p[f"{q_}.fc2.bias"]).astype(self.dt)
            hs.append(x)
        hs[-1] = layer_norm(x[None], p["decoder.layer_norm.weight"], p["decoder.layer_norm.bias"], eps)[0]
        return hs

    def embed_both(self, waves, enc_indices, dec_indices):
        """extract_whisper_embeddings_fixed restated: (enc [B][n_enc][D], dec [B][n_dec][D])."""
        waves = np.atleast_2d(waves)
        D = self.spec.d_model
        enc = np.zeros((waves.shape[0], len(enc_indices), D), dtype=np.float32)
        dec = np.zeros((waves.shape[0], len(dec_indices), D), dtype=np.float32)
        for b in range(waves.shape[0]):
            hs = self.hidden_states(log_mel(waves[b], self.spec.n_mels))
            for j, idx in enumerate(enc_indices):
                enc[b, j] = hs[idx].mean(axis=0)
            ds = self.decoder_hidden_states(hs[-1])
            for j, idx in enumerate(dec_indices):
                dec[b, j] = ds[idx]
        return enc, dec

    def embed(self, waves, layer_indices):
        waves = np.atleast_2d(waves)
        out = np.zeros((waves.shape[0], len(layer_indices), self.spec.d_model), dtype=np.float32)
        for b in range(waves.shape[0]):
            hs = self.hidden_states(log_mel(waves[b], self.spec.n_mels))
            for j, idx in enumerate(layer_indices):
                out[b, j] = hs[idx].mean(axis=0)
        return out
