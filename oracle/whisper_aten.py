"""ORACLE (test infrastructure only): the reference's Whisper CPU path restated on the SAME ATen ops.

``bench.py --model whisper-large-v2``'s ``cpu_baseline`` leg times this on the GPU box's host cores,
because the reference itself (``REF/whisper_embeddings_large.py``) cannot travel there.  It is the
reference's call sequence for one clip (batch 1, fp32, ``torch.no_grad``,
``REF/whisper_embeddings_large.py:234-299``) issued as the same torch calls the third-party HF
objects make (transformers 5.15.0), so the CPU time is spent in the same kernels:

  WhisperFeatureExtractor pad / truncate         HF/models/whisper/feature_extraction_whisper.py:300-307
  _torch_extract_fbank_features (torch.stft,     HF/models/whisper/feature_extraction_whisper.py:135-168
    |.|^2, mel_filters.T @ P, log10, max-8)
  WhisperEncoder.forward (conv1/conv2 + GELU,    HF/models/whisper/modeling_whisper.py:592-646
    + embed_positions, 32 layers, final LN)
  WhisperEncoderLayer / WhisperAttention         HF/models/whisper/modeling_whisper.py:284-413
    (q scaled before the product, k_proj without bias, SDPA with scale 1 -- the default
    attention implementation of a WhisperModel built in this transformers)
  WhisperDecoder.forward, 1 token (id 0, pos 0)  HF/models/whisper/modeling_whisper.py:690-795, 416-505
    (self-attention over the single token incl. its q / k projections, cross-attention whose
    K / V projections of the 1500 encoder frames dominate, FFN, final LN)
  hidden-state capture (last = post-LN)          HF/utils/output_capturing.py:105-117, 268-279
  encoder time-mean / decoder squeeze            REF/whisper_embeddings_large.py:264-297

Parity: ``tests/test_oracle_golden.py::test_whisper_aten_restatement_matches_reference`` (<= 1e-5 vs
the reference's own ``whisper_tiny.npz`` fixture, encoder and decoder keys).  Calibration against
the reference itself: ``oracle/calibrate_cpu_baseline.py --model whisper-large-v2``.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .whisper import N_FFT, HOP, N_SAMPLES, mel_filters


class WhisperAten:
    """Functional Whisper forward on CPU torch fp32, one clip per call (the reference's loop)."""

    def __init__(self, spec, sd: dict):
        self.spec = spec
        self.w = {k: (v if isinstance(v, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(v))).float()
                  for k, v in sd.items()}
        # HF keeps the float64 Slaney filters and casts them per call (:157); cast once here
        self.mel = torch.from_numpy(mel_filters(spec.n_mels)).to(torch.float32)
        self.window = torch.hann_window(N_FFT)

    def _row0(self, key: str) -> torch.Tensor:
        return self.w[key + "[0]"] if key + "[0]" in self.w else self.w[key][0]

    def log_mel(self, wave: np.ndarray) -> torch.Tensor:
        """[L] -> [1, n_mels, 3000] (HF pad / truncate to 30 s, then the torch fbank path)."""
        x = np.zeros(N_SAMPLES, np.float32)
        m = min(N_SAMPLES, wave.shape[-1])
        x[:m] = wave[:m]
        wav = torch.from_numpy(x)
        stft = torch.stft(wav, N_FFT, HOP, window=self.window, return_complex=True)
        mag = (stft[..., :-1].abs() ** 2).contiguous()
        spec = self.mel.T @ mag
        lg = torch.clamp(spec, min=1e-10).log10()
        lg = torch.maximum(lg, lg.max() - 8.0)
        return ((lg + 4.0) / 4.0)[None]

    def _attn(self, x: torch.Tensor, kv: torch.Tensor, p: str) -> torch.Tensor:
        """WhisperAttention.forward (:284-356): q scaled by d^-1/2 before the product, k unbiased."""
        w, nh = self.w, self.spec.heads
        B, T, D = x.shape
        hd = D // nh
        q = (F.linear(x, w[p + "q_proj.weight"], w[p + "q_proj.bias"]) * (hd ** -0.5)).view(B, T, nh, hd).transpose(1, 2)
        k = F.linear(kv, w[p + "k_proj.weight"]).view(B, -1, nh, hd).transpose(1, 2)
        v = F.linear(kv, w[p + "v_proj.weight"], w[p + "v_proj.bias"]).view(B, -1, nh, hd).transpose(1, 2)
        o = F.scaled_dot_product_attention(q.contiguous(), k.contiguous(), v.contiguous(), scale=1.0)
        return F.linear(o.transpose(1, 2).reshape(B, T, D), w[p + "out_proj.weight"], w[p + "out_proj.bias"])

    def encoder_hidden_states(self, mel: torch.Tensor) -> list[torch.Tensor]:
        s, w, eps = self.spec, self.w, self.spec.ln_eps
        h = F.gelu(F.conv1d(mel, w["encoder.conv1.weight"], w["encoder.conv1.bias"], padding=1))
        h = F.gelu(F.conv1d(h, w["encoder.conv2.weight"], w["encoder.conv2.bias"], stride=2, padding=1))
        h = h.permute(0, 2, 1) + w["encoder.embed_positions.weight"][: h.shape[-1]]
        hs = []
        D = s.d_model
        for l in range(s.layers):
            hs.append(h)
            p = f"encoder.layers.{l}."
            z = F.layer_norm(h, (D,), w[p + "self_attn_layer_norm.weight"], w[p + "self_attn_layer_norm.bias"], eps)
            h = h + self._attn(z, z, p + "self_attn.")
            z = F.layer_norm(h, (D,), w[p + "final_layer_norm.weight"], w[p + "final_layer_norm.bias"], eps)
            h = h + F.linear(F.gelu(F.linear(z, w[p + "fc1.weight"], w[p + "fc1.bias"])), w[p + "fc2.weight"],
                             w[p + "fc2.bias"])
        hs.append(F.layer_norm(h, (D,), w["encoder.layer_norm.weight"], w["encoder.layer_norm.bias"], eps))
        return hs

    def decoder_hidden_states(self, enc: torch.Tensor) -> list[torch.Tensor]:
        """input_ids = zeros((1, 1)) (REF :257-262): token 0 at position 0."""
        s, w, eps = self.spec, self.w, self.spec.ln_eps
        D = s.d_model
        h = (self._row0("decoder.embed_tokens.weight") + self._row0("decoder.embed_positions.weight")).view(1, 1, D)
        hs = []
        for l in range(s.decoder_layers):
            hs.append(h)
            p = f"decoder.layers.{l}."
            z = F.layer_norm(h, (D,), w[p + "self_attn_layer_norm.weight"], w[p + "self_attn_layer_norm.bias"], eps)
            h = h + self._attn(z, z, p + "self_attn.")
            z = F.layer_norm(h, (D,), w[p + "encoder_attn_layer_norm.weight"], w[p + "encoder_attn_layer_norm.bias"],
                             eps)
            h = h + self._attn(z, enc, p + "encoder_attn.")
            z = F.layer_norm(h, (D,), w[p + "final_layer_norm.weight"], w[p + "final_layer_norm.bias"], eps)
            h = h + F.linear(F.gelu(F.linear(z, w[p + "fc1.weight"], w[p + "fc1.bias"])), w[p + "fc2.weight"],
                             w[p + "fc2.bias"])
        hs.append(F.layer_norm(h, (D,), w["decoder.layer_norm.weight"], w["decoder.layer_norm.bias"], eps))
        return hs

    @torch.no_grad()
    def extract(self, wave: np.ndarray, encoder_indices, decoder_indices=()) -> dict:
        """One clip -> {"encoder_layer_<i>": float32[D], "decoder_layer_<i>": float32[D]} like
        extract_whisper_embeddings_fixed (REF :234-299)."""
        enc = self.encoder_hidden_states(self.log_mel(np.asarray(wave, dtype=np.float32)))
        out = {f"encoder_layer_{i}": torch.mean(enc[i], dim=1).numpy().flatten() for i in encoder_indices
               if i < len(enc)}
        if decoder_indices:
            dec = self.decoder_hidden_states(enc[-1])
            out.update({f"decoder_layer_{i}": dec[i].squeeze(1).numpy().flatten() for i in decoder_indices
                        if i < len(dec)})
        return out
