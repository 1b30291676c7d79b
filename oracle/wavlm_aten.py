"""ORACLE (test infrastructure only): the reference's CPU path restated on the SAME ATen ops.

``bench.py``'s ``cpu_baseline`` leg times this on the GPU box's host cores, because the reference
itself (``REF/WavLM_embeddings.py``) cannot travel there.  It is the reference's call sequence —
one clip at a time (batch 1, ``REF/WavLM_embeddings.py:578-586``), fp32, ``torch.no_grad`` — issued
as the same torch functional calls the third-party HF ``WavLMModel`` makes (transformers 5.15.0),
so the CPU time is spent in the same kernels (mkldnn conv1d, BLAS addmm, ``native_group_norm``,
``native_layer_norm``, erf-GELU, ``_weight_norm_interface`` recomputed every forward,
``multi_head_attention_forward`` with the gated bias as ``attn_mask``):

  Wav2Vec2FeatureExtractor cast / norm  HF/models/wav2vec2/feature_extraction_wav2vec2.py:78-97, 214-229
  WavLMGroupNormConvLayer / NoLayerNorm HF/models/wavlm/modeling_wavlm.py:675-693, 723-744
  WavLMLayerNormConvLayer (large)       HF/models/wavlm/modeling_wavlm.py:696-720
  WavLMFeatureProjection                HF/models/wavlm/modeling_wavlm.py:93-105
  WavLMPositionalConvEmbedding+SamePad  HF/models/wavlm/modeling_wavlm.py:37-90
  WavLMEncoder(.StableLayerNorm)        HF/models/wavlm/modeling_wavlm.py:388-447, 465-522
  WavLMAttention.forward / compute_bias HF/models/wavlm/modeling_wavlm.py:146-271
  WavLMEncoderLayer(.StableLayerNorm)   HF/models/wavlm/modeling_wavlm.py:314-373
  extract_wavlm_embeddings pooling      REF/WavLM_embeddings.py:289-323

Calibration against the reference itself (same container, same clips, same thread count):
``oracle/calibrate_cpu_baseline.py`` -> ``profiles/r2_cpu_baseline_calibration.json``.
Parity: ``tests/test_oracle_golden.py::test_aten_restatement_matches_reference`` (<= 1e-5 vs the
reference's own fixture).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F


def _rel_buckets(T: int, num_buckets: int, max_distance: int) -> torch.Tensor:
    """WavLMAttention._relative_positions_bucket on relative_position = j - i
    (HF/models/wavlm/modeling_wavlm.py:246-271), int64 with the float32 log path."""
    rel = torch.arange(T, dtype=torch.long)[None, :] - torch.arange(T, dtype=torch.long)[:, None]
    nb = num_buckets // 2
    out = (rel > 0).to(torch.long) * nb
    rel = torch.abs(rel)
    max_exact = nb // 2
    large = torch.log(rel.float() / max_exact) / math.log(max_distance / max_exact) * (nb - max_exact)
    large = torch.clamp_max((max_exact + large).to(torch.long), nb - 1)
    return out + torch.where(rel < max_exact, rel, large)


class WavLMAten:
    """Functional WavLM forward on CPU torch fp32, one clip per call (the reference's loop)."""

    def __init__(self, spec, sd: dict):
        self.spec = spec
        self.w = {k: (v if isinstance(v, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(v))).float()
                  for k, v in sd.items()}

    def _conv_frontend(self, x: torch.Tensor) -> torch.Tensor:
        s, w = self.spec, self.w
        h = x[:, None]                                                     # [1, 1, L]
        for i in range(len(s.conv_dim)):
            p = f"feature_extractor.conv_layers.{i}."
            h = F.conv1d(h, w[p + "conv.weight"], w.get(p + "conv.bias"), stride=s.conv_stride[i])
            if s.feat_norm_layer:                                          # :696-720
                h = F.layer_norm(h.transpose(-2, -1), (h.shape[1],), w[p + "layer_norm.weight"],
                                 w[p + "layer_norm.bias"], 1e-5).transpose(-2, -1)
            elif i == 0:                                                   # :723-744
                h = F.group_norm(h, h.shape[1], w[p + "layer_norm.weight"], w[p + "layer_norm.bias"], 1e-5)
            h = F.gelu(h)
        return h.transpose(1, 2)                                           # [1, T, C]

    def hidden_states(self, wave: torch.Tensor, do_normalize: bool = False) -> list[torch.Tensor]:
        s, w, eps = self.spec, self.w, self.spec.ln_eps
        x = wave.float()[None]
        if do_normalize:                                                   # zero_mean_unit_var_norm
            x = (x - x.mean()) / torch.sqrt(x.var(unbiased=False) + 1e-7)
        f = self._conv_frontend(x)
        f = F.layer_norm(f, (f.shape[-1],), w["feature_projection.layer_norm.weight"],
                         w["feature_projection.layer_norm.bias"], eps)
        h = F.linear(f, w["feature_projection.projection.weight"], w["feature_projection.projection.bias"])
        # positional conv: weight norm recomputed every forward (parametrization), SamePad, GELU
        pc = "encoder.pos_conv_embed.conv."
        pw = torch._weight_norm(w[pc + "parametrizations.weight.original1"], w[pc + "parametrizations.weight.original0"], 2)
        pos = F.conv1d(h.transpose(1, 2), pw, w[pc + "bias"], padding=s.pos_kernel // 2, groups=s.pos_groups)
        if s.pos_kernel % 2 == 0:
            pos = pos[:, :, :-1]
        h = h + F.gelu(pos).transpose(1, 2)
        if not s.stable_layer_norm:
            h = F.layer_norm(h, (s.hidden,), w["encoder.layer_norm.weight"], w["encoder.layer_norm.bias"], eps)
        T, nh = h.shape[1], s.heads
        a0 = "encoder.layers.0.attention."
        bias = w[a0 + "rel_attn_embed.weight"][_rel_buckets(T, s.num_buckets, s.max_distance)].permute(2, 0, 1)
        out = []
        for l in range(s.layers):
            out.append(h)
            p = f"encoder.layers.{l}."
            a = p + "attention."
            res = h
            if s.stable_layer_norm:
                h = F.layer_norm(h, (s.hidden,), w[p + "layer_norm.weight"], w[p + "layer_norm.bias"], eps)
            # gate from the per-head split of the attention input (:163-176)
            g = F.linear(h.view(1, T, nh, -1).permute(0, 2, 1, 3), w[a + "gru_rel_pos_linear.weight"],
                         w[a + "gru_rel_pos_linear.bias"]).view(1, nh, T, 2, 4).sum(-1)
            ga, gb = torch.sigmoid(g).chunk(2, dim=-1)
            gate = ga * (gb * w[a + "gru_rel_pos_const"].view(1, nh, 1, 1) - 1.0) + 2.0
            gated = (gate.view(nh, -1, 1) * bias).view(-1, T, T)
            q = h.transpose(0, 1)
            att, _ = F.multi_head_attention_forward(
                q, q, q, s.hidden, nh, torch.empty([0]),
                torch.cat((w[a + "q_proj.bias"], w[a + "k_proj.bias"], w[a + "v_proj.bias"])), None, None, False,
                0.0, w[a + "out_proj.weight"], w[a + "out_proj.bias"], False, None, False, gated,
                use_separate_proj_weight=True, q_proj_weight=w[a + "q_proj.weight"],
                k_proj_weight=w[a + "k_proj.weight"], v_proj_weight=w[a + "v_proj.weight"])
            h = res + att.transpose(0, 1)
            ff = p + "feed_forward."
            if s.stable_layer_norm:
                z = F.layer_norm(h, (s.hidden,), w[p + "final_layer_norm.weight"], w[p + "final_layer_norm.bias"], eps)
                h = h + F.linear(F.gelu(F.linear(z, w[ff + "intermediate_dense.weight"], w[ff + "intermediate_dense.bias"])),
                                 w[ff + "output_dense.weight"], w[ff + "output_dense.bias"])
            else:
                h = F.layer_norm(h, (s.hidden,), w[p + "layer_norm.weight"], w[p + "layer_norm.bias"], eps)
                h = h + F.linear(F.gelu(F.linear(h, w[ff + "intermediate_dense.weight"], w[ff + "intermediate_dense.bias"])),
                                 w[ff + "output_dense.weight"], w[ff + "output_dense.bias"])
                h = F.layer_norm(h, (s.hidden,), w[p + "final_layer_norm.weight"], w[p + "final_layer_norm.bias"], eps)
        if s.stable_layer_norm:
            h = F.layer_norm(h, (s.hidden,), w["encoder.layer_norm.weight"], w["encoder.layer_norm.bias"], eps)
        out.append(h)
        return out

    @torch.no_grad()
    def extract(self, wave: np.ndarray, layer_indices, do_normalize: bool = False) -> dict:
        """One clip -> {"layer_<i>": float32[H]} like extract_wavlm_embeddings (REF :313-323)."""
        hs = self.hidden_states(torch.from_numpy(np.asarray(wave, dtype=np.float32)), do_normalize)
        return {f"layer_{i}": torch.mean(hs[i], dim=1).cpu().numpy().flatten() for i in layer_indices
                if i < len(hs)}

    def embed(self, waves: np.ndarray, layer_indices, do_normalize: bool = False) -> np.ndarray:
        """[N, L] clips in a batch-1 loop -> [N, n_layers, H] float32."""
        rows = []
        for c in waves:
            d = self.extract(c, layer_indices, do_normalize)
            rows.append(np.stack([d[f"layer_{i}"] for i in layer_indices]))
        return np.stack(rows).astype(np.float32)
