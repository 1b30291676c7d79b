"""ORACLE (test infrastructure only): numpy restatement of the WavLM embedding path.

Follows, in order:
  Wav2Vec2FeatureExtractor            HF/models/wav2vec2/feature_extraction_wav2vec2.py:78-97, 214-229
  WavLMFeatureEncoder                 HF/models/wavlm/modeling_wavlm.py:675-782
  WavLMFeatureProjection              HF/models/wavlm/modeling_wavlm.py:93-105
  WavLMPositionalConvEmbedding        HF/models/wavlm/modeling_wavlm.py:37-90
  WavLMEncoder(.StableLayerNorm)      HF/models/wavlm/modeling_wavlm.py:388-447, 465-522
  WavLMAttention (gated rel-pos bias) HF/models/wavlm/modeling_wavlm.py:108-271
  WavLMEncoderLayer(.StableLayerNorm) HF/models/wavlm/modeling_wavlm.py:274-373
  extract_wavlm_embeddings pooling    REF/WavLM_embeddings.py:302-323
Arithmetic is fp32 by default (the reference runs fp32 on CPU); ``dtype=np.float64`` gives
a higher-precision restatement for error budgeting.
"""
from __future__ import annotations

import math

import numpy as np
from scipy.special import erf


def gelu(x):
    """erf-GELU (ACT2FN["gelu"] -> nn.functional.gelu, exact)."""
    return (0.5 * x * (1.0 + erf(x / np.asarray(math.sqrt(2.0), dtype=x.dtype)))).astype(x.dtype)


def layer_norm(x, w, b, eps):
    mu = x.mean(axis=-1, keepdims=True)
    var = ((x - mu) ** 2).mean(axis=-1, keepdims=True)
    return ((x - mu) / np.sqrt(var + eps) * w + b).astype(x.dtype)


def normalize(wave: np.ndarray) -> np.ndarray:
    """zero_mean_unit_var_norm, unpadded case (feature_extraction_wav2vec2.py:94)."""
    x = wave.astype(np.float32)
    return ((x - x.mean()) / np.sqrt(x.var() + 1e-7)).astype(np.float32)


def _frames(x: np.ndarray, k: int, s: int) -> np.ndarray:
    """[T_in, C] channels-last -> im2col view [T_out, k*C] (row t = x[s*t : s*t+k])."""
    t_in, c = x.shape
    t_out = (t_in - k) // s + 1
    x = np.ascontiguousarray(x)
    v = np.lib.stride_tricks.as_strided(x, shape=(t_out, k * c), strides=(s * c * x.itemsize, x.itemsize))
    return np.ascontiguousarray(v)     # BLAS needs a dense operand (a strided view takes numpy's slow loop)


def conv1d_cl(x, w, stride, bias=None):
    """Conv1d on channels-last input. w: HF layout [out, in, k]."""
    co, ci, k = w.shape
    wk = np.ascontiguousarray(w.transpose(2, 1, 0).reshape(k * ci, co))  # [(j, c), out]
    y = _frames(x, k, stride) @ wk
    if bias is not None:
        y = y + bias
    return y.astype(x.dtype)


def rel_position_buckets(q_len: int, k_len: int, num_buckets: int = 320, max_distance: int = 800):
    """WavLMAttention._relative_positions_bucket (modeling_wavlm.py:246-271), float32 log path."""
    ctx = np.arange(q_len, dtype=np.int64)[:, None]
    mem = np.arange(k_len, dtype=np.int64)[None, :]
    rel = mem - ctx
    nb = num_buckets // 2
    buckets = (rel > 0).astype(np.int64) * nb
    rel = np.abs(rel)
    max_exact = nb // 2
    is_small = rel < max_exact
    with np.errstate(divide="ignore"):
        lg = np.log(rel.astype(np.float32) / np.float32(max_exact))
    lg = lg / np.float32(math.log(max_distance / max_exact))
    lg = lg * np.float32(nb - max_exact)
    with np.errstate(invalid="ignore"):
        large = (np.float32(max_exact) + lg).astype(np.int64)
    large = np.minimum(large, nb - 1)
    return buckets + np.where(is_small, rel, large)


def weight_norm_dim2(g, v):
    """nn.utils.parametrizations.weight_norm(dim=2): w = g * v / ||v|| over dims (0, 1)."""
    n = np.sqrt((v.astype(np.float64) ** 2).sum(axis=(0, 1), keepdims=True))
    return (g * (v / n)).astype(np.float32)


class WavLMOracle:
    def __init__(self, spec, sd: dict, dtype=np.float32):
        self.spec, self.dt = spec, dtype
        self.p = {k: np.asarray(v, dtype=dtype) for k, v in sd.items()}
        pre = "encoder.pos_conv_embed.conv.parametrizations.weight."
        self.pos_w = weight_norm_dim2(sd[pre + "original0"], sd[pre + "original1"]).astype(dtype)

    # --- conv feature encoder (HF :675-782) ------------------------------------------
    def feature_encoder(self, wave):
        s, p = self.spec, self.p
        x = wave.astype(self.dt)[:, None]                       # [L, 1] channels-last
        for i, (k, st) in enumerate(zip(s.conv_kernel, s.conv_stride)):
            q = f"feature_extractor.conv_layers.{i}"
            x = conv1d_cl(x, p[f"{q}.conv.weight"], st, p.get(f"{q}.conv.bias"))
            if s.feat_norm_layer:
                x = layer_norm(x, p[f"{q}.layer_norm.weight"], p[f"{q}.layer_norm.bias"], 1e-5)
            elif i == 0:                                        # GroupNorm(C, C): per channel over time
                mu = x.mean(axis=0, keepdims=True)
                var = ((x - mu) ** 2).mean(axis=0, keepdims=True)
                x = ((x - mu) / np.sqrt(var + 1e-5) * p[f"{q}.layer_norm.weight"]
                     + p[f"{q}.layer_norm.bias"]).astype(self.dt)
            x = gelu(x)
        return x                                                # [T, C]

    def pos_conv(self, x):
        """Grouped conv k=128, pad 64, drop last frame, GELU (HF :48-90)."""
        s = self.spec
        T, H = x.shape
        G, K = s.pos_groups, s.pos_kernel
        cg = H // G
        pad = np.zeros((T + 2 * (K // 2), H), dtype=self.dt)
        pad[K // 2:K // 2 + T] = x
        out = np.empty((T, H), dtype=self.dt)
        for g in range(G):
            wg = self.pos_w[g * cg:(g + 1) * cg]                 # [cg_out, cg_in, K]
            wk = np.ascontiguousarray(wg.transpose(2, 1, 0).reshape(K * cg, cg))
            xg = np.ascontiguousarray(pad[:, g * cg:(g + 1) * cg])
            out[:, g * cg:(g + 1) * cg] = _frames(xg, K, 1)[:T] @ wk
        out = out + self.p["encoder.pos_conv_embed.conv.bias"]
        return gelu(out.astype(self.dt))

    def attention(self, x, l, bias_hij):
        """WavLMAttention.forward (HF :141-186) + F.multi_head_attention_forward (SDPA, scale 1/sqrt(d))."""
        s, p = self.spec, self.p
        q_ = f"encoder.layers.{l}.attention"
        T, H = x.shape
        nh, hd = s.heads, s.head_dim
        q = x @ p[f"{q_}.q_proj.weight"].T + p[f"{q_}.q_proj.bias"]
        k = x @ p[f"{q_}.k_proj.weight"].T + p[f"{q_}.k_proj.bias"]
        v = x @ p[f"{q_}.v_proj.weight"].T + p[f"{q_}.v_proj.bias"]
        # gate from the layer's attention INPUT split per head (HF :158-170)
        gh = x.reshape(T, nh, hd)
        rp = gh @ p[f"{q_}.gru_rel_pos_linear.weight"].T + p[f"{q_}.gru_rel_pos_linear.bias"]  # [T, nh, 8]
        rp = rp.reshape(T, nh, 2, 4).sum(-1)
        sg = 1.0 / (1.0 + np.exp(-rp))
        const = p[f"{q_}.gru_rel_pos_const"].reshape(nh)
        gate = sg[..., 0] * (sg[..., 1] * const - 1.0) + 2.0                                     # [T, nh]
        qh, kh, vh = (a.reshape(T, nh, hd).transpose(1, 0, 2) for a in (q, k, v))
        sc = qh @ kh.transpose(0, 2, 1) * np.asarray(1.0 / math.sqrt(hd), self.dt)
        sc = sc + gate.T[:, :, None] * bias_hij
        sc = sc - sc.max(-1, keepdims=True)
        e = np.exp(sc)
        pr = e / e.sum(-1, keepdims=True)
        ctx = (pr @ vh).transpose(1, 0, 2).reshape(T, H).astype(self.dt)
        return (ctx @ p[f"{q_}.out_proj.weight"].T + p[f"{q_}.out_proj.bias"]).astype(self.dt)

    def ffn(self, x, l):
        p, q_ = self.p, f"encoder.layers.{l}.feed_forward"
        h = gelu((x @ p[f"{q_}.intermediate_dense.weight"].T + p[f"{q_}.intermediate_dense.bias"]).astype(self.dt))
        return (h @ p[f"{q_}.output_dense.weight"].T + p[f"{q_}.output_dense.bias"]).astype(self.dt)

    def hidden_states(self, wave, do_normalize=False):
        """All len(layers)+1 hidden states of WavLMModel(..., output_hidden_states=True), one clip."""
        s, p, eps = self.spec, self.p, self.spec.ln_eps
        if do_normalize:
            wave = normalize(wave)
        f = self.feature_encoder(wave)
        f = layer_norm(f, p["feature_projection.layer_norm.weight"], p["feature_projection.layer_norm.bias"], eps)
        x = (f @ p["feature_projection.projection.weight"].T + p["feature_projection.projection.bias"]).astype(self.dt)
        x = x + self.pos_conv(x)
        if not s.stable_layer_norm:
            x = layer_norm(x, p["encoder.layer_norm.weight"], p["encoder.layer_norm.bias"], eps)
        T = x.shape[0]
        bk = rel_position_buckets(T, T, s.num_buckets, s.max_distance)
        # [nh, T, T], made contiguous: added to every layer's scores (a strided view makes numpy's
        # broadcast add ~5x slower, which only mattered for the timed CPU baseline)
        bias = np.ascontiguousarray(p["encoder.layers.0.attention.rel_attn_embed.weight"][bk].transpose(2, 0, 1))
        hs = []
        for l in range(s.layers):
            hs.append(x)
            q_ = f"encoder.layers.{l}"
            if s.stable_layer_norm:                              # HF :339-373
                a = self.attention(layer_norm(x, p[f"{q_}.layer_norm.weight"], p[f"{q_}.layer_norm.bias"], eps), l, bias)
                x = x + a
                x = x + self.ffn(layer_norm(x, p[f"{q_}.final_layer_norm.weight"],
                                            p[f"{q_}.final_layer_norm.bias"], eps), l)
            else:                                                # HF :314-336
                x = layer_norm(x + self.attention(x, l, bias), p[f"{q_}.layer_norm.weight"],
                               p[f"{q_}.layer_norm.bias"], eps)
                x = layer_norm(x + self.ffn(x, l), p[f"{q_}.final_layer_norm.weight"],
                               p[f"{q_}.final_layer_norm.bias"], eps)
        if s.stable_layer_norm:
            x = layer_norm(x, p["encoder.layer_norm.weight"], p["encoder.layer_norm.bias"], eps)
        hs.append(x)
        return hs

    def embed(self, waves, layer_indices, do_normalize=False):
        """Batched form of extract_wavlm_embeddings: [B, L] -> [B, n_layers, H] (REF :313-323)."""
        waves = np.atleast_2d(waves)
        out = np.zeros((waves.shape[0], len(layer_indices), self.spec.hidden), dtype=np.float32)
        for b in range(waves.shape[0]):
            hs = self.hidden_states(waves[b], do_normalize)
            for j, idx in enumerate(layer_indices):
                out[b, j] = hs[idx].mean(axis=0)
        return out
