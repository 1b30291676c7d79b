"""Model shapes for the hot path and the canonical weight order of the C-ABI blob.

The reference never builds a model itself: it calls ``WavLMModel.from_pretrained`` /
``WhisperModel.from_pretrained`` by hub name (REF/WavLM_embeddings.py:482-483,
REF/whisper_embeddings_large.py:437-438) and reads the shapes from the hub
``config.json``.  The two specs below restate those shapes:

* ``WavLMSpec()`` == ``transformers.WavLMConfig()`` defaults == microsoft/wavlm-base
  (HF/models/wavlm/configuration_wavlm.py:159-213).
* ``WAVLM_LARGE`` == microsoft/wavlm-large (layer-norm conv frontend, stable-LN
  encoder; HF/models/wavlm/modeling_wavlm.py:696-720, 339-373, 450-522).
* ``WHISPER_LARGE_V2`` / ``WHISPER_TINY`` == the encoder of openai/whisper-large-v2 / -tiny
  (HF/models/whisper/modeling_whisper.py:540-646).

``param_specs(spec)`` is the ONE canonical ordering of HF state-dict tensors that the
C-ABI ``sse_model_create`` consumes as a flat fp32 blob.  ``csrc/sse_model.hip``
(build_wavlm / build_whisper) walks the same order; ``sse_weight_floats`` lets the host check that both sides agree.
"""
from __future__ import annotations

from dataclasses import dataclass, field

KIND_WAVLM = 0
KIND_WHISPER = 1


@dataclass(frozen=True)
class WavLMSpec:
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    ffn: int = 3072
    conv_dim: tuple = (512, 512, 512, 512, 512, 512, 512)
    conv_kernel: tuple = (10, 3, 3, 3, 3, 2, 2)
    conv_stride: tuple = (5, 2, 2, 2, 2, 2, 2)
    conv_bias: bool = False
    feat_norm_layer: bool = False      # False: GroupNorm on conv0 only ("group"); True: LN after every conv ("layer")
    stable_layer_norm: bool = False    # False: post-LN encoder (base); True: pre-LN + final LN (large)
    pos_kernel: int = 128
    pos_groups: int = 16
    num_buckets: int = 320
    max_distance: int = 800
    ln_eps: float = 1e-5
    name: str = "wavlm-base"
    kind: int = field(default=KIND_WAVLM)

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads

    @property
    def num_hidden_states(self) -> int:
        # WavLMEncoder.forward records the input of every layer plus the last output
        # (HF/models/wavlm/modeling_wavlm.py:412-439): layers + 1 entries.
        return self.layers + 1

    def frames(self, n_samples: int) -> int:
        """Output length of the conv feature encoder (HF ``_get_feat_extract_output_lengths``)."""
        t = n_samples
        for k, s in zip(self.conv_kernel, self.conv_stride):
            t = (t - k) // s + 1
        return t

    def default_layer_indices(self) -> list[int]:
        """``[N-1, N-2, N-3, N//2]`` with N = len(hidden_states) (REF/WavLM_embeddings.py:506)."""
        n = self.num_hidden_states
        return [n - 1, n - 2, n - 3, n // 2]


WAVLM_BASE = WavLMSpec()
WAVLM_LARGE = WavLMSpec(hidden=1024, layers=24, heads=16, ffn=4096, feat_norm_layer=True,
                        stable_layer_norm=True, name="wavlm-large")


@dataclass(frozen=True)
class WhisperSpec:
    d_model: int = 1280
    layers: int = 32
    heads: int = 20
    ffn: int = 5120
    n_mels: int = 80
    max_positions: int = 1500
    ln_eps: float = 1e-5
    name: str = "whisper-large-v2"
    kind: int = field(default=KIND_WHISPER)

    @property
    def hidden(self) -> int:
        return self.d_model

    @property
    def head_dim(self) -> int:
        return self.d_model // self.heads

    @property
    def num_hidden_states(self) -> int:
        return self.layers + 1

    n_samples: int = 480000      # 30 s @ 16 kHz (WhisperFeatureExtractor.n_samples)
    n_frames: int = 3000         # mel frames after dropping the last STFT frame
    decoder_layers: int = 0      # >0: also the 1-token decoder pass (REF/whisper_embeddings_large.py:257-262)
    dec_ffn: int = 0             # decoder_ffn_dim (defaults to ffn)
    vocab_size: int = 51865
    max_target_positions: int = 448

    @property
    def dec_ffn_dim(self) -> int:
        return self.dec_ffn or self.ffn

    def default_decoder_indices(self) -> list[int]:
        """``decoder_indices`` of the reference: the last three decoder hidden states."""
        n = self.decoder_layers + 1
        return [n - 1, n - 2, n - 3]

    def default_layer_indices(self) -> list[int]:
        """``encoder_indices`` of the reference: the last three hidden states
        (REF/whisper_embeddings_large.py:454-455)."""
        n = self.num_hidden_states
        return [n - 1, n - 2, n - 3]


WHISPER_LARGE_V2 = WhisperSpec()
WHISPER_TINY = WhisperSpec(d_model=384, layers=4, heads=6, ffn=1536, name="whisper-tiny")
# openai/whisper-small: the reference's default --model_name (REF/whisper_embeddings_large.py:34)
WHISPER_SMALL = WhisperSpec(d_model=768, layers=12, heads=12, ffn=3072, name="whisper-small")
# encoder + the reference's 1-token decoder pass (decoder_layer_* embeddings)
WHISPER_LARGE_V2_DEC = WhisperSpec(decoder_layers=32, name="whisper-large-v2+decoder")
WHISPER_TINY_DEC = WhisperSpec(d_model=384, layers=4, heads=6, ffn=1536, decoder_layers=4, name="whisper-tiny+decoder")
WHISPER_SMALL_DEC = WhisperSpec(d_model=768, layers=12, heads=12, ffn=3072, decoder_layers=12,
                                name="whisper-small+decoder")


def param_specs(spec) -> list[tuple[str, tuple]]:
    """Canonical (HF state-dict key, shape) order of the C-ABI weight blob."""
    out: list[tuple[str, tuple]] = []
    if isinstance(spec, WavLMSpec):
        H, F = spec.hidden, spec.ffn
        cin = 1
        for i, (cd, k) in enumerate(zip(spec.conv_dim, spec.conv_kernel)):
            p = f"feature_extractor.conv_layers.{i}"
            out.append((f"{p}.conv.weight", (cd, cin, k)))
            if spec.conv_bias:
                out.append((f"{p}.conv.bias", (cd,)))
            if spec.feat_norm_layer or i == 0:
                out.append((f"{p}.layer_norm.weight", (cd,)))
                out.append((f"{p}.layer_norm.bias", (cd,)))
            cin = cd
        C = spec.conv_dim[-1]
        out += [("feature_projection.layer_norm.weight", (C,)),
                ("feature_projection.layer_norm.bias", (C,)),
                ("feature_projection.projection.weight", (H, C)),
                ("feature_projection.projection.bias", (H,)),
                ("encoder.pos_conv_embed.conv.parametrizations.weight.original0", (1, 1, spec.pos_kernel)),
                ("encoder.pos_conv_embed.conv.parametrizations.weight.original1",
                 (H, H // spec.pos_groups, spec.pos_kernel)),
                ("encoder.pos_conv_embed.conv.bias", (H,)),
                ("encoder.layer_norm.weight", (H,)),
                ("encoder.layer_norm.bias", (H,)),
                ("encoder.layers.0.attention.rel_attn_embed.weight", (spec.num_buckets, spec.heads))]
        for l in range(spec.layers):
            p = f"encoder.layers.{l}"
            for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
                out.append((f"{p}.attention.{n}.weight", (H, H)))
                out.append((f"{p}.attention.{n}.bias", (H,)))
            out += [(f"{p}.attention.gru_rel_pos_const", (1, spec.heads, 1, 1)),
                    (f"{p}.attention.gru_rel_pos_linear.weight", (8, spec.head_dim)),
                    (f"{p}.attention.gru_rel_pos_linear.bias", (8,)),
                    (f"{p}.layer_norm.weight", (H,)),
                    (f"{p}.layer_norm.bias", (H,)),
                    (f"{p}.feed_forward.intermediate_dense.weight", (F, H)),
                    (f"{p}.feed_forward.intermediate_dense.bias", (F,)),
                    (f"{p}.feed_forward.output_dense.weight", (H, F)),
                    (f"{p}.feed_forward.output_dense.bias", (H,)),
                    (f"{p}.final_layer_norm.weight", (H,)),
                    (f"{p}.final_layer_norm.bias", (H,))]
        return out
    if isinstance(spec, WhisperSpec):
        D, F = spec.d_model, spec.ffn
        out += [("encoder.conv1.weight", (D, spec.n_mels, 3)), ("encoder.conv1.bias", (D,)),
                ("encoder.conv2.weight", (D, D, 3)), ("encoder.conv2.bias", (D,)),
                ("encoder.embed_positions.weight", (spec.max_positions, D))]
        for l in range(spec.layers):
            p = f"encoder.layers.{l}"
            out += [(f"{p}.self_attn.q_proj.weight", (D, D)), (f"{p}.self_attn.q_proj.bias", (D,)),
                    (f"{p}.self_attn.k_proj.weight", (D, D)),
                    (f"{p}.self_attn.v_proj.weight", (D, D)), (f"{p}.self_attn.v_proj.bias", (D,)),
                    (f"{p}.self_attn.out_proj.weight", (D, D)), (f"{p}.self_attn.out_proj.bias", (D,)),
                    (f"{p}.self_attn_layer_norm.weight", (D,)), (f"{p}.self_attn_layer_norm.bias", (D,)),
                    (f"{p}.fc1.weight", (F, D)), (f"{p}.fc1.bias", (F,)),
                    (f"{p}.fc2.weight", (D, F)), (f"{p}.fc2.bias", (D,)),
                    (f"{p}.final_layer_norm.weight", (D,)), (f"{p}.final_layer_norm.bias", (D,))]
        out += [("encoder.layer_norm.weight", (D,)), ("encoder.layer_norm.bias", (D,))]
        if spec.decoder_layers:
            # Only what the 1-token pass with input id 0 at position 0 reads: row 0 of both
            # embedding tables; of the causal self-attention (one key) only v_proj / out_proj
            # matter (softmax over a single key is exactly 1).
            Fd = spec.dec_ffn_dim
            out += [("decoder.embed_tokens.weight[0]", (D,)), ("decoder.embed_positions.weight[0]", (D,))]
            for l in range(spec.decoder_layers):
                p = f"decoder.layers.{l}"
                out += [(f"{p}.self_attn_layer_norm.weight", (D,)), (f"{p}.self_attn_layer_norm.bias", (D,)),
                        (f"{p}.self_attn.v_proj.weight", (D, D)), (f"{p}.self_attn.v_proj.bias", (D,)),
                        (f"{p}.self_attn.out_proj.weight", (D, D)), (f"{p}.self_attn.out_proj.bias", (D,)),
                        (f"{p}.encoder_attn_layer_norm.weight", (D,)), (f"{p}.encoder_attn_layer_norm.bias", (D,)),
                        (f"{p}.encoder_attn.q_proj.weight", (D, D)), (f"{p}.encoder_attn.q_proj.bias", (D,)),
                        (f"{p}.encoder_attn.k_proj.weight", (D, D)),
                        (f"{p}.encoder_attn.v_proj.weight", (D, D)), (f"{p}.encoder_attn.v_proj.bias", (D,)),
                        (f"{p}.encoder_attn.out_proj.weight", (D, D)), (f"{p}.encoder_attn.out_proj.bias", (D,)),
                        (f"{p}.final_layer_norm.weight", (D,)), (f"{p}.final_layer_norm.bias", (D,)),
                        (f"{p}.fc1.weight", (Fd, D)), (f"{p}.fc1.bias", (Fd,)),
                        (f"{p}.fc2.weight", (D, Fd)), (f"{p}.fc2.bias", (D,))]
            out += [("decoder.layer_norm.weight", (D,)), ("decoder.layer_norm.bias", (D,))]
        return out
    raise TypeError(f"unknown spec {spec!r}")


def weight_floats(spec) -> int:
    n = 0
    for _, shp in param_specs(spec):
        c = 1
        for s in shp:
            c *= s
        n += c
    return n
