"""CPU-side checks of the C-ABI library: it loads, exports every symbol include/sse.h
declares, and its host-only helpers agree with the reference-side math (no GPU calls)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "sse.h")).read()
    return sorted(set(re.findall(r"\b(sse_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    from ssr_amd import _lib
    L = _lib.lib()
    syms = _header_symbols()
    assert len(syms) >= 15
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert set(_lib.EXPORTED) <= set(syms)
    assert L.sse_version().decode().startswith("sse ")


def test_weight_floats_match_param_specs():
    from ssr_amd import _lib, config as C
    L = _lib.lib()
    for spec in (C.WAVLM_BASE, C.WAVLM_LARGE, C.WHISPER_TINY, C.WHISPER_LARGE_V2, C.WHISPER_TINY_DEC,
                 C.WHISPER_LARGE_V2_DEC):
        cfg = _lib.make_cfg(spec)
        assert L.sse_weight_floats(ctypes.byref(cfg)) == C.weight_floats(spec), spec.name


def test_invalid_config_rejected():
    from ssr_amd import _lib, config as C
    L = _lib.lib()
    cfg = _lib.make_cfg(C.WAVLM_BASE)
    cfg.heads = 7                                   # head_dim != 64
    assert L.sse_weight_floats(ctypes.byref(cfg)) == 0
    h = ctypes.c_void_p()
    blob = np.zeros(10, np.float32)
    assert L.sse_model_create(ctypes.byref(cfg), blob.ctypes.data, blob.nbytes, 0, 0, ctypes.byref(h)) == -1
    cfg = _lib.make_cfg(C.WAVLM_BASE)
    assert L.sse_model_create(ctypes.byref(cfg), blob.ctypes.data, blob.nbytes, 0, 0, ctypes.byref(h)) == -5
    assert L.sse_strerror(-5).decode().startswith("weight blob")


def test_rel_bucket_table_matches_torch():
    """The C++ bucket (used to build the device bias table) equals HF's float32 torch path
    for every distance the table covers (|d| <= 4095)."""
    import torch
    from ssr_amd import _lib
    from transformers.models.wavlm.modeling_wavlm import WavLMAttention
    L = _lib.lib()
    d = torch.arange(-4095, 4096)[None, :]
    ref = WavLMAttention(768, 12)._relative_positions_bucket(d)[0].numpy()
    ours = np.array([L.sse_rel_bucket(int(x), 320, 800) for x in range(-4095, 4096)])
    assert np.array_equal(ours, ref)


def test_mel_filters_match_hf():
    from ssr_amd import _lib
    from transformers.audio_utils import mel_filter_bank
    fb = np.zeros((201, 80), np.float32)
    assert _lib.lib().sse_mel_filters(80, fb.ctypes.data) == 0
    hf = mel_filter_bank(201, 80, 0.0, 8000.0, 16000, norm="slaney", mel_scale="slaney").astype(np.float32)
    assert np.allclose(fb, hf, rtol=0, atol=1e-12)


def test_ssemodel_refuses_cpu_device(wavlm_sd):
    from ssr_amd import config as C
    from ssr_amd.model import SSEModel
    with pytest.raises(ValueError):
        SSEModel(C.WAVLM_BASE, wavlm_sd, device="cpu")


def test_options_are_explicit_only():
    """A/B kernel switches exist only through sse_set_option (the library reads no environment)."""
    from ssr_amd import _lib
    L = _lib.lib()
    for name in (b"gemm_cfg", b"gemm_nonpersist", b"gelu_exact", b"conv0_valu", b"posconv_gemm", b"no_lnfold",
                 b"gemm_mx_staged", b"fp8_attn_bf16", b"f8_oproj", b"gemm_4phase"):
        assert L.sse_get_option(name) == 0
        with _lib.option(name.decode(), 1):
            assert L.sse_get_option(name) == 1
        assert L.sse_get_option(name) == 0
    assert L.sse_set_option(b"no_such_switch", 1) < 0


def test_option_values_out_of_range_are_rejected():
    """A value outside a switch's range is an error, not a silent fallback (attn_short = 2 used to be
    accepted and run the production kernel); the switch keeps its value."""
    from ssr_amd import _lib
    L = _lib.lib()
    for name, top in ((b"attn_short", 2), (b"attn_long", 2), (b"gemm_cfg", 3), (b"no_split", 1)):
        assert L.sse_get_option(name) == 0
        assert L.sse_set_option(name, top + 1) < 0
        assert L.sse_set_option(name, -1) < 0
        assert L.sse_get_option(name) == 0
        assert L.sse_set_option(name, top) == 0
        assert L.sse_set_option(name, 0) == top


def test_attention_hook_rejects_q_log2_with_other_scale():
    """sse_attention validates before any device work: q_log2 = 1 requires scale = ln 2 (the 32x32 flash
    kernel reads log2-domain logits and never applies a scale; the short-T kernels would)."""
    from ssr_amd import _lib
    L = _lib.lib()
    fake = ctypes.c_void_p(256)   # never dereferenced: rejected on the arguments alone
    assert L.sse_attention(fake, fake, 1, 300, 128, 2, 384, 1.0, 1, None) == _lib.SSE_ERR_INVALID
    assert L.sse_attention(fake, fake, 1, 300, 128, 2, 384, 0.125, 1, None) == _lib.SSE_ERR_INVALID
