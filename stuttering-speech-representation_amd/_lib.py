"""ctypes binding of libsse.so (include/sse.h).

The library is built in-tree (``csrc/Makefile`` -> ``libsse.so`` next to this file) by
``__graft_entry__.build()``.  There is deliberately NO fallback: if the library is missing
or a call fails, this module raises, so a GPU run can never silently fall back to CPU or
eager-PyTorch math.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

from .config import KIND_WAVLM, WavLMSpec, WhisperSpec

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsse.so")

SSE_DTYPE_F32 = 0
SSE_DTYPE_BF16 = 1
SSE_DTYPE_FP8 = 2   # bf16 activations + MX-fp8 encoder-layer GEMMs (Whisper)
SSE_DTYPE_FP16X3 = 3   # fp32 activations, split-fp16 (hi/lo) GEMMs: fp32-class results (WavLM-base)
SSE_DTYPE_FP16 = 4   # the bf16 path with fp16 activations / weights / MFMA operands (WavLM-base)
SSE_ERR_INVALID = -1
SSE_ERR_OOM = -6
SSE_ERR_RANGE = -7   # an fp16-range call wrote a non-finite value (sse_check_range)

EXPORTED = ("sse_weight_floats", "sse_model_create", "sse_model_destroy", "sse_output_frames",
            "sse_workspace_bytes", "sse_logmel_workspace_bytes", "sse_logmel", "sse_embed",
            "sse_hidden_states", "sse_strerror", "sse_rel_bucket", "sse_mel_filters", "sse_version",
            "sse_normalize", "sse_normalize_workspace_bytes", "sse_whisper_hidden_states_from_mel",
            "sse_profile_start", "sse_profile_read", "sse_profile_stop", "sse_gemm", "sse_whisper_embed",
            "sse_whisper_decoder_hidden_states", "sse_mono", "sse_resample_length", "sse_resample_workspace_bytes",
            "sse_resample", "sse_augment", "sse_mx_scale_bytes", "sse_mx_scale_offset", "sse_mx_quantize",
            "sse_mx_quantize_host", "sse_gemm_mx", "sse_pitch_shift_workspace_bytes", "sse_pitch_shift",
            "sse_set_option", "sse_get_option", "sse_embed_ragged", "sse_gemm_lnfold", "sse_check_range",
            "sse_attention", "sse_gemm_ex", "sse_attention_f8", "sse_layernorm_mx", "sse_attention_f8_mx")


class SSEError(RuntimeError):
    def __init__(self, rc: int, what: str):
        self.rc = rc
        super().__init__(f"{what}: {strerror(rc)} ({rc})")


class SSEOutOfMemoryError(SSEError, MemoryError):
    pass


class SSERangeError(SSEError, OverflowError):
    """An fp16-range dtype (fp16, fp16x3) produced a non-finite output: an activation left the fp16
    range somewhere in the forward (sse_check_range)."""


class sse_gemm_desc(ctypes.Structure):
    """include/sse.h sse_gemm_desc (the sse_gemm_ex test hook)."""
    _fields_ = [(n, ctypes.c_int32) for n in ("dtype", "M", "N", "K", "ldc", "act", "apart_nt")] + \
        [("ln_eps", ctypes.c_float)] + \
        [(n, ctypes.c_void_p) for n in ("a", "b", "bias", "acol", "apart", "resid", "resid_t", "rpart", "rln_w",
                                         "rln_b", "opart", "cf", "ct", "zero", "a_scale", "b_scale", "c_scale",
                                         "vamax")] + \
        [(n, ctypes.c_int32) for n in ("c_scale_rm", "vamax_rows")] + \
        [("ct2", ctypes.c_void_p)] + [(n, ctypes.c_int32) for n in ("n_split", "ldc2")]


class sse_cfg(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("hidden", ctypes.c_int32), ("layers", ctypes.c_int32),
                ("heads", ctypes.c_int32), ("ffn", ctypes.c_int32), ("n_conv", ctypes.c_int32),
                ("conv_dim", ctypes.c_int32 * 8), ("conv_kernel", ctypes.c_int32 * 8),
                ("conv_stride", ctypes.c_int32 * 8), ("conv_bias", ctypes.c_int32),
                ("feat_norm_layer", ctypes.c_int32), ("stable_layer_norm", ctypes.c_int32),
                ("pos_kernel", ctypes.c_int32), ("pos_groups", ctypes.c_int32),
                ("num_buckets", ctypes.c_int32), ("max_distance", ctypes.c_int32),
                ("do_normalize", ctypes.c_int32), ("n_mels", ctypes.c_int32),
                ("max_positions", ctypes.c_int32), ("ln_eps", ctypes.c_float),
                ("decoder_layers", ctypes.c_int32), ("dec_ffn", ctypes.c_int32)]


def make_cfg(spec, do_normalize: bool = False) -> sse_cfg:
    c = sse_cfg()
    c.kind = spec.kind
    c.hidden, c.layers, c.heads, c.ffn = spec.hidden, spec.layers, spec.heads, spec.ffn
    c.ln_eps = spec.ln_eps
    if isinstance(spec, WavLMSpec):
        c.n_conv = len(spec.conv_dim)
        for i in range(c.n_conv):
            c.conv_dim[i], c.conv_kernel[i], c.conv_stride[i] = (spec.conv_dim[i], spec.conv_kernel[i],
                                                                spec.conv_stride[i])
        c.conv_bias = int(spec.conv_bias)
        c.feat_norm_layer = int(spec.feat_norm_layer)
        c.stable_layer_norm = int(spec.stable_layer_norm)
        c.pos_kernel, c.pos_groups = spec.pos_kernel, spec.pos_groups
        c.num_buckets, c.max_distance = spec.num_buckets, spec.max_distance
        c.do_normalize = int(do_normalize)
    elif isinstance(spec, WhisperSpec):
        c.n_mels, c.max_positions = spec.n_mels, spec.max_positions
        c.decoder_layers, c.dec_ffn = spec.decoder_layers, spec.dec_ffn_dim
    else:
        raise TypeError(spec)
    assert c.kind in (KIND_WAVLM, 1)
    return c


_lib = None


def use_library(path: str) -> None:
    """Load another build of the same ABI instead of the in-tree libsse.so (same-box A/B timing,
    ``bench.py --lib``).  Must be called before the first ``lib()``; explicit only, never read
    from the environment."""
    global LIB_PATH
    if _lib is not None:
        raise RuntimeError("libsse.so is already loaded")
    LIB_PATH = os.path.abspath(path)


def lib() -> ctypes.CDLL:
    """Load libsse.so (raises ImportError with the build hint if it is absent)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; "
                          f"g.build()'` (hipcc --offload-arch=gfx950); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    L.sse_weight_floats.argtypes = [ctypes.POINTER(sse_cfg)]
    L.sse_weight_floats.restype = sz
    L.sse_model_create.argtypes = [ctypes.POINTER(sse_cfg), vp, sz, i32, i32, ctypes.POINTER(vp)]
    L.sse_model_create.restype = i32
    L.sse_model_destroy.argtypes = [vp]
    L.sse_model_destroy.restype = None
    L.sse_output_frames.argtypes = [vp, i32]
    L.sse_output_frames.restype = i32
    L.sse_workspace_bytes.argtypes = [vp, i32, i32]
    L.sse_workspace_bytes.restype = sz
    L.sse_logmel_workspace_bytes.argtypes = [i32, i32]
    L.sse_logmel_workspace_bytes.restype = sz
    L.sse_logmel.argtypes = [vp, i32, i32, i32, vp, vp, sz, vp]
    L.sse_logmel.restype = i32
    L.sse_embed.argtypes = [vp, vp, i32, i32, vp, i32, vp, vp, sz, vp]
    L.sse_embed.restype = i32
    L.sse_embed_ragged.argtypes = [vp, vp, vp, i32, i32, vp, i32, vp, vp, sz, vp]
    L.sse_embed_ragged.restype = i32
    L.sse_check_range.argtypes = [vp, vp]
    L.sse_check_range.restype = i32
    L.sse_hidden_states.argtypes = [vp, vp, i32, i32, vp, vp, sz, vp]
    L.sse_hidden_states.restype = i32
    L.sse_whisper_hidden_states_from_mel.argtypes = [vp, vp, i32, vp, vp, sz, vp]
    L.sse_whisper_hidden_states_from_mel.restype = i32
    L.sse_normalize.argtypes = [vp, i32, i32, vp, vp, sz, vp]
    L.sse_normalize.restype = i32
    L.sse_normalize_workspace_bytes.argtypes = [i32]
    L.sse_normalize_workspace_bytes.restype = sz
    L.sse_profile_start.argtypes = [vp, i32]
    L.sse_profile_start.restype = i32
    L.sse_profile_read.argtypes = [vp, i32, vp, vp, vp, vp]
    L.sse_profile_read.restype = i32
    L.sse_profile_stop.argtypes = [vp]
    L.sse_profile_stop.restype = i32
    L.sse_gemm.argtypes = [i32, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, vp, vp]
    L.sse_gemm.restype = i32
    L.sse_attention.argtypes = [vp, vp, i32, i32, i32, i32, i32, ctypes.c_float, i32, vp]
    L.sse_attention.restype = i32
    if hasattr(L, "sse_gemm_ex"):   # (absent from pre-round-5 builds loaded for A/B runs via set_lib_path)
        L.sse_gemm_ex.argtypes = [ctypes.POINTER(sse_gemm_desc), vp]
        L.sse_gemm_ex.restype = i32
    if hasattr(L, "sse_attention_f8"):
        L.sse_attention_f8.argtypes = [vp, vp, vp, vp, vp, i32, i32, i32, i32, vp]
        L.sse_attention_f8.restype = i32
    if hasattr(L, "sse_attention_f8_mx"):
        L.sse_attention_f8_mx.argtypes = [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, vp]
        L.sse_attention_f8_mx.restype = i32
    L.sse_gemm_lnfold.argtypes = [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, ctypes.c_float, vp, vp]
    L.sse_gemm_lnfold.restype = i32
    L.sse_whisper_embed.argtypes = [vp, vp, i32, i32, vp, i32, vp, vp, i32, vp, vp, sz, vp]
    L.sse_whisper_embed.restype = i32
    L.sse_whisper_decoder_hidden_states.argtypes = [vp, vp, i32, vp, vp, sz, vp]
    L.sse_whisper_decoder_hidden_states.restype = i32
    L.sse_mono.argtypes = [vp, i32, i32, i32, vp, vp]
    L.sse_mono.restype = i32
    L.sse_resample_length.argtypes = [i32, i32, i32]
    L.sse_resample_length.restype = i32
    L.sse_resample_workspace_bytes.argtypes = [i32, i32, i32, i32]
    L.sse_resample_workspace_bytes.restype = sz
    L.sse_resample.argtypes = [vp, i32, i32, i32, i32, vp, vp, sz, vp]
    L.sse_resample.restype = i32
    L.sse_augment.argtypes = [vp, vp, i32, i32, vp, vp, vp, ctypes.c_uint64, vp]
    L.sse_augment.restype = i32
    L.sse_pitch_shift_workspace_bytes.argtypes = [i32, i32, i32, i32]
    L.sse_pitch_shift_workspace_bytes.restype = sz
    L.sse_pitch_shift.argtypes = [vp, i32, i32, i32, i32, vp, vp, sz, vp]
    L.sse_pitch_shift.restype = i32
    L.sse_mx_scale_bytes.argtypes = [i32, i32]
    L.sse_mx_scale_bytes.restype = sz
    L.sse_mx_scale_offset.argtypes = [i32, i32, i32, i32]
    L.sse_mx_scale_offset.restype = ctypes.c_longlong
    L.sse_mx_quantize.argtypes = [vp, i32, i32, i32, vp, vp, vp]
    L.sse_mx_quantize.restype = i32
    L.sse_mx_quantize_host.argtypes = [vp, i32, i32, i32, vp, vp]
    L.sse_mx_quantize_host.restype = i32
    if hasattr(L, "sse_layernorm_mx"):   # (a round-5 build loaded for an A/B lacks this test hook)
        L.sse_layernorm_mx.argtypes = [vp, vp, vp, i32, i32, ctypes.c_float, vp, vp, vp]
        L.sse_layernorm_mx.restype = i32
    L.sse_gemm_mx.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, vp]
    L.sse_gemm_mx.restype = i32
    L.sse_strerror.argtypes = [i32]
    L.sse_strerror.restype = ctypes.c_char_p
    L.sse_rel_bucket.argtypes = [i32, i32, i32]
    L.sse_rel_bucket.restype = i32
    L.sse_mel_filters.argtypes = [i32, vp]
    L.sse_mel_filters.restype = i32
    L.sse_set_option.argtypes = [ctypes.c_char_p, i32]
    L.sse_set_option.restype = i32
    L.sse_get_option.argtypes = [ctypes.c_char_p]
    L.sse_get_option.restype = i32
    L.sse_version.argtypes = []
    L.sse_version.restype = ctypes.c_char_p
    _lib = L
    return L


def strerror(rc: int) -> str:
    try:
        return lib().sse_strerror(rc).decode()
    except ImportError:
        return str(rc)


def check(rc: int, what: str) -> None:
    if rc == 0:
        return
    if rc == SSE_ERR_OOM:
        raise SSEOutOfMemoryError(rc, what)
    if rc == SSE_ERR_RANGE:
        raise SSERangeError(rc, what)
    raise SSEError(rc, what)


@contextlib.contextmanager
def option(name: str, value: int):
    """Temporarily set one of libsse.so's A/B kernel-selection switches (sse_set_option)."""
    prev = lib().sse_set_option(name.encode(), int(value))
    if prev < 0:
        raise SSEError(prev, f"sse_set_option({name!r})")
    try:
        yield
    finally:
        lib().sse_set_option(name.encode(), prev)
