"""Host-side model handle over libsse.so: weights in, batched embeddings out.

``SSEModel`` is the perf surface of SURVEY.md §8(b):
``embed(wave[B, L]) -> [B, n_layers, H]`` (the fused mean-pooled output of
``extract_wavlm_embeddings`` / ``extract_whisper_embeddings_fixed`` for a whole batch),
plus ``hidden_states`` (the full HF-shaped tuple, materialised only on request).

Every tensor argument lives on the model's GPU; all compute runs in the HIP kernels of
``csrc/`` on the current torch stream.  There is no CPU path.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .config import WavLMSpec, WhisperSpec, param_specs

DTYPES = {"fp32": _lib.SSE_DTYPE_F32, "float32": _lib.SSE_DTYPE_F32, "f32": _lib.SSE_DTYPE_F32,
          "bf16": _lib.SSE_DTYPE_BF16, "bfloat16": _lib.SSE_DTYPE_BF16,
          "fp8": _lib.SSE_DTYPE_FP8, "mxfp8": _lib.SSE_DTYPE_FP8, "fp16x3": _lib.SSE_DTYPE_FP16X3,
          "fp16": _lib.SSE_DTYPE_FP16, "float16": _lib.SSE_DTYPE_FP16}
# dtypes whose activations live in the fp16 range: their calls are range-checked (sse_check_range)
FP16_RANGE = ("fp16", "float16", "fp16x3")


def _as_numpy(v) -> np.ndarray:
    if isinstance(v, torch.Tensor):
        v = v.detach().to("cpu", torch.float32).numpy()
    return np.ascontiguousarray(np.asarray(v, dtype=np.float32))


def pack_weights(spec, state_dict: dict) -> np.ndarray:
    """Concatenate an HF state dict into the canonical fp32 blob (config.param_specs order).

    Accepts WavLMModel / WhisperModel state dicts (``encoder.``-prefixed keys for Whisper, as
    ``WhisperModel.state_dict()`` has them) with numpy arrays or torch tensors; the legacy
    ``weight_g`` / ``weight_v`` names of the WavLM pos-conv weight norm are mapped to the
    parametrization names.
    """
    sd = dict(state_dict)
    pre = "encoder.pos_conv_embed.conv."
    if pre + "weight_g" in sd and pre + "parametrizations.weight.original0" not in sd:
        sd[pre + "parametrizations.weight.original0"] = sd.pop(pre + "weight_g")
        sd[pre + "parametrizations.weight.original1"] = sd.pop(pre + "weight_v")
    parts = []
    for key, shape in param_specs(spec):
        if key.endswith("[0]") and key not in sd:        # row 0 of an embedding table
            base = key[:-3]
            if base not in sd:
                raise KeyError(f"state dict lacks {base}")
            v = sd[base]
            a = _as_numpy(v[0] if isinstance(v, torch.Tensor) else np.asarray(v)[0])
        elif key not in sd:
            raise KeyError(f"state dict lacks {key}")
        else:
            a = _as_numpy(sd[key])
        if tuple(a.shape) != tuple(shape):
            raise ValueError(f"{key}: shape {tuple(a.shape)} != expected {tuple(shape)}")
        parts.append(a.ravel())
    return np.concatenate(parts)


class SSEModel:
    """One model on one GPU.  ``dtype``: "bf16" (throughput path), "fp32" (parity path), "fp16x3"
    (WavLM-base: fp32 activations, split-fp16 GEMMs -- fp32-class parity at ~3x the fp32 path's
    throughput) or "fp8" (Whisper only: bf16 activations, MX-fp8 QKV / fc1 / fc2 GEMMs, BASELINE
    configs[4]), "fp16" (WavLM-base: the bf16 path with fp16 activations and operands -- the same
    matrix-core rate, 8 more mantissa bits).

    fp16 / fp16x3 keep activations in the fp16 range: with ``check_range`` (default) every embed /
    hidden_states call synchronises and raises ``SSERangeError`` if it produced a non-finite value
    (an overflow); throughput loops pass ``check_range=False`` and call ``check_range_now()`` once."""

    def __init__(self, spec, state_dict: dict, device="cuda:0", dtype: str = "bf16", do_normalize: bool = False,
                 check_range: bool = True):
        if not isinstance(spec, (WavLMSpec, WhisperSpec)):
            raise TypeError(spec)
        self.spec = spec
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("SSEModel runs on a GPU device (no CPU fallback)")
        self.dtype = dtype
        self.do_normalize = bool(do_normalize)
        L = _lib.lib()
        self._cfg = _lib.make_cfg(spec, do_normalize)
        blob = pack_weights(spec, state_dict)
        need = L.sse_weight_floats(ctypes.byref(self._cfg))
        if need != blob.size:
            raise ValueError(f"weight blob has {blob.size} floats, library expects {need}")
        h = ctypes.c_void_p()
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.device = torch.device("cuda", idx)
        torch.cuda.set_device(self.device)   # make sure the HIP context exists on this device
        _lib.check(L.sse_model_create(ctypes.byref(self._cfg), blob.ctypes.data, blob.nbytes, idx,
                                      DTYPES[dtype], ctypes.byref(h)), "sse_model_create")
        self._h = h
        self._ws = None
        self.check_range = bool(check_range) and dtype in FP16_RANGE

    # -- plumbing -------------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.lib().sse_model_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def hidden_size(self) -> int:
        return self.spec.hidden

    def output_frames(self, n_samples: int) -> int:
        return _lib.lib().sse_output_frames(self._h, int(n_samples))

    def workspace(self, B: int, L: int) -> torch.Tensor:
        n = _lib.lib().sse_workspace_bytes(self._h, int(B), int(L))
        if n == 0:
            raise _lib.SSEError(-1, f"sse_workspace_bytes(B={B}, L={L})")
        if self._ws is None or self._ws.numel() < n:
            self._ws = None
            self._ws = torch.empty(n, dtype=torch.uint8, device=self.device)
        return self._ws

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def check_range_now(self) -> None:
        """Synchronise the current stream; raise SSERangeError if a call since the last check wrote a
        non-finite value (fp16 / fp16x3 models; a no-op for the others)."""
        _lib.check(_lib.lib().sse_check_range(self._h, self._stream()), "sse_check_range")

    def _after(self, check_range: bool | None = None):
        if self.check_range if check_range is None else (check_range and self.dtype in FP16_RANGE):
            self.check_range_now()

    def _check_wave(self, wave: torch.Tensor) -> torch.Tensor:
        if not isinstance(wave, torch.Tensor) or wave.device != self.device:
            raise ValueError(f"expected a tensor on {self.device}")
        if wave.dim() == 1:
            wave = wave[None]
        if wave.dim() != 2:
            raise ValueError("expected [B, L] waves")
        return wave.to(torch.float32).contiguous()

    # -- live launch timing (bench.py) ------------------------------------------------------
    def profile_start(self, max_launches: int = 8192) -> None:
        _lib.check(_lib.lib().sse_profile_start(self._h, int(max_launches)), "sse_profile_start")
        self._prof_cap = int(max_launches)

    def profile_read(self) -> list:
        """[(tag, ms, flops, bytes)] for every launch since profile_start / the last read."""
        cap = self._prof_cap
        tags = ctypes.create_string_buffer(32 * cap)
        ms = np.zeros(cap, np.float32)
        fl = np.zeros(cap, np.float64)
        by = np.zeros(cap, np.float64)
        n = _lib.lib().sse_profile_read(self._h, cap, tags, ms.ctypes.data, fl.ctypes.data, by.ctypes.data)
        if n < 0:
            _lib.check(n, "sse_profile_read")
        raw = tags.raw
        return [(raw[32 * i:32 * i + 32].split(b"\0", 1)[0].decode(), float(ms[i]), float(fl[i]), float(by[i]))
                for i in range(min(n, cap))]

    def profile_stop(self) -> None:
        _lib.check(_lib.lib().sse_profile_stop(self._h), "sse_profile_stop")

    # -- compute --------------------------------------------------------------------------
    def embed(self, wave: torch.Tensor, layer_indices, out: torch.Tensor | None = None,
              lengths=None, workspace: torch.Tensor | None = None, check_range: bool | None = None) -> torch.Tensor:
        """[B, L] fp32 16 kHz waves -> [B, len(layer_indices), H] fp32 time-means of hidden states.
        ``lengths`` (ragged batch): samples of each clip, its first lengths[b] samples of row b; each
        clip is embedded at its own length (sse_embed_ragged).  ``check_range`` overrides the model's
        per-call fp16-range check (False in throughput loops, which call check_range_now() once)."""
        wave = self._check_wave(wave)
        B, L = wave.shape
        ids = torch.tensor([int(i) for i in layer_indices], dtype=torch.int32)
        n = ids.numel()
        if out is None:
            out = torch.empty((B, n, self.spec.hidden), dtype=torch.float32, device=self.device)
        elif (out.device != self.device or out.dtype != torch.float32 or tuple(out.shape) != (B, n, self.spec.hidden)
              or not out.is_contiguous()):
            raise ValueError(f"out must be a contiguous fp32 [{B}, {n}, {self.spec.hidden}] tensor on {self.device}")
        ws = self.workspace(B, L) if workspace is None else workspace
        if ws.numel() < _lib.lib().sse_workspace_bytes(self._h, int(B), int(L)):
            raise ValueError("workspace too small")
        if lengths is None:
            _lib.check(_lib.lib().sse_embed(self._h, wave.data_ptr(), B, L, ids.data_ptr(), n, out.data_ptr(),
                                            ws.data_ptr(), ws.numel(), self._stream()), "sse_embed")
            self._after(check_range)
            return out
        lens = [int(v) for v in (lengths.tolist() if isinstance(lengths, torch.Tensor) else lengths)]
        if len(lens) != B or min(lens) < 1 or max(lens) > L:
            raise ValueError(f"lengths must be {B} values in [1, {L}]")
        if isinstance(self.spec, WavLMSpec) and min(self.spec.frames(v) for v in lens) <= 0:
            raise _lib.SSEError(-1, "a clip is shorter than the conv receptive field")
        # pinned + non_blocking: the copy is ordered on the current stream without a host sync, so a
        # staged corpus loop keeps its copy / compute overlap (the caching host allocator keeps the
        # pinned buffer alive until the copy has run)
        d_len = torch.tensor(lens, dtype=torch.int32).pin_memory().to(self.device, non_blocking=True)
        _lib.check(_lib.lib().sse_embed_ragged(self._h, wave.data_ptr(), d_len.data_ptr(), B, L, ids.data_ptr(), n,
                                               out.data_ptr(), ws.data_ptr(), ws.numel(), self._stream()),
                   "sse_embed_ragged")
        self._after(check_range)
        return out

    def embed_clips(self, clips, layer_indices) -> torch.Tensor:
        """A list of 1-D clips of any lengths -> [N, len(layer_indices), H]: one ragged batch
        (zero-padded rows + lengths), every clip embedded at its own length."""
        lens = [int(c.shape[-1]) for c in clips]
        wave = torch.zeros((len(clips), max(lens)), dtype=torch.float32, device=self.device)
        for i, c in enumerate(clips):
            c = c if isinstance(c, torch.Tensor) else torch.from_numpy(np.asarray(c, dtype=np.float32))
            wave[i, :lens[i]] = c.to(self.device, torch.float32)
        return self.embed(wave, layer_indices, lengths=lens)

    def hidden_states(self, wave: torch.Tensor) -> tuple:
        """[B, L] -> tuple of layers+1 tensors [B, T, H] (HF ``output_hidden_states`` semantics)."""
        wave = self._check_wave(wave)
        B, L = wave.shape
        T = self.output_frames(L)
        n_hs = self.spec.layers + 1
        hs = torch.empty((n_hs, B, T, self.spec.hidden), dtype=torch.float32, device=self.device)
        ws = self.workspace(B, L)
        _lib.check(_lib.lib().sse_hidden_states(self._h, wave.data_ptr(), B, L, hs.data_ptr(), ws.data_ptr(),
                                                ws.numel(), self._stream()), "sse_hidden_states")
        self._after()
        return tuple(hs.unbind(0))

    def hidden_states_from_mel(self, mel: torch.Tensor) -> tuple:
        """Whisper only: [B, n_mels, 3000] log-mel -> layers+1 tensors [B, 1500, H]."""
        if not isinstance(self.spec, WhisperSpec):
            raise TypeError("hidden_states_from_mel is Whisper-only")
        if mel.device != self.device:
            raise ValueError(f"expected a tensor on {self.device}")
        mel = mel.to(torch.float32).contiguous()
        if mel.dim() != 3 or mel.shape[1] != self.spec.n_mels or mel.shape[2] != 2 * self.spec.max_positions:
            raise ValueError(f"expected [B, {self.spec.n_mels}, {2 * self.spec.max_positions}] log-mel, "
                             f"got {tuple(mel.shape)}")
        B = mel.shape[0]
        T = self.spec.max_positions
        hs = torch.empty((self.spec.layers + 1, B, T, self.spec.hidden), dtype=torch.float32, device=self.device)
        ws = self.workspace(B, self.spec.n_samples)
        _lib.check(_lib.lib().sse_whisper_hidden_states_from_mel(self._h, mel.data_ptr(), B, hs.data_ptr(),
                                                                 ws.data_ptr(), ws.numel(), self._stream()),
                   "sse_whisper_hidden_states_from_mel")
        return tuple(hs.unbind(0))


    def whisper_embed(self, wave: torch.Tensor, encoder_indices, decoder_indices, enc_out=None, dec_out=None):
        """Whisper: encoder time-means AND 1-token decoder states in one pass
        (REF/whisper_embeddings_large.py:234-299) -> ([B, n_enc, H], [B, n_dec, H]) fp32."""
        if not isinstance(self.spec, WhisperSpec):
            raise TypeError("whisper_embed is Whisper-only")
        if decoder_indices and not self.spec.decoder_layers:
            raise ValueError(f"{self.spec.name} was built without the decoder (decoder_layers=0)")
        wave = self._check_wave(wave)
        B, L = wave.shape
        H = self.spec.hidden
        eid = torch.tensor([int(i) for i in encoder_indices], dtype=torch.int32)
        did = torch.tensor([int(i) for i in decoder_indices], dtype=torch.int32)
        if enc_out is None:
            enc_out = torch.empty((B, eid.numel(), H), dtype=torch.float32, device=self.device)
        if dec_out is None:
            dec_out = torch.empty((B, did.numel(), H), dtype=torch.float32, device=self.device)
        ws = self.workspace(B, L)
        _lib.check(_lib.lib().sse_whisper_embed(self._h, wave.data_ptr(), B, L, eid.data_ptr(), eid.numel(),
                                                enc_out.data_ptr() if eid.numel() else None, did.data_ptr(),
                                                did.numel(), dec_out.data_ptr() if did.numel() else None,
                                                ws.data_ptr(), ws.numel(), self._stream()), "sse_whisper_embed")
        return enc_out, dec_out

    def decoder_hidden_states(self, enc: torch.Tensor) -> tuple:
        """Whisper: ``model.decoder(input_ids=zeros([B, 1]), encoder_hidden_states=enc)`` hidden states:
        enc [B, 1500, H] -> decoder_layers+1 tensors [B, 1, H] fp32."""
        if not isinstance(self.spec, WhisperSpec) or not self.spec.decoder_layers:
            raise TypeError("decoder_hidden_states needs a Whisper spec with decoder_layers > 0")
        T, H = self.spec.max_positions, self.spec.hidden
        if enc.device != self.device or enc.dim() != 3 or tuple(enc.shape[1:]) != (T, H):
            raise ValueError(f"expected [B, {T}, {H}] encoder states on {self.device}, got {tuple(enc.shape)}")
        enc = enc.to(torch.float32).contiguous()
        B = enc.shape[0]
        hs = torch.empty((self.spec.decoder_layers + 1, B, 1, H), dtype=torch.float32, device=self.device)
        ws = self.workspace(B, self.spec.n_samples)
        _lib.check(_lib.lib().sse_whisper_decoder_hidden_states(self._h, enc.data_ptr(), B, hs.data_ptr(),
                                                                ws.data_ptr(), ws.numel(), self._stream()),
                   "sse_whisper_decoder_hidden_states")
        return tuple(hs.unbind(0))


def logmel(wave: torch.Tensor, n_mels: int = 80) -> torch.Tensor:
    """Whisper log-mel on device: [B, L] (L <= 480000) -> [B, n_mels, 3000] (HF layout)."""
    if wave.dim() == 1:
        wave = wave[None]
    wave = wave.to(torch.float32).contiguous()
    B, L = wave.shape
    L_ = _lib.lib()
    n = L_.sse_logmel_workspace_bytes(B, n_mels)
    ws = torch.empty(n, dtype=torch.uint8, device=wave.device)
    out = torch.empty((B, n_mels, 3000), dtype=torch.float32, device=wave.device)
    _lib.check(L_.sse_logmel(wave.data_ptr(), B, L, n_mels, out.data_ptr(), ws.data_ptr(), n,
                             ctypes.c_void_p(torch.cuda.current_stream(wave.device).cuda_stream)), "sse_logmel")
    return out


def normalize(wave: torch.Tensor) -> torch.Tensor:
    """Wav2Vec2FeatureExtractor(do_normalize=True) on device: per-clip zero mean / unit variance."""
    if wave.dim() == 1:
        wave = wave[None]
    wave = wave.to(torch.float32).contiguous()
    B, L = wave.shape
    ws = torch.empty(8 * B, dtype=torch.uint8, device=wave.device)
    out = torch.empty_like(wave)
    _lib.check(_lib.lib().sse_normalize(wave.data_ptr(), B, L, out.data_ptr(), ws.data_ptr(), ws.numel(),
                                        ctypes.c_void_p(torch.cuda.current_stream(wave.device).cuda_stream)),
               "sse_normalize")
    return out


_ZERO = {}


def gemm(a: torch.Tensor, b: torch.Tensor, bias=None, resid=None, act: str | None = None,
         out_dtype=torch.float32) -> torch.Tensor:
    """The path's MFMA GEMM on its own: a [M, K] @ b[N, K]^T (+bias) (gelu) (+resid).
    a, b both bf16 (bf16 MFMA) or both fp32 (exact-f32 MFMA).  act: None | "gelu" (erf form) |
    "gelu_fast" (the bf16 path's gelu_fast2 epilogue, common.h)."""
    if a.dtype != b.dtype or a.dtype not in (torch.bfloat16, torch.float32):
        raise TypeError("a and b must both be bf16 or both fp32")
    M, K = a.shape
    N = b.shape[0]
    dev = a.device
    z = _ZERO.get(dev)
    if z is None:
        z = _ZERO[dev] = torch.zeros(64, dtype=torch.float32, device=dev)
    a, b = a.contiguous(), b.contiguous()
    cf = torch.empty((M, N), dtype=torch.float32, device=dev) if out_dtype == torch.float32 else None
    ct = torch.empty((M, N), dtype=a.dtype, device=dev) if out_dtype != torch.float32 else None
    dt = _lib.SSE_DTYPE_BF16 if a.dtype == torch.bfloat16 else _lib.SSE_DTYPE_F32
    bias_p = bias.contiguous().data_ptr() if bias is not None else None
    res_p = resid.contiguous().data_ptr() if resid is not None else None
    _lib.check(_lib.lib().sse_gemm(dt, a.data_ptr(), b.data_ptr(), bias_p, res_p,
                                   cf.data_ptr() if cf is not None else None,
                                   ct.data_ptr() if ct is not None else None, M, N, K, {None: 0, "gelu": 1, "gelu_fast": 2}[act],
                                   z.data_ptr(), ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)),
               "sse_gemm")
    return cf if cf is not None else ct


def mx_scale_bytes(R: int, K: int) -> int:
    return int(_lib.lib().sse_mx_scale_bytes(R, K))


def mx_quantize(x: torch.Tensor, role: int = 0) -> tuple[torch.Tensor, torch.Tensor]:
    """MX-fp8 quantisation on the GPU: fp32 x [R, K] (K % 128 == 0) -> (e4m3 bytes uint8 [R, K],
    E8M0 scales uint8 in the GEMM's role-0 (A) / role-1 (B) tile layout)."""
    x = x.contiguous()
    R, K = x.shape
    q = torch.empty((R, K), dtype=torch.uint8, device=x.device)
    sc = torch.empty(mx_scale_bytes(R, K), dtype=torch.uint8, device=x.device)
    _lib.check(_lib.lib().sse_mx_quantize(x.data_ptr(), R, K, role, q.data_ptr(), sc.data_ptr(),
                                          ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)),
               "sse_mx_quantize")
    return q, sc


def mx_quantize_host(x: np.ndarray, role: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """The host quantiser libsse.so applies to weights at sse_model_create (no GPU needed)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    R, K = x.shape
    q = np.empty((R, K), dtype=np.uint8)
    sc = np.empty(mx_scale_bytes(R, K), dtype=np.uint8)
    _lib.check(_lib.lib().sse_mx_quantize_host(x.ctypes.data, R, K, role, q.ctypes.data, sc.ctypes.data),
               "sse_mx_quantize_host")
    return q, sc


def gemm_mx(a_q: torch.Tensor, a_s: torch.Tensor, b_q: torch.Tensor, b_s: torch.Tensor, bias=None, resid=None,
            act: str | None = None, out: str = "fp32"):
    """MX-fp8 GEMM: dequant(a) [M, K] @ dequant(b)[N, K]^T (+bias) (gelu) (+resid).  out: "fp32",
    "bf16" or "fp8" (returns (e4m3 [M, N], scales in the A layout of a GEMM with K = N))."""
    M, K = a_q.shape
    N = b_q.shape[0]
    dev = a_q.device
    cf = torch.empty((M, N), dtype=torch.float32, device=dev) if out == "fp32" else None
    ct = None
    cs = None
    if out == "bf16":
        ct = torch.empty((M, N), dtype=torch.bfloat16, device=dev)
    elif out == "fp8":
        ct = torch.empty((M, N), dtype=torch.uint8, device=dev)
        cs = torch.empty(mx_scale_bytes(M, N), dtype=torch.uint8, device=dev)
    bias_p = bias.contiguous().data_ptr() if bias is not None else None
    res_p = resid.contiguous().data_ptr() if resid is not None else None
    _lib.check(_lib.lib().sse_gemm_mx(a_q.data_ptr(), a_s.data_ptr(), b_q.data_ptr(), b_s.data_ptr(), bias_p, res_p,
                                      cf.data_ptr() if cf is not None else None,
                                      ct.data_ptr() if ct is not None else None,
                                      cs.data_ptr() if cs is not None else None, M, N, K,
                                      {None: 0, "gelu": 1, "gelu_fast": 2}[act],
                                      ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "sse_gemm_mx")
    if out == "fp32":
        return cf
    return (ct, cs) if out == "fp8" else ct
