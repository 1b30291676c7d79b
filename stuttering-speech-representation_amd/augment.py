"""Batched augmentation re-extraction.

Drop-in for the reference's ``augment_audio`` / ``apply_data_augmentation``
(REF/model_training_1.py:167-214, 318-464; variant REF/model_training_01.py:140-192, 290-388):

* Random choices and factors are drawn with Python's ``random`` in exactly the reference's call
  order (``random.choice`` of the kind, then ``random.uniform`` / ``random.randint`` for its
  factor), so a seeded run picks the same augmentation per clip.
* The signal work runs on the GPU and is batched: speed = torchaudio-default resampling
  16 kHz -> int(16000*f) -> 16 kHz (``sse_resample``); noise / volume / clamp in one
  ``sse_augment`` launch per equal-length group.  Noise samples come from the build's
  counter-hash Gaussian (``synth.gaussian`` stream), not torch's CPU generator: same
  distribution, reproducible on any device, different sample values than ``torch.randn_like``.
* The augmented clips are embedded in batches (grouped by length) through the fused path,
  and ``apply_data_augmentation(..., cache=dict)`` computes every requested layer once and
  reuses it across the reference's per-layer loop (REF/model_training_1.py:920-940 recomputes
  all augmentations for every layer).
* Pitch shift (model_training_01 only, REF/model_training_01.py:172-177): torchaudio
  PitchShift's STFT -> phase vocoder -> iSTFT -> resample on the GPU (``sse_pitch_shift``,
  kernels_pitch.hip), then the clamp.  Clips of 256 samples or fewer make torch.stft's reflect
  padding raise in the reference; here too, and augment_audio returns the original clip.
"""
from __future__ import annotations

import ctypes
import logging
import os
import random as _random
from dataclasses import dataclass

import numpy as np
import pandas as pd
import torch

from . import _lib
from .ingest import resample

logger = logging.getLogger(__name__)

KIND_CODE = {"none": 0, "noise": 1, "volume": 2, "clamp": 3}
VARIANTS = {
    # REF/model_training_1.py:179-205
    "1": {"choices": ["speed", "noise", "volume", "none"], "speed": (0.95, 1.05), "noise": (0.001, 0.005),
          "volume": (0.9, 1.1)},
    # REF/model_training_01.py:153-181
    "01": {"choices": ["speed", "noise", "pitch", "volume"], "speed": (0.9, 1.1), "noise": (0.005, 0.02),
           "volume": (0.8, 1.2), "pitch": (-2, 2)},
}

# (augmentation_factor, minority_threshold) defaults of each reference variant's apply_data_augmentation
VARIANT_DEFAULTS = {"1": (2, 200), "01": (3, 100)}


@dataclass
class AugSpec:
    kind: str
    factor: float = 1.0
    new_sr: int = 0
    n_steps: int = 0


def draw(rng=_random, variant: str = "1", augmentation_type: str = "random", sample_rate: int = 16000) -> AugSpec:
    """The random draws of augment_audio, in its order."""
    v = VARIANTS[variant]
    t = rng.choice(v["choices"]) if augmentation_type == "random" else augmentation_type
    if t == "speed":
        f = rng.uniform(*v["speed"])
        return AugSpec("speed", f, new_sr=int(sample_rate * f))
    if t in ("noise", "volume"):
        return AugSpec(t, rng.uniform(*v[t]))
    if t == "pitch":
        return AugSpec("pitch", n_steps=rng.randint(*v["pitch"]))
    return AugSpec("none")


def _pointwise(x: torch.Tensor, kinds, factors, streams, seed: int) -> torch.Tensor:
    """x [B, L] cuda -> clamp(op(x)) via sse_augment."""
    B, L = x.shape
    dev = x.device
    k = torch.tensor(kinds, dtype=torch.int32).to(dev)
    f = torch.tensor(factors, dtype=torch.float32).to(dev)
    s = torch.tensor(streams, dtype=torch.int64).to(dev)
    y = torch.empty_like(x)
    _lib.check(_lib.lib().sse_augment(x.data_ptr(), y.data_ptr(), B, L, k.data_ptr(), f.data_ptr(), s.data_ptr(),
                                      ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF),
                                      ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "sse_augment")
    return y


def pitch_shift(x: torch.Tensor, sample_rate: int, n_steps: int) -> torch.Tensor:
    """torchaudio.transforms.PitchShift(sample_rate, n_steps)(x) on the GPU: [L] or [B, L] fp32
    cuda -> the same shape (no clamp).  Raises SSEError for L <= 256 (torch.stft's reflect pad)."""
    if x.device.type != "cuda":
        raise ValueError("pitch_shift runs on a GPU device (no CPU fallback)")
    squeeze = x.dim() == 1
    x = (x[None] if squeeze else x).to(torch.float32).contiguous()
    B, L = x.shape
    lib = _lib.lib()
    n = lib.sse_pitch_shift_workspace_bytes(B, L, int(sample_rate), int(n_steps))
    ws = torch.empty(max(n, 256), dtype=torch.uint8, device=x.device)
    y = torch.empty_like(x)
    _lib.check(lib.sse_pitch_shift(x.data_ptr(), B, L, int(sample_rate), int(n_steps), y.data_ptr(), ws.data_ptr(),
                                   ws.numel(), ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)),
               "sse_pitch_shift")
    return y[0] if squeeze else y


def augment_batch(waves, specs, seed: int = 0, streams=None, sample_rate: int = 16000) -> list:
    """Apply ``specs[i]`` to ``waves[i]`` (1-D float32 cuda tensors, any lengths) on the GPU.
    Returns a list of 1-D tensors (speed changes the length by at most a sample or two)."""
    n = len(waves)
    streams = list(range(n)) if streams is None else list(streams)
    out = [None] * n
    groups = {}
    for i, (w, sp) in enumerate(zip(waves, specs)):
        if sp.kind == "pitch" and sp.n_steps == 0:   # REF: `if n_steps != 0` -> unchanged, then clamp
            sp = AugSpec("none")
        if sp.kind == "speed":
            w = resample(resample(w, sample_rate, sp.new_sr), sp.new_sr, sample_rate)
            kind, fac = "clamp", 1.0
        elif sp.kind == "pitch":
            w = pitch_shift(w, sample_rate, sp.n_steps)
            kind, fac = "clamp", 1.0
        else:
            kind, fac = sp.kind, sp.factor
        groups.setdefault((int(w.shape[-1]), str(w.device)), []).append((i, w, KIND_CODE[kind], fac))
    for items in groups.values():
        x = torch.stack([w.to(torch.float32) for _, w, _, _ in items])
        y = _pointwise(x, [k for _, _, k, _ in items], [f for _, _, _, f in items],
                       [streams[i] for i, _, _, _ in items], seed)
        for j, (i, _, _, _) in enumerate(items):
            out[i] = y[j]
    return out


def augment_audio(waveform, sample_rate=16000, augmentation_type="random", *, rng=_random, variant="1", seed=0,
                  stream=0, device=None):
    """REF/model_training_1.py:167-214 twin: numpy (or tensor) in, float32 numpy out; any failure
    logs a warning and returns the input, as the reference does."""
    x = torch.as_tensor(np.asarray(waveform, dtype=np.float32)).reshape(-1)
    try:
        spec = draw(rng, variant, augmentation_type, sample_rate)
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        return augment_batch([x.to(dev)], [spec], seed, [stream], sample_rate)[0].cpu().numpy()
    except Exception as e:
        logger.warning(f"Augmentation failed: {e}. Returning original audio.")
        return x.numpy()


def _recoverable(e: BaseException) -> bool:
    """Errors one clip can cause and a per-clip retry can get past: out of memory, an invalid clip
    (shorter than the receptive field: SSE_ERR_INVALID, or the wrapper's ValueError) or a shape the
    kernels do not cover.  A HIP runtime failure (SSE_ERR_HIP: a fault or a sticky context error)
    and anything unexpected are NOT: after those every clip would fail again, so they propagate
    instead of silently dropping every augmented sample.  An fp16-range overflow
    (SSERangeError, fp16 / fp16x3 models) is one clip's property: the range flag is cleared when it is
    read, so the per-clip retry finds the offending clip and skips only it."""
    from ._lib import SSEError, SSEOutOfMemoryError, SSERangeError
    if isinstance(e, (SSEOutOfMemoryError, SSERangeError, torch.OutOfMemoryError, ValueError)):
        return True
    return isinstance(e, SSEError) and e.rc in (-1, -3, -4)


def _per_clip_fallback(run, part):
    """run(part) -> one result per clip.  A batch failing with a recoverable error (a clip shorter
    than the receptive field, OOM, ...) is retried one clip at a time; a clip that still fails gets
    None and is skipped, as the reference's per-sample try/except does
    (REF/model_training_1.py:379-419).  Unrecoverable errors propagate."""
    try:
        return run(part)
    except Exception as e:
        if not _recoverable(e):
            raise
        if len(part) == 1:
            logger.warning(f"Error extracting embeddings from augmented audio: {e}")
            return [None]
        logger.warning(f"Batched embedding of {len(part)} augmented clips failed ({e}); retrying one at a time")
        return [r for j in part for r in _per_clip_fallback(run, [j])]


def _length_sorted_batches(audios, batch):
    """Ragged batches of up to `batch` clips, clips sorted by length so a batch's padding stays
    small: every clip of any length shares a batch (sse_embed_ragged embeds each at its own length)
    instead of one batch per exact length."""
    order = sorted(range(len(audios)), key=lambda j: int(audios[j].shape[-1]))
    return [order[c:c + batch] for c in range(0, len(order), batch)]


def _embed_jobs(audios, model, feature_extractor, device, layer_names, model_type, batch):
    """Embed a list of 1-D cuda clips -> list of {layer_name: float32[H]} (None on failure)."""
    from .extract import extract_embeddings_from_audio_wavlm, extract_embeddings_from_audio_whisper
    from .hf import WavLMModel, WhisperModel
    out = [None] * len(audios)
    mt = model_type.lower()
    if mt in ("wavlm", "wavlm_large"):
        idx = [int(n.split("_")[1]) for n in layer_names if n.startswith("layer_")]
        if isinstance(model, WavLMModel):
            n_hs = model.sse.spec.layers + 1
            valid = [i for i in idx if i < n_hs]
            if not valid:                      # no requested layer exists: {} per clip (REF :259-264)
                return [{} for _ in audios]

            def run(part):
                # the feature extractor per clip (its normalisation statistics cover that clip only,
                # like the reference's batch-1 call), then one ragged batch
                xs = [feature_extractor(audios[j], sampling_rate=16000, return_tensors="pt").to(device)
                      .input_values[0] for j in part]
                e = model.sse.embed_clips(xs, valid).cpu().numpy()
                return [{f"layer_{i}": e[r, q].copy() for q, i in enumerate(valid)} for r in range(len(part))]

            for part in _length_sorted_batches(audios, batch):
                for j, r in zip(part, _per_clip_fallback(run, part)):
                    out[j] = r
            return out
        for j, a in enumerate(audios):
            out[j] = extract_embeddings_from_audio_wavlm(a.cpu().numpy(), model, feature_extractor, device, idx)
        return out
    if mt in ("whisper", "whisper_large_fixed"):
        if isinstance(model, WhisperModel):
            spec = model.sse.spec
            enc = [int(n.split("_")[-1]) for n in layer_names if n.startswith("encoder_layer_")]
            dec = [int(n.split("_")[-1]) for n in layer_names if n.startswith("decoder_layer_")]
            enc = [i for i in enc if i < spec.layers + 1]
            dec = [i for i in dec if i < spec.decoder_layers + 1] if spec.decoder_layers else []
            if not enc and not dec:
                return [{} for _ in audios]

            def run(part):
                # Whisper pads every clip to 30 s (the feature extractor does): a zero-padded batch
                # is the ragged batch
                L = max(int(audios[j].shape[-1]) for j in part)
                x = torch.zeros((len(part), L), dtype=torch.float32, device=model.sse.device)
                for r, j in enumerate(part):
                    x[r, :audios[j].shape[-1]] = audios[j]
                e, d = model.sse.whisper_embed(x, enc, dec)
                e, d = e.cpu().numpy(), d.cpu().numpy()
                res = []
                for r in range(len(part)):
                    x = {f"encoder_layer_{i}": e[r, q].copy() for q, i in enumerate(enc)}
                    x.update({f"decoder_layer_{i}": d[r, q].copy() for q, i in enumerate(dec)})
                    res.append(x)
                return res

            for part in _length_sorted_batches(audios, batch):
                for j, r in zip(part, _per_clip_fallback(run, part)):
                    out[j] = r
            return out
        for j, a in enumerate(audios):
            out[j] = extract_embeddings_from_audio_whisper(a.cpu().numpy(), model, feature_extractor, device,
                                                           layer_names)
        return out
    logger.warning(f"Unsupported model type for augmentation: {model_type}")
    return out


def apply_data_augmentation(train_meta, train_embeddings, model, feature_extractor, device, layer_names, model_type,
                            augmentation_factor=None, minority_threshold=None, *, rng=_random, variant="1", seed=0,
                            batch=64, cache=None):
    """REF/model_training_1.py:318-464 twin, batched on the GPU.  ``cache`` (a dict) hoists the
    work out of the caller's per-layer loop: the first call augments and embeds every layer in
    ``layer_names`` once; later calls with the same clips reuse it (no further random draws)."""
    from .extract import load_audio
    # per-variant defaults: REF/model_training_1.py:319 (2, 200), REF/model_training_01.py:291 (3, 100)
    d_factor, d_thresh = VARIANT_DEFAULTS[variant]
    augmentation_factor = d_factor if augmentation_factor is None else augmentation_factor
    minority_threshold = d_thresh if minority_threshold is None else minority_threshold
    logger.info("\n=== Applying Data Augmentation ===")
    if "path" not in train_meta.columns:
        logger.warning("No audio file paths found. Skipping data augmentation.")
        return train_meta, train_embeddings
    if "label" not in train_meta.columns:
        logger.warning("No labels found. Skipping data augmentation.")
        return train_meta, train_embeddings
    class_counts = train_meta["label"].value_counts()
    minority = class_counts[class_counts < minority_threshold].index.tolist()
    logger.info(f"Classes to augment (< {minority_threshold} samples): {minority}")
    if not minority:
        logger.info("No minority classes found. Skipping augmentation.")
        return train_meta, train_embeddings

    key = (tuple(train_meta["path"].tolist()), tuple(train_meta["label"].tolist()), int(augmentation_factor),
           int(minority_threshold), variant, int(seed), tuple(layer_names), model_type)
    if cache is not None and key in cache:
        aug_rows, aug_embs = cache[key]
    else:
        jobs, audios, specs = [], [], []
        for cls in minority:
            for _, row in train_meta[train_meta["label"] == cls].iterrows():
                if not os.path.exists(row["path"]):
                    logger.warning(f"Audio file not found: {row['path']}")
                    continue
                audio = load_audio(row["path"], device=device)
                if audio is None:
                    continue
                a = torch.from_numpy(audio).to(device)
                for aug_idx in range(augmentation_factor):
                    spec = draw(rng, variant)
                    jobs.append((row, aug_idx))
                    audios.append(a)
                    specs.append(spec)
        aug_audio = []
        for j, (a, sp) in enumerate(zip(audios, specs)):
            try:
                aug_audio.append(augment_batch([a], [sp], seed, [j])[0] if sp.kind in ("speed", "pitch") else None)
            except Exception as e:
                logger.warning(f"Augmentation failed: {e}. Returning original audio.")
                aug_audio.append(a)
        # pointwise kinds batched in one launch per length group
        pw = [j for j, x in enumerate(aug_audio) if x is None]
        if pw:
            res = augment_batch([audios[j] for j in pw], [specs[j] for j in pw], seed, pw)
            for j, y in zip(pw, res):
                aug_audio[j] = y
        embs = _embed_jobs(aug_audio, model, feature_extractor, device, layer_names, model_type, batch)
        aug_rows, aug_embs = [], []
        for (row, aug_idx), e in zip(jobs, embs):
            if e is None:
                continue
            m = row.copy()
            m["filename"] = f"{row['filename']}_aug_{aug_idx}"
            m["augmented"] = True
            m["augmentation_type"] = "mixed"
            aug_rows.append(m)
            aug_embs.append(e)
        if cache is not None:
            cache[key] = (aug_rows, aug_embs)

    if not aug_rows:
        logger.warning("No augmented samples were created.")
        return train_meta, train_embeddings
    combined_meta = pd.concat([train_meta, pd.DataFrame(aug_rows)], ignore_index=True)
    combined = {}
    for name, orig in train_embeddings.items():
        extra = [e[name] for e in aug_embs if name in e]
        combined[name] = np.vstack([orig, np.array(extra)]) if extra else orig
        logger.info(f"Combined {name}: {orig.shape[0]} original + {len(extra)} augmented = {combined[name].shape[0]}")
    logger.info(f"Data augmentation complete: {len(train_meta)} → {len(combined_meta)} samples")
    return combined_meta, combined
