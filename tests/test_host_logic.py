"""Host-side logic that needs no GPU: the augmentation driver's error classification (which
failures a per-clip retry may swallow) and its length-sorted ragged batching."""
import importlib

import pytest
import torch

importlib.import_module("stuttering-speech-representation_amd")


def test_recoverable_errors_only():
    from ssr_amd._lib import SSEError, SSEOutOfMemoryError
    from ssr_amd.augment import _per_clip_fallback, _recoverable
    assert _recoverable(SSEOutOfMemoryError(-6, "x")) and _recoverable(SSEError(-1, "x"))
    assert _recoverable(ValueError("short")) and _recoverable(SSEError(-3, "x"))
    assert not _recoverable(SSEError(-2, "hip fault")) and not _recoverable(RuntimeError("x"))

    def bad_clip(part):                    # clip 1 is invalid: the batch fails, the others survive
        if 1 in part:
            raise SSEError(-1, "too short")
        return [f"e{j}" for j in part]
    assert _per_clip_fallback(bad_clip, [0, 1, 2]) == ["e0", None, "e2"]

    from ssr_amd._lib import SSERangeError
    assert _recoverable(SSERangeError(-7, "fp16 overflow"))

    def overflow_clip(part):               # an fp16 overflow of clip 2 drops only clip 2
        if 2 in part:
            raise SSERangeError(-7, "non-finite output")
        return [f"e{j}" for j in part]
    assert _per_clip_fallback(overflow_clip, [0, 1, 2, 3]) == ["e0", "e1", None, "e3"]

    def dead_gpu(part):                    # a HIP failure is not swallowed clip by clip
        raise SSEError(-2, "hip error")
    with pytest.raises(SSEError):
        _per_clip_fallback(dead_gpu, [0, 1, 2])


def test_length_sorted_batches_cover_every_clip_once():
    from ssr_amd.augment import _length_sorted_batches
    clips = [torch.zeros(n) for n in (500, 48000, 16000, 700, 16000, 30000, 9000)]
    parts = _length_sorted_batches(clips, 3)
    assert sorted(j for p in parts for j in p) == list(range(len(clips)))
    assert [len(p) for p in parts] == [3, 3, 1]
    flat = [clips[j].shape[0] for p in parts for j in p]
    assert flat == sorted(flat)
