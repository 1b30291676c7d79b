"""The head-pipelined short-T attention kernels (kernels_misc.hip: attention_pipe_kernel, double-buffered, one block
per CU, option attn_short = 0, the default; attention_pipe2_kernel, two blocks per CU, attn_short = 2, round 6) against
the one-head-at-a-time kernel (attention_full_kernel, attn_short = 1): per wave the
same fragments, the same softmax order and the same MFMA chain, so the embeddings must agree bit for
bit -- at batch sizes that select 1, 3, 6 and 12 heads per block (the double-buffered head loop),
at 49 and 149 frames (4 and 10 key blocks), on ragged batches (per-clip masks, long clips left to
the flash kernel) and for both 16-bit operand types.  Reference semantics: the WavLM self-attention
with gated relative position bias (REF/WavLM_embeddings.py:267-341 -> transformers WavLMAttention)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _batch(lens, seed):
    from ssr_amd import synth
    rng = np.random.default_rng(seed)
    wave = rng.standard_normal((len(lens), max(lens))).astype(np.float32) * 3.0   # garbage past each end
    clips = [synth.synth_clips(1, n, seed=seed + i)[0] for i, n in enumerate(lens)]
    for i, c in enumerate(clips):
        wave[i, :len(c)] = c
    return torch.from_numpy(wave).cuda(), clips


def _both(m, w, idx, mode, **kw):
    from ssr_amd import _lib
    with _lib.option("attn_short", 1):
        a = m.embed(w, idx, **kw)
    with _lib.option("attn_short", mode):
        b = m.embed(w, idx, **kw)
    return a, b


@pytest.mark.parametrize("mode", [0, 2])
@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
@pytest.mark.parametrize("n_clips,samples", [(6, 48000), (48, 48000), (128, 48000), (256, 48000), (5, 16000),
                                             (40, 16000)])
def test_attention_pipe_bit_identical(wavlm_sd, mode, dtype, n_clips, samples):
    from ssr_amd import config as C, synth
    from ssr_amd.model import SSEModel
    m = SSEModel(C.WAVLM_BASE, wavlm_sd, device="cuda:0", dtype=dtype)
    w = torch.from_numpy(synth.synth_clips(min(n_clips, 16), samples, seed=31)).cuda()
    if n_clips > 16:   # distinct clips in every position (a different gain per copy)
        reps = (n_clips + 15) // 16
        gains = torch.linspace(0.5, 1.5, reps * 16, device="cuda:0")[:n_clips, None]
        w = w.repeat(reps, 1)[:n_clips] * gains
    a, b = _both(m, w, list(range(13)), mode)
    assert torch.isfinite(a).all()
    assert torch.equal(a, b)


@pytest.mark.parametrize("mode", [0, 2])
@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
def test_attention_pipe_ragged(wavlm_sd, mode, dtype):
    from ssr_amd import config as C
    from ssr_amd.model import SSEModel
    m = SSEModel(C.WAVLM_BASE, wavlm_sd, device="cuda:0", dtype=dtype)
    for lens in ([48000, 400, 12345, 47999, 30000, 16000], [48000, 80000, 3000, 51840, 51199, 160000]):
        wave, clips = _batch(lens, 91)
        a, b = _both(m, wave, [12, 6, 0], mode, lengths=lens)
        assert torch.equal(a, b), lens
        # and each clip still equals its solo call on the pipelined kernel
        from ssr_amd import _lib
        with _lib.option("attn_short", mode):
            for i in (0, 2):
                one = m.embed(torch.from_numpy(clips[i]).cuda()[None], [12, 6, 0])
                assert torch.equal(b[i:i + 1], one), (lens, i)
