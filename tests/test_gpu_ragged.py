"""Ragged batches (sse_embed_ragged): clips of different lengths share one batch and each is
embedded at its own length, exactly as the reference embeds every file alone
(REF/WavLM_embeddings.py:284-307; REF/whisper_embeddings_large.py:242-254 pads to 30 s).

Properties: every clip of a ragged batch equals that clip run alone -- bit for bit when the batch's
longest clip selects the same WavLM attention kernel (all clips <= 160 frames, or all > 160), and
whatever the padding rows hold (random values are written past each clip's end); the fp32 path
matches the oracle at every length (rel-L2 <= 1e-4)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return np.linalg.norm(a - b, axis=-1) / np.linalg.norm(b, axis=-1)


def _batch(lens, seed, garbage=True):
    from ssr_amd import synth
    L = max(lens)
    rng = np.random.default_rng(seed)
    wave = (rng.standard_normal((len(lens), L)).astype(np.float32) * 3.0) if garbage else np.zeros((len(lens), L), np.float32)
    clips = [synth.synth_clips(1, n, seed=seed + i)[0] for i, n in enumerate(lens)]
    for i, c in enumerate(clips):
        wave[i, :len(c)] = c
    return torch.from_numpy(wave).cuda(), clips


@pytest.mark.parametrize("dtype", ["fp32", "bf16", "fp16x3", "fp16"])
@pytest.mark.parametrize("lens", [[48000, 400, 12345, 47999, 30000, 16000], [80000, 60000, 52000, 70001]])
def test_wavlm_ragged_equals_per_clip(wavlm_sd, dtype, lens):
    from ssr_amd import config as C
    from ssr_amd.model import SSEModel
    m = SSEModel(C.WAVLM_BASE, wavlm_sd, device="cuda:0", dtype=dtype)
    idx = [12, 11, 10, 6, 0]
    wave, clips = _batch(lens, 300)
    got = m.embed(wave, idx, lengths=lens)
    assert torch.isfinite(got).all()
    for i, c in enumerate(clips):
        one = m.embed(torch.from_numpy(c).cuda()[None], idx)
        assert torch.equal(got[i:i + 1], one), (dtype, i, lens[i])
    if dtype == "fp32":
        from oracle.wavlm import WavLMOracle
        o = WavLMOracle(C.WAVLM_BASE, wavlm_sd)
        for i in (0, 1, len(lens) - 1):
            ref = o.embed(clips[i], idx)
            assert _rel(got[i:i + 1].cpu().numpy(), ref).max() <= 1e-4


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
def test_wavlm_ragged_mixed_attention_paths(wavlm_sd, dtype):
    """Clips on both sides of the 160-frame attention split in one batch: each clip runs the attention
    kernel it runs alone (short-T kernel for <= 160 frames, flash kernel above), so every clip equals
    its per-clip call bit for bit."""
    from ssr_amd import config as C
    from ssr_amd.model import SSEModel
    m = SSEModel(C.WAVLM_BASE, wavlm_sd, device="cuda:0", dtype=dtype)
    lens = [48000, 80000, 3000, 51840, 51199, 160000]   # 149, 249, 9, 161, 159, 499 frames
    wave, clips = _batch(lens, 77)
    got = m.embed(wave, [12, 6], lengths=lens)
    for i, c in enumerate(clips):
        one = m.embed(torch.from_numpy(c).cuda()[None], [12, 6])
        assert torch.equal(got[i:i + 1], one), (i, lens[i])


def test_wavlm_ragged_normalize_and_embed_clips(wavlm_sd):
    """do_normalize statistics over each clip's own samples; embed_clips builds the padded batch."""
    from ssr_amd import config as C
    from ssr_amd.model import SSEModel
    m = SSEModel(C.WAVLM_BASE, wavlm_sd, device="cuda:0", dtype="fp32", do_normalize=True)
    lens = [20000, 48000, 9000]
    _, clips = _batch(lens, 12)
    got = m.embed_clips([torch.from_numpy(c) for c in clips], [12, 3])
    for i, c in enumerate(clips):
        assert torch.equal(got[i:i + 1], m.embed(torch.from_numpy(c).cuda()[None], [12, 3]))
    with pytest.raises(Exception):
        m.embed_clips([torch.zeros(300)], [12])


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_whisper_ragged_equals_per_clip(dtype):
    from ssr_amd import config as C, synth
    from ssr_amd.model import SSEModel
    m = SSEModel(C.WHISPER_TINY, synth.synth_whisper_state_dict(C.WHISPER_TINY, seed=11), device="cuda:0", dtype=dtype)
    lens = [16000, 48000, 7000]
    wave, clips = _batch(lens, 5)
    idx = [4, 3, 0]
    got = m.embed(wave, idx, lengths=lens)
    for i, c in enumerate(clips):
        assert torch.equal(got[i:i + 1], m.embed(torch.from_numpy(c).cuda()[None], idx)), i


def test_wavlm_ragged_c_abi_clamps_out_of_range_lengths(wavlm_sd):
    """the C-ABI clamps d_lengths on the device.  Called past the Python wrapper's checks
    with a length beyond the row (treated as the row), one under the 400-sample receptive field and a
    negative one (both pooled as zeros): no kernel reads outside its clip, every output is finite and
    the in-range clips are untouched."""
    import ctypes
    from ssr_amd import _lib, config as C, synth
    from ssr_amd.model import SSEModel
    m = SSEModel(C.WAVLM_BASE, wavlm_sd, device="cuda:0", dtype="bf16")
    L = 48000
    clips = synth.synth_clips(4, L, seed=41)
    wave = torch.from_numpy(clips).cuda()
    lens = torch.tensor([L, 10 * L, 200, -5], dtype=torch.int32, device="cuda")
    ids = torch.tensor([12, 6, 0], dtype=torch.int32)
    out = torch.full((4, 3, 768), float("nan"), device="cuda")
    ws = m.workspace(4, L)
    rc = _lib.lib().sse_embed_ragged(m._h, wave.data_ptr(), lens.data_ptr(), 4, L, ids.data_ptr(), 3, out.data_ptr(),
                                     ws.data_ptr(), ws.numel(), m._stream())
    assert rc == 0
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    full = m.embed(wave[:2], [12, 6, 0])
    assert torch.equal(out[0], full[0]) and torch.equal(out[1], full[1])
    assert (out[2:] == 0).all()


def test_whisper_ragged_c_abi_clamps_out_of_range_lengths():
    """the log-mel kernels clamp each ragged length to [0, min(L, 480000)], so a Whisper clip
    whose length exceeds its row reads only its row (the same as lens = L) and a negative length is
    silence (the same as an all-zero row)."""
    from ssr_amd import _lib, config as C, synth
    from ssr_amd.model import SSEModel
    m = SSEModel(C.WHISPER_TINY, synth.synth_whisper_state_dict(C.WHISPER_TINY, seed=11), device="cuda:0",
                 dtype="fp32")
    L = 32000
    wave = torch.from_numpy(synth.synth_clips(3, L, seed=43)).cuda()
    lens = torch.tensor([10 * L, -5, L // 2], dtype=torch.int32, device="cuda")
    ids = torch.tensor([C.WHISPER_TINY.layers, 0], dtype=torch.int32)
    out = torch.full((3, 2, C.WHISPER_TINY.hidden), float("nan"), device="cuda")
    ws = m.workspace(3, L)
    rc = _lib.lib().sse_embed_ragged(m._h, wave.data_ptr(), lens.data_ptr(), 3, L, ids.data_ptr(), 2, out.data_ptr(),
                                     ws.data_ptr(), ws.numel(), m._stream())
    assert rc == 0
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    ref = wave.clone()
    ref[1].zero_()
    ref[2, L // 2:].zero_()
    full = m.embed(ref, [C.WHISPER_TINY.layers, 0])
    assert torch.equal(out, full)
