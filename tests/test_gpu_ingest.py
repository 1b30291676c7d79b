"""GPU parity of the ingest row: sse_mono / sse_resample against the
numpy restatement of torchaudio's default resampler (oracle/resample.py; parity against
torchaudio itself is unpinned — it is absent from this image).  Tolerance: max abs error
<= 2e-6 on O(0.5) signals (the GPU sums the ~475 taps in fp32 with MFMA, the oracle in fp64)."""
import numpy as np
import pytest
import torch

from test_wavio import write_wav

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sr", [44100, 48000, 22050, 8000, 32000, 11025])
def test_resample_matches_oracle(sr):
    from oracle.resample import resample as ref
    from ssr_amd.ingest import resample
    rng = np.random.default_rng(sr)
    for L in (5, sr // 3 + 17, 3 * sr):
        x = (0.5 * rng.standard_normal((3, L))).astype(np.float32)
        got = resample(torch.from_numpy(x).cuda(), sr, 16000).cpu().numpy()
        want = ref(x, sr, 16000)
        assert got.shape == want.shape
        err = np.abs(got - want).max()
        print(sr, L, "max abs err", err)
        assert err <= 2e-6


def test_resample_identity_and_mono():
    from oracle.resample import mono as ref_mono
    from ssr_amd.ingest import mono, resample
    x = torch.randn(2, 1000, device="cuda")
    assert torch.equal(resample(x, 16000, 16000), x)
    s = np.random.default_rng(0).standard_normal((2, 3, 777)).astype(np.float32)
    got = mono(torch.from_numpy(s).cuda()).cpu().numpy()
    for b in range(2):
        assert np.array_equal(got[b], ref_mono(s[b]))


def test_load_audio_stereo_44k1(tmp_path):
    """load_audio: stereo 44.1 kHz PCM -> mono -> 16 kHz -> trim, as REF/WavLM_embeddings.py:87-125."""
    from oracle.resample import mono, resample
    from ssr_amd.extract import load_audio, read_wav
    rng = np.random.default_rng(7)
    x = (0.3 * rng.standard_normal((2, 44100 * 2))).astype(np.float32)
    p = str(tmp_path / "s.wav")
    write_wav(p, x, sr=44100, fmt="pcm16")
    pcm, sr = read_wav(p)
    want = resample(mono(pcm), 44100, 16000)[:16000]
    got = load_audio(p, max_length=1.0, device="cuda:0")
    assert got.shape == (16000,) and np.abs(got - want).max() <= 2e-6


def test_extract_from_44k1_file_matches_16k_embedding(tmp_path):
    """End to end: a 44.1 kHz file through extract_wavlm_embeddings equals embedding the
    oracle-resampled clip directly (fp32 path, 1e-4)."""
    from oracle.resample import resample
    from ssr_amd import config as C, synth
    from ssr_amd.extract import extract_wavlm_embeddings
    from ssr_amd.hf import Wav2Vec2FeatureExtractor, WavLMModel
    clip = synth.synth_clips(1, 44100 * 2, seed=3)[0]
    p = str(tmp_path / "c.wav")
    write_wav(p, clip, sr=44100, fmt="float")
    model = WavLMModel.from_state_dict(C.WAVLM_BASE, synth.synth_wavlm_state_dict(C.WAVLM_BASE), "cuda:0", "fp32")
    fe = Wav2Vec2FeatureExtractor(do_normalize=False, device="cuda:0")
    d = extract_wavlm_embeddings(p, model, fe, "cuda:0", [12, 6])
    ref = model.embed(torch.from_numpy(resample(clip, 44100, 16000)).cuda(), [12, 6]).cpu().numpy()[0]
    for j, k in enumerate((12, 6)):
        v = d[f"layer_{k}"]
        assert np.linalg.norm(v - ref[j]) / np.linalg.norm(ref[j]) <= 1e-4
