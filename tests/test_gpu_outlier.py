"""Stress parity: heavy-tailed weights with outlier feature channels (synth.outlier_weights: four
LayerNorm channels x30 per LN, Student-t(3) projections), the shape real WavLM / Whisper
checkpoints have and the uniform synthetic weights do not.  Fixtures from the reference's own
glue (tests/golden/make_golden.py --only outlier).

Bars (stated here and in DESIGN.md "Parity bars"):
  fp32, fp16x3   rel-L2 <= 1e-4 (north star), as for the benign weights;
  bf16 (WavLM)   rel-L2 <= 0.25, cosine >= 0.97 -- FORMAT-bound: the same forward with ideal bf16
                 GEMM operands and fp32 accumulation (oracle/emulate.py) reaches rel-L2 0.226 /
                 cosine 0.9746 on these inputs (profiles/r2_emulate_outlier.json; 7.8e-3 on the
                 benign weights, where the bar stays 3e-2).  The unnormalised conv feature encoder
                 dominates; inputs like these need fp16x3 (observed 2.1e-5);
  bf16 (Whisper) rel-L2 <= 3e-2, cosine >= 0.999;  MX-fp8 rel-L2 <= 0.08, cosine >= 0.995."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return np.linalg.norm(a - b, axis=-1) / np.linalg.norm(b, axis=-1)


def _cos(a, b):
    return (a * b).sum(-1) / (np.linalg.norm(a, axis=-1) * np.linalg.norm(b, axis=-1))


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(GOLDEN, "outlier.npz"))


@pytest.mark.parametrize("dtype,tol,cos", [("fp32", 1e-4, 0.99999), ("fp16x3", 1e-4, 0.99999), ("bf16", 0.25, 0.97)])
def test_wavlm_outlier_weights(golden, dtype, tol, cos):
    from ssr_amd import config as C, synth
    from ssr_amd.model import SSEModel
    sd = synth.outlier_weights(synth.synth_wavlm_state_dict(C.WAVLM_BASE, seed=7))
    m = SSEModel(C.WAVLM_BASE, sd, device="cuda:0", dtype=dtype)
    clips = synth.synth_clips(4, 48000, seed=1234)
    got = m.embed(torch.from_numpy(clips).cuda(), [int(i) for i in golden["wavlm_layer_indices"]]).cpu().numpy()
    ref = golden["wavlm_emb"]
    print(dtype, "outlier WavLM-base rel-L2", _rel(got, ref).max(), "cos", _cos(got, ref).min())
    assert _rel(got, ref).max() <= tol and _cos(got, ref).min() >= cos


@pytest.mark.parametrize("dtype,tol,cos", [("fp32", 1e-4, 0.99999), ("bf16", 3e-2, 0.999), ("fp8", 0.08, 0.995)])
def test_whisper_outlier_weights(golden, dtype, tol, cos):
    from ssr_amd import config as C, synth
    from ssr_amd.model import SSEModel
    spec = C.WhisperSpec(d_model=512, layers=3, heads=8, ffn=2048, name="whisper-mx-test")
    sd = synth.outlier_weights(synth.synth_whisper_state_dict(spec, seed=21))
    m = SSEModel(spec, sd, device="cuda:0", dtype=dtype)
    clips = synth.synth_clips(2, 48000, seed=99)
    got = m.embed(torch.from_numpy(clips).cuda(), [int(i) for i in golden["whisper_layer_indices"]]).cpu().numpy()
    ref = golden["whisper_emb"]
    print(dtype, "outlier Whisper rel-L2", _rel(got, ref).max(), "cos", _cos(got, ref).min())
    assert _rel(got, ref).max() <= tol and _cos(got, ref).min() >= cos


def test_wavlm_outlier_bf16_residual_cost_measured(golden):
    """the bf16 residual stream + folded LayerNorm (the production bf16 flow) and the
    materialised flow (no_lnfold=1: LayerNorm kernels, fp32 residual) both measured against the
    reference's outlier fixture every run, so the accuracy cost of the bf16 stream stays visible;
    the production flow may not be worse than the fp32-residual one by more than the format's noise."""
    from ssr_amd import _lib, config as C, synth
    from ssr_amd.model import SSEModel
    sd = synth.outlier_weights(synth.synth_wavlm_state_dict(C.WAVLM_BASE, seed=7))
    m = SSEModel(C.WAVLM_BASE, sd, device="cuda:0", dtype="bf16")
    clips = torch.from_numpy(synth.synth_clips(4, 48000, seed=1234)).cuda()
    idx = [int(i) for i in golden["wavlm_layer_indices"]]
    ref = golden["wavlm_emb"]
    a = m.embed(clips, idx).cpu().numpy()
    with _lib.option("no_lnfold", 1):
        b = m.embed(clips, idx).cpu().numpy()
    ea, eb = _rel(a, ref).max(), _rel(b, ref).max()
    print("outlier bf16: bf16 residual + folded LN", ea, "| fp32 residual, materialised LN", eb)
    assert ea <= 0.25 and eb <= 0.25 and ea <= 1.25 * eb + 0.02
