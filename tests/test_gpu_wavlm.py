"""GPU parity of the WavLM hot path (libsse.so HIP kernels) against the reference's own
outputs (golden fixtures from REF/WavLM_embeddings.py:extract_wavlm_embeddings) and the
numpy oracle.

Tolerances (written here, stated in DESIGN.md):
  fp32 path: max rel-L2 per pooled vector <= 1e-4 (north star), per hidden state <= 1e-4.
  bf16 path: max rel-L2 per pooled vector <= 3e-2 and min cosine >= 0.999.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

FP32_TOL = 1e-4
BF16_TOL = 3e-2
BF16_COS = 0.999


def _rel(a, b):
    return np.linalg.norm(a - b, axis=-1) / np.linalg.norm(b, axis=-1)


def _cos(a, b):
    return (a * b).sum(-1) / (np.linalg.norm(a, axis=-1) * np.linalg.norm(b, axis=-1))


@pytest.fixture(scope="module")
def m32(wavlm_sd):
    from ssr_amd import config as C
    from ssr_amd.model import SSEModel
    return SSEModel(C.WAVLM_BASE, wavlm_sd, device="cuda:0", dtype="fp32")


@pytest.fixture(scope="module")
def m16(wavlm_sd):
    from ssr_amd import config as C
    from ssr_amd.model import SSEModel
    return SSEModel(C.WAVLM_BASE, wavlm_sd, device="cuda:0", dtype="bf16")


def test_fp32_embed_matches_reference(m32, wavlm_clips, golden_wavlm):
    idx = [int(i) for i in golden_wavlm["layer_indices"]]
    got = m32.embed(torch.from_numpy(wavlm_clips).cuda(), idx).cpu().numpy()
    ref = golden_wavlm["emb_norm0"]
    rel = _rel(got, ref)
    print("fp32 max rel-L2", rel.max())
    assert rel.max() <= FP32_TOL


def test_bf16_embed_matches_reference(m16, wavlm_clips, golden_wavlm):
    idx = [int(i) for i in golden_wavlm["layer_indices"]]
    got = m16.embed(torch.from_numpy(wavlm_clips).cuda(), idx).cpu().numpy()
    ref = golden_wavlm["emb_norm0"]
    rel, cos = _rel(got, ref), _cos(got, ref)
    print("bf16 max rel-L2", rel.max(), "min cos", cos.min())
    assert rel.max() <= BF16_TOL and cos.min() >= BF16_COS


def test_fp32_all_hidden_states(m32, wavlm_clips, golden_wavlm):
    hs = m32.hidden_states(torch.from_numpy(wavlm_clips[:2]).cuda())
    assert len(hs) == 13
    pooled = torch.stack([h.mean(dim=1) for h in hs], dim=1).cpu().numpy()   # [2, 13, 768]
    rel = _rel(pooled, golden_wavlm["emb_all_layers"])
    assert rel.max() <= FP32_TOL, rel.max()
    h0 = hs[0][0].cpu().numpy()
    assert np.linalg.norm(h0 - golden_wavlm["hs0_clip0"]) / np.linalg.norm(golden_wavlm["hs0_clip0"]) <= FP32_TOL
    h1 = hs[1][0].cpu().numpy()
    assert np.linalg.norm(h1 - golden_wavlm["hs1_clip0"]) / np.linalg.norm(golden_wavlm["hs1_clip0"]) <= FP32_TOL


def test_fp32_do_normalize(wavlm_sd, wavlm_clips, golden_wavlm):
    from ssr_amd import config as C
    from ssr_amd.model import SSEModel
    m = SSEModel(C.WAVLM_BASE, wavlm_sd, device="cuda:0", dtype="fp32", do_normalize=True)
    idx = [int(i) for i in golden_wavlm["layer_indices"]]
    got = m.embed(torch.from_numpy(wavlm_clips[:4]).cuda(), idx).cpu().numpy()
    assert _rel(got, golden_wavlm["emb_norm1"]).max() <= FP32_TOL


def test_batch_invariance_full_batch(m16, m32):
    """Size-independent property at the bench shape (B=256): every clip's embedding in the
    batch equals the embedding of that clip run alone, bit for bit (no cross-clip reduction, and no
    dependence on where a clip's rows fall inside the GEMM tiles: the library is built without
    implicit FMA contraction, see the Makefile).  bf16: all 256 clips; fp32: every 8th."""
    from ssr_amd import synth
    clips = torch.from_numpy(synth.synth_clips(256, 48000, seed=99)).cuda()
    idx = [12, 11, 10, 6]
    for m in (m16, m32):
        full = m.embed(clips, idx)
        for i in (range(256) if m is m16 else range(0, 256, 8)):
            one = m.embed(clips[i:i + 1], idx)
            assert torch.equal(full[i:i + 1], one), (m.dtype, i)
        assert torch.isfinite(full).all()


def test_oracle_subset_at_full_batch(m32):
    """Full-size run, a subset of clips checked against the numpy oracle."""
    from oracle.wavlm import WavLMOracle
    from ssr_amd import config as C, synth
    sd = synth.synth_wavlm_state_dict(C.WAVLM_BASE, seed=7)
    clips = synth.synth_clips(256, 48000, seed=5)
    idx = [12, 11, 10, 6]
    got = m32.embed(torch.from_numpy(clips).cuda(), idx).cpu().numpy()
    o = WavLMOracle(C.WAVLM_BASE, sd)
    sel = [3, 128, 250]
    ref = o.embed(clips[sel], idx)
    assert _rel(got[sel], ref).max() <= FP32_TOL


def test_edge_lengths(m32, wavlm_sd):
    """Ragged clip lengths: shortest valid clip (T=1 frame), odd lengths, 10 s clip."""
    from oracle.wavlm import WavLMOracle
    from ssr_amd import config as C, synth
    o = WavLMOracle(C.WAVLM_BASE, wavlm_sd)
    for L in (400, 12345, 160000):
        clip = synth.synth_clips(1, L, seed=L)
        got = m32.embed(torch.from_numpy(clip).cuda(), [12, 6, 0]).cpu().numpy()
        ref = o.embed(clip, [12, 6, 0])
        assert _rel(got, ref).max() <= FP32_TOL, L
    with pytest.raises(Exception):
        m32.embed(torch.zeros((1, 399), device="cuda:0"), [12])    # shorter than the receptive field (T = 0)


@pytest.mark.parametrize("dtype,tol", [("fp32", FP32_TOL), ("bf16", BF16_TOL), ("fp16", 5e-3), ("fp16x3", FP32_TOL)])
def test_wavlm_large_matches_reference(dtype, tol):
    """WavLM-large shape (layer-norm conv frontend, stable-LN encoder, do_normalize=True), the
    reference's default --model_name (REF/WavLM_embeddings.py:34).  fp16x3 (split-fp16 GEMMs) holds the
    fp32 bar, 1e-4."""
    import os
    from conftest import GOLDEN
    from ssr_amd import config as C, synth
    from ssr_amd.model import SSEModel
    g = np.load(os.path.join(GOLDEN, "wavlm_large.npz"))
    m = SSEModel(C.WAVLM_LARGE, synth.synth_wavlm_state_dict(C.WAVLM_LARGE, seed=9), device="cuda:0", dtype=dtype,
                 do_normalize=True)
    clips = synth.synth_clips(3, 48000, seed=77)
    got = m.embed(torch.from_numpy(clips).cuda(), [int(i) for i in g["layer_indices"]]).cpu().numpy()
    rel = _rel(got, g["emb"])
    print(dtype, "wavlm-large rel", rel.max())
    assert rel.max() <= tol and _cos(got, g["emb"]).min() >= BF16_COS


def test_bf16_lnfold_matches_materialised(wavlm_sd):
    """The bf16 post-LN path runs no LayerNorm kernel inside the layer loop: oproj / ffn2 write the
    un-normalised sum in bf16 (at once the next residual and the next GEMM's A operand; no fp32
    stream) and per-256-column partial statistics of the rounded values;
    QKV / FFN1 apply the LayerNorm through folded weights (rstd (acc - mean acol) + b'), the next
    residual GEMM on its residual load, the pool on its loads.  Against the materialised flow
    (no_lnfold=1: LayerNorm kernels, bf16(LN(x)) operands): both are bf16 paths with different
    rounding points, so they are compared by tolerance and by their distance to the fp32 path."""
    from ssr_amd import _lib, config as C, synth
    from ssr_amd.model import SSEModel
    m = SSEModel(C.WAVLM_BASE, wavlm_sd, device="cuda:0", dtype="bf16")
    w = torch.from_numpy(synth.synth_clips(6, 48000, seed=21)).cuda()
    idx = list(range(13))
    a = m.embed(w, idx).cpu().numpy()
    ha = [h.clone() for h in m.hidden_states(w[:2])]
    with _lib.option("no_lnfold", 1):
        b = m.embed(w, idx).cpu().numpy()
        hb = m.hidden_states(w[:2])
    m32 = SSEModel(C.WAVLM_BASE, wavlm_sd, device="cuda:0", dtype="fp32")
    r = m32.embed(w, idx).cpu().numpy()
    e_a, e_b = _rel(a, r).max(), _rel(b, r).max()
    print("folded vs materialised", _rel(a, b).max(), "| vs fp32: folded", e_a, "materialised", e_b)
    assert _rel(a, b).max() <= 2e-2
    assert e_a <= 1.25 * e_b + 1e-3 and e_a <= BF16_TOL
    for x, y in zip(ha, hb):
        x, y = x.cpu().numpy().reshape(2, -1), y.cpu().numpy().reshape(2, -1)
        assert _rel(x, y).max() <= 2e-2
    # the pool's LayerNorm from the GEMM partials == the LayerNorm kernel's own statistics
    pooled_hs = torch.stack([h.mean(dim=1) for h in ha], dim=1).cpu().numpy()
    assert _rel(a[:2], pooled_hs).max() <= 1e-5


def test_large_bf16_qkv_fold_matches_materialised():
    """WavLM-large (stable-LN) in bf16: layers l > 0 run no attention LayerNorm kernel -- the previous
    ffn2 writes per-256-column partials of the rounded bf16 stream and the QKV GEMM applies the
    LayerNorm through folded weights (FNT = 4 partials per row, H = 1024).  Against the materialised
    flow (no_lnfold=1) by tolerance and by the distance of each to the fp32 path."""
    from ssr_amd import _lib, config as C, synth
    from ssr_amd.model import SSEModel
    sd = synth.synth_wavlm_state_dict(C.WAVLM_LARGE, seed=9)
    m = SSEModel(C.WAVLM_LARGE, sd, device="cuda:0", dtype="bf16", do_normalize=True)
    w = torch.from_numpy(synth.synth_clips(5, 48000, seed=23)).cuda()
    idx = [24, 18, 12, 6, 1]
    a = m.embed(w, idx).cpu().numpy()
    with _lib.option("no_lnfold", 1):
        b = m.embed(w, idx).cpu().numpy()
    del m
    m32 = SSEModel(C.WAVLM_LARGE, sd, device="cuda:0", dtype="fp32", do_normalize=True)
    r = m32.embed(w, idx).cpu().numpy()
    e_a, e_b = _rel(a, r).max(), _rel(b, r).max()
    print("large folded vs materialised", _rel(a, b).max(), "| vs fp32: folded", e_a, "materialised", e_b)
    assert _rel(a, b).max() <= 2e-2
    assert e_a <= 1.25 * e_b + 1e-3 and e_a <= BF16_TOL


@pytest.mark.parametrize("n_clips,samples", [(7, 48000), (2, 16000), (3, 80000), (3, 160000), (1, 170000)])
def test_bf16_posconv_kernel_matches_grouped_gemm(wavlm_sd, n_clips, samples):
    """The dedicated positional-conv kernel (input window staged once per block, kernels_posconv.hip)
    against the grouped-GEMM path it replaces (posconv_gemm=1), on hidden_states[0] (the
    layer right after it) and the pooled layers: same math, fp32 accumulation in another order.
    Odd clip counts (the second clip of the last block is empty) and T = 49 / 149 / 249 frames, and
    clips over 256 frames (T = 499 / 530: 256-frame chunks, each with its own window borders)."""
    from ssr_amd import config as C, synth
    from ssr_amd.model import SSEModel
    m = SSEModel(C.WAVLM_BASE, wavlm_sd, device="cuda:0", dtype="bf16")
    w = torch.from_numpy(synth.synth_clips(n_clips, samples, seed=5)).cuda()
    idx = [0, 6, 12]
    a = m.embed(w, idx).cpu().numpy()
    h0 = m.hidden_states(w[:1])[0].cpu().numpy()
    from ssr_amd import _lib
    with _lib.option("posconv_gemm", 1):
        b = m.embed(w, idx).cpu().numpy()
        g0 = m.hidden_states(w[:1])[0].cpu().numpy()
    assert _rel(h0.reshape(-1), g0.reshape(-1)) <= 1e-5
    assert _rel(a[:, 0], b[:, 0]).max() <= 1e-5
    assert _rel(a, b).max() <= 5e-3
    # 4 clips per block (48-channel groups, <= 160 frames) vs 2 (option posconv_2cl): the same K order
    # per output, so bit-identical; 7 / 3 / 2 clips leave partial 4-clip blocks
    with _lib.option("posconv_2cl", 1):
        c2 = m.embed(w, idx).cpu().numpy()
    assert np.array_equal(a, c2)


@pytest.mark.parametrize("samples", [16000, 20001, 48000])
def test_bf16_conv0_matrix_core_matches_valu(wavlm_sd, samples):
    """conv0 + GroupNorm + GELU on the matrix cores (split-bf16 K = 32 MFMA, conv0_mfma_kernel)
    against the packed-fp32 VALU kernel (conv0_valu=1).  The convolutions agree to ~1e-5 before
    the bf16 output rounding; the rare rounding flips then propagate through six bf16 conv GEMMs like
    any bf16 noise, so the two bf16 paths are compared by their distance to the fp32 path (which
    runs conv0 in fp32 FMAs): the matrix-core path must be no farther from it than the VALU path."""
    from ssr_amd import config as C, synth
    from ssr_amd.model import SSEModel
    w = torch.from_numpy(synth.synth_clips(3, samples, seed=17)).cuda()
    idx = [0, 6, 12]
    m32 = SSEModel(C.WAVLM_BASE, wavlm_sd, device="cuda:0", dtype="fp32")
    ref, h_ref = m32.embed(w, idx).cpu().numpy(), m32.hidden_states(w[:1])[0].cpu().numpy().reshape(-1)
    del m32
    m = SSEModel(C.WAVLM_BASE, wavlm_sd, device="cuda:0", dtype="bf16")
    a = m.embed(w, idx).cpu().numpy()
    h0 = m.hidden_states(w[:1])[0].cpu().numpy().reshape(-1)
    from ssr_amd import _lib
    with _lib.option("conv0_valu", 1):
        b = m.embed(w, idx).cpu().numpy()
        g0 = m.hidden_states(w[:1])[0].cpu().numpy().reshape(-1)
    e_m, e_v = _rel(h0, h_ref), _rel(g0, h_ref)
    E_m, E_v = _rel(a, ref).max(), _rel(b, ref).max()
    print("hidden_states[0] vs fp32: mfma", e_m, "valu", e_v, "| embeddings: mfma", E_m, "valu", E_v,
          "| mfma vs valu", _rel(h0, g0))
    assert _rel(h0, g0) <= 1e-2
    assert e_m <= 1.25 * e_v and E_m <= 1.25 * E_v + 1e-3


@pytest.mark.parametrize("dtype,tol", [("fp32", FP32_TOL), ("bf16", BF16_TOL)])
def test_clip_longer_than_bias_table(dtype, tol, wavlm_sd):
    """A clip of 4124 frames (> the 4095-distance relative-position table, ~82.5 s): the kernels
    clamp |key - query| to the table edge, exact because the bucket saturates at max_distance = 800
    (HF _relative_positions_bucket); the reference embeds any length (REF/WavLM_embeddings.py:297-307)."""
    from oracle.wavlm import WavLMOracle
    from ssr_amd import config as C, synth
    from ssr_amd.model import SSEModel
    L = 320 * 4124 + 80
    assert C.WAVLM_BASE.frames(L) == 4124
    clip = synth.synth_clips(1, L, seed=4124)
    m = SSEModel(C.WAVLM_BASE, wavlm_sd, device="cuda:0", dtype=dtype)
    got = m.embed(torch.from_numpy(clip).cuda(), [12, 6, 0]).cpu().numpy()
    ref = WavLMOracle(C.WAVLM_BASE, wavlm_sd).embed(clip, [12, 6, 0])
    rel = _rel(got, ref).max()
    print(dtype, "T=4124 rel-L2", rel)
    assert rel <= tol


@pytest.fixture(scope="module")
def mx3(wavlm_sd):
    from ssr_amd import config as C
    from ssr_amd.model import SSEModel
    return SSEModel(C.WAVLM_BASE, wavlm_sd, device="cuda:0", dtype="fp16x3")


def test_fp16x3_embed_matches_reference(mx3, wavlm_clips, golden_wavlm):
    """Split-fp16 GEMMs (operands hi + lo, three fp16 products accumulated in fp32): the north star's
    fp32 bar, pooled rel-L2 <= 1e-4 against the reference's own fixture, with and without the
    feature extractor's normalisation; every hidden state of one clip too."""
    idx = [int(i) for i in golden_wavlm["layer_indices"]]
    got = mx3.embed(torch.from_numpy(wavlm_clips).cuda(), idx).cpu().numpy()
    rel = _rel(got, golden_wavlm["emb_norm0"])
    print("fp16x3 max rel-L2", rel.max())
    assert rel.max() <= FP32_TOL
    hs = mx3.hidden_states(torch.from_numpy(wavlm_clips[:2]).cuda())
    pooled = torch.stack([h.mean(dim=1) for h in hs], dim=1).cpu().numpy()
    assert _rel(pooled, golden_wavlm["emb_all_layers"]).max() <= FP32_TOL
    h1 = hs[1][0].cpu().numpy()
    assert np.linalg.norm(h1 - golden_wavlm["hs1_clip0"]) / np.linalg.norm(golden_wavlm["hs1_clip0"]) <= FP32_TOL


def test_fp16x3_normalize_and_batch_invariance(wavlm_sd, golden_wavlm):
    from ssr_amd import config as C, synth
    from ssr_amd.model import SSEModel
    m = SSEModel(C.WAVLM_BASE, wavlm_sd, device="cuda:0", dtype="fp16x3", do_normalize=True)
    idx = [int(i) for i in golden_wavlm["layer_indices"]]
    clips = synth.synth_clips(16, 48000, seed=1234)
    got = m.embed(torch.from_numpy(clips[:4]).cuda(), idx).cpu().numpy()
    assert _rel(got, golden_wavlm["emb_norm1"]).max() <= FP32_TOL
    w = torch.from_numpy(synth.synth_clips(40, 48000, seed=8)).cuda()
    full = m.embed(w, idx)
    for i in (0, 39):
        assert torch.equal(full[i:i + 1], m.embed(w[i:i + 1], idx))


def test_fp16x3_multirow_layernorm_is_bit_identical(mx3):
    """The R-rows-per-wave split-fp16 LayerNorm (layernorm_x3_rows_kernel) against the one-row-per-wave
    kernel it replaced (option ln_x3_v1): the same sums and expressions, so embeddings and every hidden
    state agree bit for bit (17 clips: a ragged last block of rows)."""
    from ssr_amd import _lib, synth
    w = torch.from_numpy(synth.synth_clips(17, 48000, seed=21)).cuda()
    idx = [12, 7, 0]
    new = mx3.embed(w, idx)
    hs_new = mx3.hidden_states(w[:3])
    with _lib.option("ln_x3_v1", 1):
        old = mx3.embed(w, idx)
        hs_old = mx3.hidden_states(w[:3])
    assert torch.equal(new, old)
    for a, b in zip(hs_new, hs_old):
        assert torch.equal(a, b)


@pytest.mark.parametrize("shape", [(3, 48000), (2, 160000), (3, 5000)])
def test_fp16x3_posconv_kernel_matches_fp32_grouped_gemm(mx3, shape):
    """The split-fp16 positional conv (posconv_x3_kernel: three fp16 products per term, ~22 bits per
    operand) against the exact-fp32 grouped GEMM it replaced (option posconv_gemm): every hidden state
    within 1e-5 rel-L2 -- 149 frames (one 160-frame chunk), 499 (four, the last partial), 15 (32-frame
    tile)."""
    from ssr_amd import _lib, synth
    w = torch.from_numpy(synth.synth_clips(shape[0], shape[1], seed=33)).cuda()
    new = mx3.hidden_states(w)
    with _lib.option("posconv_gemm", 1):
        ref = mx3.hidden_states(w)
    for a, b in zip(new, ref):
        rel = ((a - b).norm() / b.norm()).item()
        assert rel <= 1e-5, rel


@pytest.mark.parametrize("shape", [(3, 48000), (2, 160000), (3, 5000)])
def test_fp16x3_attention_matches_exact_fp32(mx3, shape):
    """The split-fp16 attention (attention_kernel X3: q/k/v and P split into fp16 hi + lo', three f16
    matrix-core products per term) against the exact-f32 MFMA form (option attn_x3_f32): every hidden
    state within 1e-5 rel-L2 at 149, 499 (8 key tiles, ragged last) and 15 frames."""
    from ssr_amd import _lib, synth
    w = torch.from_numpy(synth.synth_clips(shape[0], shape[1], seed=34)).cuda()
    new = mx3.hidden_states(w)
    with _lib.option("attn_x3_f32", 1):
        ref = mx3.hidden_states(w)
    for a, b in zip(new, ref):
        rel = ((a - b).norm() / b.norm()).item()
        assert rel <= 1e-5, rel


@pytest.mark.parametrize("dtype", ["bf16", "fp16x3", "fp16"])
def test_two_stream_split_equals_one_stream(wavlm_sd, dtype):
    """Batches of >= 128 WavLM clips run as two half-batches on two streams (split_forward): bit-identical
    to the single-stream call (no_split=1), for an odd batch and a ragged one, and the result is on the
    caller's stream when the call returns (the join)."""
    from ssr_amd import _lib, synth
    from ssr_amd import config as C
    from ssr_amd.model import SSEModel
    m = SSEModel(C.WAVLM_BASE, wavlm_sd, device="cuda:0", dtype=dtype)
    w = torch.from_numpy(synth.synth_clips(131, 48000, seed=17)).cuda()
    idx = [12, 11, 10, 6, 0]
    a = m.embed(w, idx)
    with _lib.option("no_split", 1):
        b = m.embed(w, idx)
    assert torch.equal(a, b)
    lens = [48000 - 97 * i for i in range(131)]
    a = m.embed(w, idx, lengths=lens)
    with _lib.option("no_split", 1):
        b = m.embed(w, idx, lengths=lens)
    assert torch.equal(a, b)


@pytest.mark.parametrize("dtype", ["fp16"])
def test_wavlm_large_posconv_kernel_matches_grouped_gemm(dtype):
    """WavLM-large's 64-channel positional-conv groups on the dedicated kernel (kernels_posconv.hip,
    CG = 64; the fp16 path's only form -- bf16 keeps the grouped GEMM, measured faster there) against
    the fp32 path, 3 s and 10 s clips (one chunk / 192-frame chunks)."""
    from ssr_amd import _lib, config as C, synth
    from ssr_amd.model import SSEModel
    sd = synth.synth_wavlm_state_dict(C.WAVLM_LARGE, seed=9)
    m = SSEModel(C.WAVLM_LARGE, sd, device="cuda:0", dtype=dtype)
    for L in (48000, 160000):
        w = torch.from_numpy(synth.synth_clips(3, L, seed=5)).cuda()
        h0 = m.hidden_states(w[:1])[0].cpu().numpy()
        if dtype == "bf16":
            with _lib.option("posconv_gemm", 1):
                g0 = m.hidden_states(w[:1])[0].cpu().numpy()
            assert _rel(h0.reshape(-1), g0.reshape(-1)) <= 1e-5, L
        else:
            f0 = SSEModel(C.WAVLM_LARGE, sd, device="cuda:0", dtype="fp32").hidden_states(w[:1])[0].cpu().numpy()
            assert _rel(h0.reshape(-1), f0.reshape(-1)) <= 5e-3, L


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
def test_wide_row_layernorm_matches_one_row_kernel(dtype):
    """WavLM-large's 1024-wide 16-bit LayerNorms (pre-LN stream) on the 2-rows-per-wave kernel
    (layernorm_bf16_rows_kernel NC = 2, weights held per wave) against the one-row-per-wave kernel
    (option ln_rows_v1): the same expression with the row sum in another order, so outputs agree to
    the 16-bit rounding -- pooled embeddings within 2e-3 rel-L2, batch invariance bit for bit."""
    from ssr_amd import _lib, config as C, synth
    from ssr_amd.model import SSEModel
    sd = synth.synth_wavlm_state_dict(C.WAVLM_LARGE, seed=9)
    m = SSEModel(C.WAVLM_LARGE, sd, device="cuda:0", dtype=dtype)
    w = torch.from_numpy(synth.synth_clips(5, 48000, seed=6)).cuda()
    idx = [24, 12, 3]
    new = m.embed(w, idx)
    with _lib.option("ln_rows_v1", 1):
        old = m.embed(w, idx)
    rel = ((new - old).norm(dim=-1) / old.norm(dim=-1)).max().item()
    assert rel <= 2e-3, rel
    assert torch.equal(new[3:4], m.embed(w[3:4], idx))
