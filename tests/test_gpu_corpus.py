"""BASELINE configs[3] code path on the GPU: ``corpus.extract_corpus`` driving the HIP embed
(``sse_embed_fn`` -> libsse.so) inside a real RCCL ("nccl") process group, the loop that replaces
the reference's per-file driver (REF/WavLM_embeddings.py:575-586).

World size 1 on the one-GPU box (8-GPU runs belong to the driver's scaling bench); the multi-rank
sharding / tail / trim logic is covered with gloo in tests/test_corpus_dist.py.  Here: ragged N
(600 clips, batch 256 -> batches of 256, 256, 88), the all-gather over RCCL, bit-identity with one
``embed`` over the same clips, and a subset against the fp32 oracle.
"""
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def nccl_group():
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    yield dist
    dist.destroy_process_group()


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_extract_corpus_hip_path_rccl(nccl_group, wavlm_sd, dtype):
    from ssr_amd import config as C, synth
    from ssr_amd.corpus import extract_corpus, sse_embed_fn
    from ssr_amd.model import SSEModel
    spec = C.WAVLM_BASE
    N, B = 600, 256
    idx = spec.default_layer_indices()
    clips = torch.from_numpy(synth.synth_clips(N, 48000, seed=606)).cuda()
    m = SSEModel(spec, wavlm_sd, device="cuda:0", dtype=dtype)
    calls = []

    def source(s, e):
        calls.append((s, e))
        return clips[s:e]

    emb = extract_corpus(source, N, sse_embed_fn(m, idx), (len(idx), spec.hidden), device="cuda:0", batch=B)
    torch.cuda.synchronize()
    assert calls == [(0, 256), (256, 512), (512, 600)]
    assert emb.shape == (N, len(idx), spec.hidden) and torch.isfinite(emb).all()
    one = m.embed(clips, idx)              # the whole corpus as one batch: no cross-clip reduction
    assert torch.equal(emb, one)
    if dtype == "fp32":
        from oracle.wavlm import WavLMOracle
        sel = [0, 300, 599]
        ref = WavLMOracle(spec, wavlm_sd).embed(clips[sel].cpu().numpy(), idx)
        got = emb[sel].cpu().numpy()
        rel = np.linalg.norm(got - ref, axis=-1) / np.linalg.norm(ref, axis=-1)
        assert rel.max() <= 1e-4, rel.max()


def test_extract_corpus_mixed_lengths_host_staged(nccl_group, wavlm_sd):
    """a 600-clip corpus of MIXED lengths (0.5-3.2 s, every clip under the
    160-frame attention split) from HOST memory through extract_corpus: ragged batches of 256 staged
    by the double-buffered pinned H2D on the side stream, embedded into the shard buffer through
    out=, the all-gather over RCCL -- bit-identical to embedding each clip alone."""
    from ssr_amd import config as C, synth
    from ssr_amd.corpus import extract_corpus, sse_embed_fn
    from ssr_amd.model import SSEModel
    spec = C.WAVLM_BASE
    N = 600
    idx = spec.default_layer_indices()
    rng = np.random.default_rng(5)
    lens = rng.integers(8000, 51000, size=N)
    clips = [synth.synth_clips(1, int(n), seed=900 + i)[0] for i, n in enumerate(lens)]
    m = SSEModel(spec, wavlm_sd, device="cuda:0", dtype="bf16")
    emb = extract_corpus(lambda s, e: clips[s:e], N, sse_embed_fn(m, idx), (len(idx), spec.hidden),
                         device="cuda:0", batch=256)
    torch.cuda.synchronize()
    assert emb.shape == (N, len(idx), spec.hidden) and torch.isfinite(emb).all()
    for i in range(N):
        one = m.embed(torch.from_numpy(clips[i]).cuda()[None], idx)
        assert torch.equal(emb[i:i + 1], one), (i, int(lens[i]))
