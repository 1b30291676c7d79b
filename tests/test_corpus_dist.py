"""Multi-process (gloo, world_size 2 and 3, CPU) coverage of the clip-sharded extraction and
its all-gather (corpus.py), with a deterministic CPU stand-in for the per-clip embedding so
sharding, padding and ordering are checked exactly."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _clips(start, stop, L=64):
    i = np.arange(start, stop, dtype=np.float32)[:, None]
    return (np.sin(i * 0.37 + np.arange(L, dtype=np.float32)[None, :] * 0.11)).astype(np.float32)


def _embed(wave):
    # [b, L] -> [b, 2, 3]: per-clip chunk means (depends only on that clip)
    b = wave.shape[0]
    return wave.reshape(b, 2, 3, -1).mean(-1)


def _ragged_clip(i):
    n = 20 + (i * 7919) % 41          # lengths 20..60
    return np.sin(i * 0.37 + np.arange(n, dtype=np.float32) * 0.11).astype(np.float32)


def _embed_one(x):
    # one clip at its own length -> [2, 3] (depends on no padding)
    return torch.stack([torch.stack([x.mean(), x.abs().max(), x[:7].sum()]),
                        torch.stack([(x * x).mean(), x.min(), torch.tensor(float(x.numel()))])])


def _embed_ragged(wave, lengths=None, out=None):
    lens = lengths if lengths is not None else [wave.shape[1]] * wave.shape[0]
    res = torch.stack([_embed_one(wave[b, :lens[b]]) for b in range(wave.shape[0])])
    if out is not None:
        out.copy_(res)
        return out
    return res


def _worker(rank, world, port, n_items, batch, q, ragged=False):
    import importlib
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    importlib.import_module("stuttering-speech-representation_amd")
    import torch.distributed as dist
    from ssr_amd.corpus import extract_corpus
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if ragged:   # mixed lengths: a list of 1-D clips per batch -> padded batch + lengths
            out = extract_corpus(lambda s, e: [_ragged_clip(i) for i in range(s, e)], n_items, _embed_ragged, (2, 3),
                                 "cpu", batch=batch)
        else:
            out = extract_corpus(lambda s, e: _clips(s, e, 66), n_items, _embed, (2, 3), "cpu", batch=batch)
        q.put((rank, out.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_items,batch", [(2, 10, 3), (3, 7, 4), (2, 1, 256)])
def test_sharded_extraction_matches_single_process(world, n_items, batch):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000) + world * 7 + n_items
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_items, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _embed(torch.from_numpy(_clips(0, n_items, 66))).numpy()
    for r in range(world):
        assert res[r].shape == (n_items, 2, 3)
        assert np.array_equal(res[r], ref), r


def test_shard_bounds_cover_exactly_once():
    import importlib
    importlib.import_module("stuttering-speech-representation_amd")
    from ssr_amd.corpus import shard_bounds
    for n in (0, 1, 7, 50000):
        for w in (1, 2, 3, 8):
            seen = []
            for r in range(w):
                s, e, per = shard_bounds(n, w, r)
                assert e - s <= per
                seen.extend(range(s, e))
            assert seen == list(range(n))
    with pytest.raises(ValueError):
        shard_bounds(10, 2, 2)


@pytest.mark.parametrize("world,n_items,batch", [(2, 11, 4), (3, 8, 3)])
def test_sharded_ragged_extraction_matches_per_clip(world, n_items, batch):
    """Mixed-length corpus (REF/WavLM_embeddings.py:284-307 embeds each file at its own length):
    every rank's ragged batches give exactly each clip's own embedding, in corpus order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + (os.getpid() % 1000) + world * 11 + n_items
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_items, batch, q, True)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = torch.stack([_embed_one(torch.from_numpy(_ragged_clip(i))) for i in range(n_items)]).numpy()
    for r in range(world):
        assert np.array_equal(res[r], ref), r


def test_extract_corpus_out_and_lengths_protocol():
    """Single process: embed_fn receives out= slices of the shard buffer (no per-batch allocation)
    and lengths= only for ragged batches; an embed_fn without lengths= rejects a ragged batch."""
    import importlib
    importlib.import_module("stuttering-speech-representation_amd")
    from ssr_amd.corpus import extract_corpus
    seen = []

    def fn(wave, lengths=None, out=None):
        seen.append((lengths, out is not None))
        return _embed_ragged(wave, lengths, out)

    out = extract_corpus(lambda s, e: [_ragged_clip(i) for i in range(s, e)], 5, fn, (2, 3), "cpu", batch=2)
    ref = torch.stack([_embed_one(torch.from_numpy(_ragged_clip(i))) for i in range(5)])
    assert torch.equal(out, ref) and all(o for _, o in seen) and [len(l) for l, _ in seen] == [2, 2, 1]
    extract_corpus(lambda s, e: _clips(s, e, 66), 3, fn, (2, 3), "cpu", batch=2)
    assert seen[-1][0] is None
    with pytest.raises(ValueError):
        extract_corpus(lambda s, e: [_ragged_clip(i) for i in range(s, e)], 3, _embed, (2, 3), "cpu", batch=2)


def _balanced_worker(rank, world, port, lens, batch, q):
    import importlib
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    importlib.import_module("stuttering-speech-representation_amd")
    import torch.distributed as dist
    from ssr_amd.corpus import extract_corpus
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = {"finish": 0, "samples": 0}

    def fn(wave, lengths=None, out=None):
        calls["samples"] += sum(lengths)
        return _embed_ragged(wave, lengths=lengths, out=out)
    fn.finish = lambda: calls.__setitem__("finish", calls["finish"] + 1)

    def clip(i):
        return np.sin(i * 0.37 + np.arange(lens[i], dtype=np.float32) * 0.11).astype(np.float32)
    try:
        out = extract_corpus(lambda s, e: [clip(i) for i in range(s, e)], len(lens), fn, (2, 3), "cpu", batch=batch,
                             item_lengths=lens)
        q.put((rank, (out.numpy(), calls["finish"], calls["samples"])))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,batch", [(2, 4), (3, 3)])
def test_length_balanced_shards_restore_corpus_order(world, batch):
    """a corpus ordered by length (a sorted manifest) sharded by samples, not by count:
    every rank embeds ~1/world of the samples, finish() runs once per rank, and the gathered matrix is
    each clip's own embedding in corpus order."""
    lens = [20 + 3 * i for i in range(13)]          # ascending lengths: count shards would be unbalanced
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 33500 + (os.getpid() % 1000) + world * 13
    procs = [ctx.Process(target=_balanced_worker, args=(r, world, port, lens, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = torch.stack([_embed_one(torch.from_numpy(
        np.sin(i * 0.37 + np.arange(n, dtype=np.float32) * 0.11).astype(np.float32))) for i, n in enumerate(lens)]).numpy()
    total = sum(lens)
    for r in range(world):
        out, fin, samples = res[r]
        assert np.array_equal(out, ref), r
        assert fin == 1
        assert abs(samples - total / world) <= max(lens), (r, samples, total / world)


def test_balanced_bounds_cover_and_balance():
    import importlib
    importlib.import_module("stuttering-speech-representation_amd")
    from ssr_amd.corpus import balanced_bounds
    rng = np.random.default_rng(5)
    for n, w in [(1, 1), (5, 8), (8, 8), (13, 3), (1000, 8)]:
        for lens in (sorted(rng.integers(400, 480000, n).tolist()), [48000] * n, rng.integers(1, 10, n).tolist()):
            b = balanced_bounds(lens, w)
            assert b[0] == 0 and b[-1] == n and len(b) == w + 1
            assert all(b[i] <= b[i + 1] for i in range(w))
            if n >= w:
                assert all(b[i] < b[i + 1] for i in range(w)), (n, w, b)
                share = [sum(lens[b[i]:b[i + 1]]) for i in range(w)]
                assert max(share) - sum(lens) / w <= 2 * max(lens)


def _step_gather_worker(rank, world, port, steps, q):
    import importlib
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    importlib.import_module("stuttering-speech-representation_amd")
    import torch.distributed as dist
    from ssr_amd.corpus import StepGather
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        k = [0]

        def embed(out):      # step k on rank r writes r * 1000 + k + the row index
            out.copy_(torch.arange(out.shape[0], dtype=torch.float32)[:, None, None].expand_as(out) + rank * 1000 + k[0])
            k[0] += 1
        pipe = StepGather(embed, (3, 2, 4), world, "cpu", dist)
        seen = []
        for _ in range(steps):
            slot = pipe.step()
            seen.append((slot, pipe.pending[1 - slot] is None or pipe.steps >= 2))
        pipe.drain()
        assert all(p is None for p in pipe.pending)
        q.put((rank, ([s for s, _ in seen], [g.numpy().copy() for g in pipe.gathered], pipe.steps)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,steps", [(2, 5), (3, 4)])
def test_step_gather_two_slots_and_drain(world, steps):
    """bench.py's weak-scaling step (async all-gather into two slots, a slot reused
    only after its gather completed, drain before the closing barrier) on gloo: after the drain each
    slot holds the all-gather of the last step that wrote it, ranks in order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 35500 + (os.getpid() % 1000) + world * 17 + steps
    procs = [ctx.Process(target=_step_gather_worker, args=(r, world, port, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        slots, gathered, n = res[r]
        assert n == steps and slots == [i % 2 for i in range(steps)]
        for slot in (0, 1):
            last = max(i for i in range(steps) if i % 2 == slot)
            exp = np.concatenate([np.arange(3, dtype=np.float32)[:, None, None] + rr * 1000 + last
                                  for rr in range(world)])
            assert np.array_equal(gathered[slot], np.broadcast_to(exp, (world * 3, 2, 4))), (r, slot)


def _finish_fail_worker(rank, world, port, q):
    import importlib
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    importlib.import_module("stuttering-speech-representation_amd")
    import torch.distributed as dist
    from ssr_amd import _lib
    from ssr_amd.corpus import ShardFinishError, extract_corpus
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def fn(wave):
        return _embed(wave)

    def fail():   # the fp16-range check of sse_embed_fn, failing on rank 1 only
        if rank == 1:
            raise _lib.SSERangeError(_lib.SSE_ERR_RANGE, "sse_check_range")
    fn.finish = fail
    try:
        extract_corpus(lambda s, e: _clips(s, e, 66), 9, fn, (2, 3), "cpu", batch=2)
        q.put((rank, "no error"))
    except ShardFinishError as e:
        q.put((rank, "peer: " + str(e)))
    except _lib.SSERangeError as e:
        q.put((rank, "own: " + str(e)))
    finally:
        dist.destroy_process_group()


def test_finish_failure_raises_on_every_rank():
    """one rank's fp16-range failure used to raise there while the other ranks blocked in the
    all-gather until the collective timed out.  Now every rank raises together: the failing rank its own
    SSERangeError with its shard bounds, the others ShardFinishError naming it -- and nobody hangs."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 34600 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_finish_fail_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1].startswith("own: ") and "rank 1, shard [3, 6)" in res[1], res[1]
    for r in (0, 2):
        assert res[r].startswith("peer: ") and "rank(s) [1]" in res[r], res[r]


def _verify_worker(rank, world, port, mode, q):
    import importlib
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    importlib.import_module("stuttering-speech-representation_amd")
    import torch.distributed as dist
    from ssr_amd.corpus import StepGather
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        k = [0]

        def embed(out):      # rank-tagged rows (bench.py: rank r embeds clips r*B ..), or every rank the same
            tag = 0 if mode == "replicated" else rank * 1000
            out.copy_(torch.arange(out.numel(), dtype=torch.float32).view_as(out) * 0.5 + tag + k[0])
            k[0] += 1
        pipe = StepGather(embed, (3, 2, 4), world, "cpu", dist)
        for _ in range(3):
            pipe.step()
        pipe.drain()
        if mode == "stale" and rank == 1:   # a block that is not the last step's (a slot mix-up)
            pipe.gathered[0].view(world, -1)[0] += 1.0
        try:
            q.put((rank, pipe.verify()))
        except RuntimeError as e:
            q.put((rank, "error: " + str(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["ok", "stale", "replicated"])
def test_step_gather_verify(mode):
    """the multi-rank bench line verifies itself -- rccl_world is the backend's own world
    size, every rank's rows sit at its block of the last gathered slot (checksums of all blocks against each
    rank's own), and rank-tagged rows are distinct.  A corrupted block or replicated rows raise."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 36700 + (os.getpid() % 1000) + len(mode)
    procs = [ctx.Process(target=_verify_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if mode == "ok":
        for r in range(world):
            assert res[r] == {"rccl_world": 2, "backend": "gloo", "blocks_checked": 2}, res[r]
    elif mode == "stale":
        assert res[1].startswith("error: ") and "[0]" in res[1], res[1]
    else:
        assert all(v.startswith("error: ") and "identical" in v for v in res.values()), res
