"""Clip-sharded multi-GPU extraction (BASELINE configs[3]).

The reference has no parallelism at all: one process, one device, batch 1, every file embedded at
its own length (REF/WavLM_embeddings.py:575-586, :284-307).  Here one process per GPU
(torch.distributed, backend "nccl" = RCCL over xGMI) each embeds a contiguous shard of the corpus
and ONE all-gather reassembles the [N, n_layers, H] embedding matrix in corpus order on every rank:

  rank r owns clips [r*P, min((r+1)*P, N)), P = ceil(N / world)
  each shard is processed in batches of `batch` clips straight into a [P, n_layers, H] buffer
  (``out=`` slices: nothing is allocated per batch; rows past the shard's end stay zero: equal
  counts for the all-gather), then all_gather_into_tensor -> [world*P, ...] -> trimmed to N rows.

Mixed-length corpora: ``clip_source`` may return a list of 1-D clips (or ``(wave, lengths)``);
the batch is then a zero-padded ragged batch and every clip is embedded at its own length
(``SSEModel.embed(lengths=)`` -> sse_embed_ragged), so a corpus of mixed lengths does not fragment
into per-length batches.

Host-staged clips (numpy / CPU tensors) are double-buffered: batch i+1 is packed into a pinned
host buffer and copied on a side stream into the other of two device buffers while batch i
computes; the compute stream waits only for its own batch's copy event, and a device / pinned
buffer is rewritten only after the compute / copy that last used it has finished.  Clips already on
the device are used in place.

The exchange is the only collective (clips are independent); it moves N*n_layers*H*4 bytes
in total (614 MB for 50k WavLM-base clips), milliseconds against seconds of compute.
``embed_fn`` is injectable so the sharding, padding and ordering logic is testable with the
gloo backend on CPU; in production it is ``sse_embed_fn`` (SSEModel.embed) on the rank's GPU.
"""
from __future__ import annotations

import inspect
import math
from typing import Callable

import numpy as np
import torch


def shard_bounds(n_items: int, world: int, rank: int) -> tuple[int, int, int]:
    """(start, stop, per_rank) of rank's contiguous shard; per_rank = ceil(n / world)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    per = math.ceil(n_items / world) if n_items else 0
    start = min(rank * per, n_items)
    return start, min(start + per, n_items), per


def balanced_bounds(item_lengths, world: int) -> list[int]:
    """Contiguous shard boundaries [b_0 = 0, b_1, ..., b_world = N] that split the corpus's total samples
    (the work: the encoder's cost is linear in a clip's length to first order) as evenly as contiguity
    allows: rank r owns [b_r, b_{r+1}).  Count-based shards of a corpus ordered by length (a sorted
    manifest) give one rank all the long clips; these give every rank ~1/world of the samples.
    Every rank gets at least one item while n >= world."""
    lens = np.asarray([max(int(v), 0) for v in item_lengths], dtype=np.float64)
    n = lens.size
    if world <= 0:
        raise ValueError(f"bad world {world}")
    cum = np.concatenate([[0.0], np.cumsum(lens)])
    total = cum[-1]
    bounds = [0]
    for r in range(1, world):
        # first index whose prefix reaches r/world of the samples, kept strictly increasing with room
        # for the remaining ranks (one item each) when possible
        b = int(np.searchsorted(cum, total * r / world, side="left")) if total > 0 else (n * r) // world
        lo = bounds[-1] + (1 if n - bounds[-1] > world - r else 0)
        hi = n - (world - r) if n >= world else n
        bounds.append(int(min(max(b, lo), max(hi, lo))))
    bounds.append(n)
    return bounds


def _as_batch(src):
    """clip_source output -> (wave [b, L] tensor or ndarray, lengths list | None)."""
    if isinstance(src, tuple):
        wave, lens = src
        return wave, (None if lens is None else [int(v) for v in lens])
    if isinstance(src, list):
        lens = [int(np.asarray(c).shape[-1]) if not isinstance(c, torch.Tensor) else int(c.shape[-1]) for c in src]
        on_dev = all(isinstance(c, torch.Tensor) and c.device.type != "cpu" for c in src)
        if on_dev:
            wave = torch.zeros((len(src), max(lens)), dtype=torch.float32, device=src[0].device)
            for i, c in enumerate(src):
                wave[i, :lens[i]] = c.to(torch.float32)
        else:
            wave = np.zeros((len(src), max(lens)), np.float32)
            for i, c in enumerate(src):
                wave[i, :lens[i]] = c.cpu().numpy() if isinstance(c, torch.Tensor) else np.asarray(c, np.float32)
        return wave, lens
    return src, None


def _accepts(fn, name: str) -> bool:
    try:
        sig = inspect.signature(fn)
    except (TypeError, ValueError):
        return False
    return name in sig.parameters or any(p.kind == p.VAR_KEYWORD for p in sig.parameters.values())


class _Stager:
    """Double-buffered pinned-host -> device staging on a side stream (CUDA devices only)."""

    def __init__(self, device):
        self.dev = torch.device(device)
        self.stream = torch.cuda.Stream(self.dev)
        self.host = [None, None]       # pinned [b, L] fp32
        self.dbuf = [None, None]       # device [b, L] fp32
        self.copied = [None, None]     # event: the copy into dbuf[k] is done
        self.freed = [None, None]      # event: the compute that read dbuf[k] is done

    def put(self, k: int, wave) -> tuple[torch.Tensor, torch.cuda.Event]:
        w = wave if isinstance(wave, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(wave, np.float32))
        w = w.to(torch.float32)
        shape = tuple(w.shape)
        if self.copied[k] is not None:
            self.copied[k].synchronize()         # the pinned buffer's last copy has been read
        direct = w.is_pinned() and w.is_contiguous()   # caller-owned pinned memory: copied from in place
        if not direct and (self.host[k] is None or self.host[k].numel() < w.numel()):
            self.host[k] = torch.empty(w.numel(), dtype=torch.float32, pin_memory=True)
        if direct:
            h = w
        else:
            h = self.host[k][:w.numel()].view(shape)
            h.copy_(w)
        with torch.cuda.stream(self.stream):
            if self.freed[k] is not None:
                self.stream.wait_event(self.freed[k])   # compute on the old contents is finished
            if self.dbuf[k] is None or self.dbuf[k].numel() < w.numel():
                self.dbuf[k] = torch.empty(w.numel(), dtype=torch.float32, device=self.dev)
            d = self.dbuf[k][:w.numel()].view(shape)
            d.copy_(h, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.copied[k] = ev
        return d, ev

    def release(self, k: int) -> None:
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.dev))
        self.freed[k] = ev


def extract_corpus(clip_source: Callable[[int, int], object], n_items: int,
                   embed_fn: Callable[..., torch.Tensor], out_shape: tuple[int, int],
                   device, batch: int = 256, group=None, prefetch: bool = True,
                   item_lengths=None) -> torch.Tensor:
    """Embed clips [0, n_items) across the process group; returns [n_items, *out_shape] fp32 on
    `device` on every rank (corpus order).

    clip_source(start, stop) -> the clips of that range: an array / tensor [stop-start, L]
    (host or device), a list of 1-D clips of any lengths, or (wave [b, L], lengths).
    embed_fn(wave [b, L] on device, lengths=None | list, out=None | [b, *out_shape]) ->
    [b, *out_shape] fp32 on device (``lengths`` / ``out`` are passed only if it accepts them;
    without ``lengths`` a ragged batch is an error).  If embed_fn has a ``finish()`` attribute it is
    called once after the rank's last batch, before the exchange (sse_embed_fn: the fp16-range check).
    item_lengths (optional, n_items sample counts): shards balanced by samples (balanced_bounds)
    instead of by count; the exchange pads every shard to the longest one and the result is
    restored to corpus order.
    """
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    if item_lengths is not None:
        if len(item_lengths) != n_items:
            raise ValueError(f"item_lengths has {len(item_lengths)} entries for {n_items} items")
        bounds = balanced_bounds(item_lengths, world)
        start, stop = bounds[rank], bounds[rank + 1]
        per = max(bounds[r + 1] - bounds[r] for r in range(world))
    else:
        start, stop, per = shard_bounds(n_items, world, rank)
        bounds = None
    dev = torch.device(device)
    local = torch.zeros((per,) + tuple(out_shape), dtype=torch.float32, device=dev)
    takes_len, takes_out = _accepts(embed_fn, "lengths"), _accepts(embed_fn, "out")
    stager = _Stager(dev) if (prefetch and dev.type == "cuda") else None
    ranges = [(s, min(s + batch, stop)) for s in range(start, stop, batch)]

    def fetch(i):
        s, e = ranges[i]
        wave, lens = _as_batch(clip_source(s, e))
        if lens is not None and not takes_len:
            raise ValueError("a ragged batch needs an embed_fn that takes lengths=")
        if isinstance(wave, torch.Tensor) and wave.device == dev:
            return wave.to(torch.float32), lens, None
        if stager is not None:
            d, ev = stager.put(i & 1, wave)
            return d, lens, ev
        w = wave if isinstance(wave, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(wave))
        return w.to(dev, torch.float32), lens, None

    nxt = fetch(0) if ranges else None
    for i, (s, e) in enumerate(ranges):
        wave, lens, ev = nxt
        if ev is not None:
            torch.cuda.current_stream(dev).wait_event(ev)
        kw = {}
        if lens is not None:
            kw["lengths"] = lens
        if takes_out:
            kw["out"] = local[s - start:e - start]
        res = embed_fn(wave, **kw)
        if stager is not None and ev is not None:
            stager.release(i & 1)
        if i + 1 < len(ranges):
            nxt = fetch(i + 1)             # staged (host pack + async copy) while batch i computes
        if res is not None and res.data_ptr() != local[s - start:e - start].data_ptr():
            local[s - start:e - start] = res
    _finish_all(getattr(embed_fn, "finish", None), dist, group, world, rank, start, stop, dev)
    if not dist.is_initialized():
        return local[:n_items]
    full = torch.empty((world * per,) + tuple(out_shape), dtype=torch.float32, device=dev)
    dist.all_gather_into_tensor(full, local, group=group)
    if bounds is None:
        return full[:n_items]
    return torch.cat([full[r * per:r * per + bounds[r + 1] - bounds[r]] for r in range(world)])


class ShardFinishError(RuntimeError):
    """Raised on every rank whose own ``finish()`` passed when another rank's failed (extract_corpus)."""


def _finish_all(finish, dist, group, world: int, rank: int, start: int, stop: int, dev) -> None:
    """Run the rank's ``finish()`` (sse_embed_fn: the fp16-range check) and agree on the outcome before the
    exchange: one all-reduce of a per-rank failure vector, then every rank raises together -- the failing
    ranks their own error with their shard bounds appended, the others ShardFinishError naming the failing
    ranks -- instead of one rank raising while the others block in all_gather until the collective times out."""
    err = None
    if callable(finish):
        try:
            finish()
        except Exception as e:   # re-raised below, after every rank knows
            err = e
    where = f"rank {rank}, shard [{start}, {stop})"
    if dist.is_initialized() and world > 1:
        on_dev = dist.get_backend(group) == "nccl"
        bad = torch.zeros(world, dtype=torch.float32, device=dev if on_dev else "cpu")
        bad[rank] = 1.0 if err is not None else 0.0
        dist.all_reduce(bad, group=group)
        failed = [r for r in range(world) if bad[r].item() > 0]
    else:
        failed = [rank] if err is not None else []
    if err is not None:
        if err.args and isinstance(err.args[0], str):
            err.args = (f"{err.args[0]} [{where}]",) + tuple(err.args[1:])
        raise err
    if failed:
        raise ShardFinishError(f"{where}: finish() failed on rank(s) {failed}; no all-gather was issued")


def sse_embed_fn(model, layer_indices) -> Callable[..., torch.Tensor]:
    """embed_fn for extract_corpus backed by the HIP path (SSEModel.embed): writes into ``out``,
    ragged batches through ``lengths``."""
    idx = [int(i) for i in layer_indices]

    # no per-batch range check (it synchronises the stream and would cancel the staged copy / compute
    # overlap): fp16 / fp16x3 models are checked once, by finish(), after the rank's last batch
    def fn(wave, lengths=None, out=None):
        return model.embed(wave, idx, out=out, lengths=lengths, check_range=False)
    fn.finish = model.check_range_now
    return fn


class StepGather:
    """The weak-scaling step of bench.py --gpus N (BASELINE configs[3] per-step form): each step embeds
    one local batch into one of two output slots, then issues the all-gather of that slot with
    ``async_op=True`` (RCCL runs it on its own stream), so step k's exchange overlaps step k+1's
    compute.  A slot is rewritten only after the gather that last read it has completed; ``drain()``
    waits for every outstanding gather (before the closing barrier of a timed region).

    embed(out) writes this rank's [B, ...] embeddings into ``out`` (on the compute stream)."""

    def __init__(self, embed: Callable[[torch.Tensor], object], out_shape: tuple, world: int, device,
                 dist=None, group=None):
        self.embed = embed
        self.dist = dist
        self.group = group
        dev = torch.device(device)
        self.outs = [torch.empty(tuple(out_shape), dtype=torch.float32, device=dev) for _ in range(2)]
        self.gathered = ([torch.empty((world * out_shape[0],) + tuple(out_shape[1:]), dtype=torch.float32, device=dev)
                          for _ in range(2)] if dist is not None else None)
        self.pending = [None, None]
        self.steps = 0

    def step(self) -> int:
        slot = self.steps % 2
        self.steps += 1
        if self.pending[slot] is not None:     # the gather that last read this slot
            self.pending[slot].wait()
            self.pending[slot] = None
        self.embed(self.outs[slot])
        if self.dist is not None:
            self.pending[slot] = self.dist.all_gather_into_tensor(self.gathered[slot], self.outs[slot],
                                                                  group=self.group, async_op=True)
        return slot

    def drain(self) -> None:
        for i in range(2):
            if self.pending[i] is not None:
                self.pending[i].wait()
                self.pending[i] = None

    def verify(self) -> dict:
        """After ``drain()``: check that the last step's gathered slot is what every rank produced, in rank
        order, and report the world size the collective backend itself saw (bench.py's line carries it, so
        a multi-GPU record proves "RCCL saw N ranks" on its own).  Raises RuntimeError on any disagreement:

          * this rank's own rows sit at block ``rank`` of the gathered slot, bit for bit;
          * block r's checksum (fp64 sum, and sum weighted by position) equals the checksum rank r computed
            over its own rows (one tiny all_gather of [world, 2] checksums), so every block came from its
            rank and from that rank's LAST step (not a stale slot);
          * the per-rank checksums are pairwise distinct when ``distinct`` data is expected (bench clips are
            rank-tagged: rank r embeds clips r*B .. r*B + B - 1), so no rank's rows were replicated.

        Returns {"rccl_world": W, "backend": ..., "blocks_checked": W}."""
        if self.dist is None or self.steps == 0:
            return {"rccl_world": 1, "backend": None, "blocks_checked": 0}
        world = self.dist.get_world_size(self.group)
        rank = self.dist.get_rank(self.group)
        slot = (self.steps - 1) % 2
        own = self.outs[slot]
        B = own.shape[0]
        if self.gathered[slot].shape[0] != world * B:
            raise RuntimeError(f"gathered slot holds {self.gathered[slot].shape[0]} rows for world {world} x {B}")
        blocks = self.gathered[slot].view(world, B, -1)
        if not torch.equal(blocks[rank], own.view(B, -1)):
            raise RuntimeError(f"rank {rank}: its own rows are not at block {rank} of the gathered slot")

        def checksum(x):
            x = x.reshape(-1).double()
            w = torch.arange(1, x.numel() + 1, dtype=torch.float64, device=x.device)
            return torch.stack([x.sum(), (x * w).sum()])
        mine = checksum(own)
        flat = torch.empty((world * 2,), dtype=torch.float64, device=own.device)
        self.dist.all_gather_into_tensor(flat, mine, group=self.group)
        allsums = flat.view(world, 2)
        got = torch.stack([checksum(blocks[r]) for r in range(world)])
        if not torch.equal(got, allsums):
            bad = [r for r in range(world) if not torch.equal(got[r], allsums[r])]
            raise RuntimeError(f"rank {rank}: gathered blocks {bad} differ from their ranks' own rows")
        if len({tuple(v) for v in allsums.cpu().tolist()}) != world:
            raise RuntimeError(f"rank {rank}: two ranks contributed identical rows (expected rank-distinct clips)")
        return {"rccl_world": world, "backend": str(self.dist.get_backend(self.group)), "blocks_checked": world}
