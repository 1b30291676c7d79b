"""Clip-sharded multi-GPU extraction (BASELINE configs[3]).

The reference has no parallelism at all: one process, one device, batch 1
(REF/WavLM_embeddings.py:575-586).  Here one process per GPU (torch.distributed, backend
"nccl" = RCCL over xGMI) each embeds a contiguous shard of the corpus and ONE all-gather
reassembles the [N, n_layers, H] embedding matrix in corpus order on every rank:

  rank r owns clips [r*P, min((r+1)*P, N)), P = ceil(N / world)
  each shard is processed in batches of `batch` clips into a [P, n_layers, H] buffer
  (rows past the shard's end stay zero: equal counts for the all-gather), then
  all_gather_into_tensor -> [world*P, ...] -> trimmed to N rows.

The exchange is the only collective (clips are independent); it moves N*n_layers*H*4 bytes
in total (614 MB for 50k WavLM-base clips), milliseconds against seconds of compute.
``embed_fn`` is injectable so the sharding, padding and ordering logic is testable with the
gloo backend on CPU; in production it is ``SSEModel.embed`` on the rank's GPU.
"""
from __future__ import annotations

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


def extract_corpus(clip_source: Callable[[int, int], np.ndarray | torch.Tensor], n_items: int,
                   embed_fn: Callable[[torch.Tensor], torch.Tensor], out_shape: tuple[int, int],
                   device, batch: int = 256, group=None) -> torch.Tensor:
    """Embed clips [0, n_items) across the process group; returns [n_items, *out_shape] fp32 on
    `device` on every rank (corpus order).

    clip_source(start, stop) -> [stop-start, L] clips of this rank's range (host or device).
    embed_fn(wave [b, L] on device) -> [b, *out_shape] fp32 on device.
    """
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    start, stop, per = shard_bounds(n_items, world, rank)
    local = torch.zeros((per,) + tuple(out_shape), dtype=torch.float32, device=device)
    for s in range(start, stop, batch):
        e = min(s + batch, stop)
        wave = clip_source(s, e)
        if not isinstance(wave, torch.Tensor):
            wave = torch.from_numpy(np.ascontiguousarray(wave))
        local[s - start:e - start] = embed_fn(wave.to(device, torch.float32))
    if not dist.is_initialized():
        return local[:n_items]
    full = torch.empty((world * per,) + tuple(out_shape), dtype=torch.float32, device=device)
    dist.all_gather_into_tensor(full, local, group=group)
    return full[:n_items]


def sse_embed_fn(model, layer_indices) -> Callable[[torch.Tensor], torch.Tensor]:
    """embed_fn for extract_corpus backed by the HIP path (SSEModel.embed)."""
    idx = [int(i) for i in layer_indices]
    return lambda wave: model.embed(wave, idx)
