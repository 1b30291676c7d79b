"""On-disk embedding format of the reference.

Writer: ``save_embeddings`` (REF/WavLM_embeddings.py:343-387, REF/whisper_embeddings_large.py:301-348)
  <output_dir>/<split>/embedding_metadata.csv   metadata columns, index=False
  <output_dir>/<split>/<col>_embeddings.npy     float32 [N, H], row-aligned with the CSV
(``split`` None or "all" writes into output_dir itself).  Reader side: ``load_data``
(REF/model_training_1.py:99-165) globs ``*_embeddings.npy`` per split and strips the suffix to
get the layer name.

For corpus runs the reference pickles the whole result list as its checkpoint
(REF/WavLM_embeddings.py:389-434).  Here each rank writes shard files plus a JSON manifest
(atomic rename) instead: ``ShardWriter`` (resume = skip rows a manifest already records) and
``merge_shards`` (rebuilds the reference layout in corpus order).
"""
from __future__ import annotations

import json
import logging
import os

import numpy as np
import pandas as pd

logger = logging.getLogger(__name__)

EMB_PREFIXES = ("layer_", "encoder_layer_", "decoder_layer_")


def _is_emb(col: str) -> bool:
    return col.startswith(EMB_PREFIXES)


def _split_dir(output_dir, split):
    d = os.path.join(output_dir, split) if split and split != "all" else output_dir
    os.makedirs(d, exist_ok=True)
    return d


def save_embeddings(embeddings_df: pd.DataFrame, output_dir, split=None, expected_dim=None):
    """Same contract as the reference's save_embeddings (both scripts): a DataFrame whose
    embedding columns hold one float32 [H] vector per row."""
    if len(embeddings_df) == 0:
        logger.warning("No embeddings to save")
        return
    split_dir = _split_dir(output_dir, split)
    meta_cols = [c for c in embeddings_df.columns if not _is_emb(c)]
    embeddings_df[meta_cols].copy().to_csv(os.path.join(split_dir, "embedding_metadata.csv"), index=False)
    logger.info(f"Saved metadata for {len(embeddings_df)} files to {split_dir}")
    for col in [c for c in embeddings_df.columns if _is_emb(c)]:
        try:
            if expected_dim is not None:
                d = len(embeddings_df[col].iloc[0])
                if d != expected_dim:
                    logger.warning(f"WARNING: {col} has dimension {d} but expected {expected_dim}")
            arr = np.stack(embeddings_df[col].values)
            np.save(os.path.join(split_dir, f"{col}_embeddings.npy"), arr)
            logger.info(f"Saved {col} embeddings with shape {arr.shape}")
        except Exception as e:
            logger.error(f"Error saving {col} embeddings: {e}")


def write_split(output_dir, split, metadata, embeddings: dict, expected_dim=None):
    """Batched form: ``metadata`` (DataFrame or list of dicts, N rows) and ``embeddings``
    {column name: float32 [N, H]} -> the same files as save_embeddings, without building a
    DataFrame of per-row arrays."""
    meta = metadata if isinstance(metadata, pd.DataFrame) else pd.DataFrame(list(metadata))
    n = len(meta)
    for name, arr in embeddings.items():
        if not _is_emb(name):
            raise ValueError(f"embedding column {name!r} must start with one of {EMB_PREFIXES}")
        if arr.shape[0] != n:
            raise ValueError(f"{name}: {arr.shape[0]} rows vs {n} metadata rows")
        if expected_dim is not None and arr.shape[1] != expected_dim:
            logger.warning(f"WARNING: {name} has dimension {arr.shape[1]} but expected {expected_dim}")
    if n == 0:
        logger.warning("No embeddings to save")
        return
    split_dir = _split_dir(output_dir, split)
    meta[[c for c in meta.columns if not _is_emb(c)]].to_csv(os.path.join(split_dir, "embedding_metadata.csv"),
                                                            index=False)
    for name, arr in embeddings.items():
        np.save(os.path.join(split_dir, f"{name}_embeddings.npy"), np.ascontiguousarray(arr, dtype=np.float32))


def load_split(output_dir, split=None):
    """Reader mirror of REF/model_training_1.py:116-160 for one split: (metadata, {layer: [N,H]})."""
    d = os.path.join(output_dir, split) if split and split != "all" else output_dir
    meta = pd.read_csv(os.path.join(d, "embedding_metadata.csv"))
    files = [f for f in os.listdir(d) if f.endswith("_embeddings.npy")]
    return meta, {os.path.splitext(f)[0].replace("_embeddings", ""): np.load(os.path.join(d, f)) for f in files}


class ShardWriter:
    """Per-rank shard files + manifest (replaces the reference's pickle checkpoints).

    ``write(row_start, metadata_rows, embeddings)`` stores rows [row_start, row_start+n) of the
    corpus as ``<dir>/shards/r{rank}_{row_start:09d}_<name>.npy`` (+ ``_meta.csv``) and then
    records them in ``manifest_r{rank}.json`` via an atomic rename, so a crash never leaves a
    manifest entry without its files.  ``done()`` lists the recorded row ranges for resume."""

    def __init__(self, output_dir, split=None, rank: int = 0):
        self.dir = _split_dir(output_dir, split)
        self.shards = os.path.join(self.dir, "shards")
        os.makedirs(self.shards, exist_ok=True)
        self.rank = int(rank)
        self.manifest = os.path.join(self.shards, f"manifest_r{self.rank}.json")
        self.entries = json.load(open(self.manifest)) if os.path.exists(self.manifest) else []

    def done(self) -> list:
        return [(e["row_start"], e["rows"]) for e in self.entries]

    def write(self, row_start: int, metadata_rows, embeddings: dict):
        meta = metadata_rows if isinstance(metadata_rows, pd.DataFrame) else pd.DataFrame(list(metadata_rows))
        n = len(meta)
        tag = f"r{self.rank}_{int(row_start):09d}"
        meta.to_csv(os.path.join(self.shards, f"{tag}_meta.csv"), index=False)
        for name, arr in embeddings.items():
            if arr.shape[0] != n:
                raise ValueError(f"{name}: {arr.shape[0]} rows vs {n} metadata rows")
            np.save(os.path.join(self.shards, f"{tag}_{name}.npy"), np.ascontiguousarray(arr, dtype=np.float32))
        self.entries.append({"row_start": int(row_start), "rows": n, "tag": tag, "columns": sorted(embeddings)})
        tmp = self.manifest + ".tmp"
        with open(tmp, "w") as f:
            json.dump(self.entries, f)
        os.replace(tmp, self.manifest)


def merge_shards(output_dir, split=None, expected_dim=None):
    """All ranks' manifests -> the reference layout (rows in corpus order).  Returns N."""
    d = os.path.join(output_dir, split) if split and split != "all" else output_dir
    sd = os.path.join(d, "shards")
    entries = []
    for f in sorted(os.listdir(sd)):
        if f.startswith("manifest_r") and f.endswith(".json"):
            entries += json.load(open(os.path.join(sd, f)))
    entries.sort(key=lambda e: e["row_start"])
    seen = {}
    for e in entries:                                   # a resumed rank may have re-written a range
        seen[e["row_start"]] = e
    entries = [seen[k] for k in sorted(seen)]
    pos = 0
    for e in entries:
        if e["row_start"] != pos:
            raise ValueError(f"shards leave a gap or overlap at row {pos} (next shard starts at {e['row_start']})")
        pos += e["rows"]
    cols = entries[0]["columns"] if entries else []
    meta = pd.concat([pd.read_csv(os.path.join(sd, f"{e['tag']}_meta.csv")) for e in entries], ignore_index=True)
    emb = {c: np.concatenate([np.load(os.path.join(sd, f"{e['tag']}_{c}.npy")) for e in entries]) for c in cols}
    write_split(output_dir, split, meta, emb, expected_dim)
    return pos
