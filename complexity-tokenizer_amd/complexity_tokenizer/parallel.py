"""Document sharding across GPUs (one process per GPU).

The encode path has no exchange step: documents are independent (the reference maps them with
rayon's order-preserving par_iter, src/huggingface/mod.rs:694-696).  A batch is cut into
contiguous, byte-balanced document ranges, one per rank; each rank encodes its range on its own
GPU; when the caller wants the whole result on one rank, the per-rank (ids, tok_off) pieces are
concatenated with their token offsets rebased.  No collective touches the data path unless the
caller asks for the gather.
"""
from __future__ import annotations

import numpy as np


def shard_bounds(off: np.ndarray, world: int, rank: int) -> tuple[int, int]:
    """Doc range [d0, d1) of `rank`: cuts at the first doc start >= k * total_bytes / world."""
    off = np.asarray(off, dtype=np.uint64)
    n_docs = len(off) - 1
    total = int(off[-1])
    if world <= 1:
        return 0, n_docs
    cuts = [0]
    for k in range(1, world):
        target = (total * k) // world
        cuts.append(int(np.searchsorted(off[:-1], np.uint64(target), side="left")))
    cuts.append(n_docs)
    for k in range(1, len(cuts)):  # monotone even when many docs are empty
        cuts[k] = max(cuts[k], cuts[k - 1])
    return cuts[rank], cuts[rank + 1]


def local_shard(text: np.ndarray, off: np.ndarray, world: int, rank: int):
    """(text slice, rebased offsets) of this rank's shard."""
    d0, d1 = shard_bounds(off, world, rank)
    b0, b1 = int(off[d0]), int(off[d1])
    return text[b0:b1], (np.asarray(off[d0:d1 + 1], dtype=np.uint64) - np.uint64(b0)), (d0, d1)


def concat_results(parts):
    """[(ids, tok_off), ...] in rank order -> one (ids, tok_off) with offsets rebased."""
    ids = np.concatenate([np.asarray(p[0], dtype=np.uint32) for p in parts]) if parts else np.zeros(0, np.uint32)
    offs = [np.zeros(1, dtype=np.uint64)]
    base = np.uint64(0)
    for _, toff in parts:
        toff = np.asarray(toff, dtype=np.uint64)
        offs.append(toff[1:] + base)
        base = base + toff[-1]
    return ids, np.concatenate(offs)


def encode_sharded(encode_fn, text, off, rank: int, world: int, gather: bool = True, group=None):
    """Encode this rank's shard with encode_fn(text, off) -> (ids, tok_off); with gather=True
    return the whole batch's (ids, tok_off) on every rank (torch.distributed all_gather_object),
    else this rank's part and its doc range."""
    t, o, (d0, d1) = local_shard(text, off, world, rank)
    ids, toff = encode_fn(t, o)
    if not gather or world == 1:
        return ids, toff, (d0, d1)
    import torch.distributed as dist
    parts = [None] * world
    dist.all_gather_object(parts, (np.asarray(ids), np.asarray(toff)), group=group)
    ids_all, toff_all = concat_results(parts)
    return ids_all, toff_all, (0, len(off) - 1)
