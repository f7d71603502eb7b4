"""Chunk-parallel sharding of a ChunkedArray across ranks (one process per GPU).

The reference canonicalizes a ChunkedArray serially (array/chunked/canonical.rs:27-122,
pack_primitives :170-187).  Chunks are independent, so on an 8x MI355X node each rank owns a
CONTIGUOUS range of chunks, balanced by compressed bytes, and decodes it straight into its
slice of the packed output; chunk i's output element offset is chunk_offsets[i]
(array/chunked/mod.rs:54-70).  No data crosses xGMI: the only collective is the barrier that
closes a timed region.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np

from . import arrays as A
from ._lib import ENC


def plan_shards(weights: Sequence[int], world: int) -> list[range]:
    """Contiguous chunk ranges, one per rank, cutting where the running compressed-byte total
    crosses r * total / world.  Every chunk is assigned exactly once; ranks may be empty when
    there are fewer chunks than ranks."""
    w = np.asarray(weights, dtype=np.float64)
    n = len(w)
    if world < 1:
        raise ValueError("world must be >= 1")
    cum = np.concatenate([[0.0], np.cumsum(w)])
    total = cum[-1]
    cuts = [0]
    for r in range(1, world):
        target = total * r / world
        c = int(np.searchsorted(cum, target, side="left"))
        c = min(max(c, cuts[-1]), n)
        cuts.append(c)
    cuts.append(n)
    return [range(cuts[r], cuts[r + 1]) for r in range(world)]


def rank_shard(chunked: A.Array, rank: int, world: int):
    """-> (sub-ChunkedArray of this rank's chunks or None, first output element, length)."""
    if chunked.encoding != ENC["CHUNKED"]:
        raise A.VortexError(3, "rank_shard expects a ChunkedArray")
    chunks = chunked.children[1:]
    offsets = np.concatenate([[0], np.cumsum([c.len for c in chunks])]).astype(np.int64)
    r = plan_shards([c.nbytes() for c in chunks], world)[rank]
    if len(r) == 0:
        return None, int(offsets[r.start]) if r.start < len(offsets) else int(offsets[-1]), 0
    sub = A.chunked([chunks[i] for i in r])
    return sub, int(offsets[r.start]), int(offsets[r.stop] - offsets[r.start])
