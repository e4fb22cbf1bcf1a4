"""Read sharding over GPUs: one process per GPU, contiguous
read ranges balanced by bases, no collective on the data path, PAF gathered
in input order afterwards (the reference maps reads independently, Q10, so
the concatenation equals a single-process run).

Used by multi-process callers (``mm2rs``-style drivers, tests/test_multirank.py);
bench.py's weak-scaling run gives every rank its own reads instead.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np


def shard_cuts(lens: Sequence[int], world: int) -> List[int]:
    """Contiguous read ranges [cuts[r], cuts[r+1]) for `world` ranks with
    about equal numbers of bases each (reads are never split)."""
    world = max(1, int(world))
    n = len(lens)
    if n == 0:
        return [0] * (world + 1)
    c = np.concatenate([[0], np.cumsum(np.asarray(lens, dtype=np.int64))])
    total = int(c[-1])
    cuts = [0]
    for r in range(1, world):
        # first read whose start reaches r/world of the bases
        cuts.append(max(cuts[-1], int(np.searchsorted(c, total * r / world, side="left"))))
    cuts.append(n)
    return [min(x, n) for x in cuts]


def gather_paf(dist, paf: bytes, rank: int, world: int) -> bytes:
    """All ranks' PAF text concatenated in rank order (= input order for
    shard_cuts ranges) on rank 0; b"" elsewhere.  Outside any timed region."""
    if world <= 1:
        return paf
    got = [None] * world if rank == 0 else None
    dist.gather_object(paf, got, dst=0)
    return b"".join(got) if rank == 0 else b""
