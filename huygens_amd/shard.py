"""Partitioning of a bank across ranks (one process per GPU).

Every bank on the path is a sum of independent units -- bands (Filterbank), partials
(Oscbank), overtones of every voice (Additive), modes (Bowl), lines (Delaybank) -- so a
rank owns a contiguous range of units and the mixes are summed with one reduce per call.
"""
from __future__ import annotations


def shard_of(rank: int, world: int, n_units: int) -> tuple[int, int]:
    """(first unit, unit count) of `rank`: contiguous, sizes differ by at most one."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("rank must be in [0, world)")
    base, rem = divmod(n_units, world)
    begin = rank * base + min(rank, rem)
    return begin, base + (1 if rank < rem else 0)
