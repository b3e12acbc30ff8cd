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


def set_time_shards(fb, rank: int, world: int, all_reduce_sum, all_reduce_max) -> bool:
    """Stationary Filterbank calls split by TIME over the ranks (hz_fb_set_time_shard): the
    whole bank's response is the sum of the band shards' responses over the largest horizon of
    the ranks (`all_reduce_sum(array) -> array`, `all_reduce_max(int) -> int`, e.g. RCCL
    all-reduces), set on every rank; each rank then convolves its run of output blocks and keeps
    its own bands' states.  Call after the last setter (setters clear it), on every rank.

    Collective-safe: every rank takes part in both all-reduces whatever its own shard can do (a
    shard without a finite horizon -- or whose horizon probe fails -- contributes a sentinel), so
    the ranks either all set the shards or all return False.  The handles then still need arming
    (arm_when_ready) before a call runs stationary."""
    import numpy as np
    none = 1 << 30   # no finite horizon on this shard (> the 2^19 the engine supports)
    try:
        fb.response(8192)   # computes the shard's horizon
        K = int(fb.response_info()[0])
    except Exception:  # noqa: BLE001 -- e.g. HZ_E_UNSUPPORTED: no horizon within 2^18 samples
        K = -1
    K_all = int(all_reduce_max(K if K > 0 else none))
    if K_all <= 0 or K_all > (1 << 19):
        return False   # every rank sees the same K_all: all leave here, no collective pending
    try:
        mine = np.ascontiguousarray(fb.response(K_all), dtype=np.float64)
        ok = True
    except Exception:  # noqa: BLE001 -- keep the collective matched, then fail together
        mine = np.zeros(K_all)
        ok = False
    full = np.asarray(all_reduce_sum(mine), dtype=np.float64)
    # agreement on success (a rank that failed after the horizon probe poisons the sum)
    if int(all_reduce_max(0 if ok else 1)) != 0:
        return False
    fb.set_bank_response(full)
    fb.set_time_shard(rank, world)
    return True


def arm_when_ready(fb, n: int, all_reduce_min) -> bool:
    """Arms the time-sharded handles of ALL ranks for the stationary engine in the same call, or
    none: every rank asks whether a call of n samples would be stationary on its own handle
    (hz_fb_stationary_ready; it depends on the shard's convergence and history), the flags are
    all-reduced with MIN (`all_reduce_min(int) -> int`) and the result armed on every rank.
    Collective: call on every rank between the same two calls.  Returns whether armed."""
    ready = 1 if fb.stationary_ready(n) else 0
    armed = int(all_reduce_min(ready)) == 1
    fb.arm_time_shard(armed)
    return armed


def time_share(rank: int, world: int, n: int, block: int = 2048) -> tuple[int, int]:
    """(first sample, count) of rank's share of a time-sharded stationary call of n samples: a
    run of whole `block`-sample output blocks (the split of hz_fb_time_shard_info)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("rank must be in [0, world)")
    nb = -(-n // block)
    lo = min(n, nb * rank // world * block)
    hi = min(n, nb * (rank + 1) // world * block)
    return lo, hi - lo


class ShareGather:
    """Assembles the ranks' time shares of a call's output on rank 0: every rank copies its share
    into a fixed-size slot (the largest share), one gather moves the slots to rank 0, which copies
    them into place.  `y` is the call's output buffer on every rank (torch tensor)."""

    def __init__(self, n: int, rank: int, world: int, like, block: int = 2048):
        import torch
        self.n, self.rank, self.world = n, rank, world
        self.shares = [time_share(r, world, n, block) for r in range(world)]
        self.slot = max(c for _, c in self.shares)
        self.buf = torch.zeros(self.slot, dtype=like.dtype, device=like.device)
        self.bufs = [torch.empty_like(self.buf) for _ in range(world)] if rank == 0 else None

    def __call__(self, y, dist):
        self.start(y, dist)
        self.finish(y)

    def start(self, y, dist, async_op=False):
        """copy this rank's share into the slot and issue the gather (async_op: returns its work
        handle; call finish(y) after it completed)"""
        f, c = self.shares[self.rank]
        self.buf[:c].copy_(y[f:f + c])
        return dist.gather(self.buf, self.bufs, dst=0, async_op=async_op) if async_op else \
            dist.gather(self.buf, self.bufs, dst=0)

    def finish(self, y):
        """(rank 0) the gathered slots into place in y"""
        if self.rank == 0:
            for (f, c), b in zip(self.shares, self.bufs):
                y[f:f + c].copy_(b[:c])
