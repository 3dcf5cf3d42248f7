"""Row-block sharding of the AJI matrix over ranks.

Every output pair is independent; the only exchange is the final gather.
Rank r owns a contiguous block of output rows, balanced by pair count
(all-vs-all row a owns n-1-a pairs; QT/QSUB rows own equal counts), runs the
hot path on it (pfaai_run(row_begin, row_end)) and rank 0 gathers the fp64
AJI blocks -- one torch.distributed.gather, which is an RCCL gather over
xGMI with the "nccl" backend (gloo on CPU in the tests).
"""
from __future__ import annotations


def split_rows(n_rows: int, world: int, all_vs_all: bool = True):
    """-> [(row_begin, row_end)] * world, contiguous, covering [0, n_rows)."""
    if not all_vs_all:
        cuts = [n_rows * r // world for r in range(world + 1)]
        return [(cuts[i], cuts[i + 1]) for i in range(world)]
    n = n_rows

    def before(a):  # pairs in rows < a of the upper triangle
        return a * n - a * (a + 1) // 2

    total = n * (n - 1) // 2
    cuts = [0]
    for r in range(1, world):
        target = total * r // world
        lo, hi = cuts[-1], n
        while lo < hi:
            mid = (lo + hi) // 2
            if before(mid) < target:
                lo = mid + 1
            else:
                hi = mid
        cuts.append(lo)
    cuts.append(n)
    return [(cuts[i], cuts[i + 1]) for i in range(world)]


def gather_rows(out_local, counts, dst=0, group=None):
    """Gather every rank's AJI block (a 1-D tensor padded to max(counts)) to
    `dst`; returns the concatenated full vector on dst, None elsewhere."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if world == 1:
        return out_local[: counts[0]]
    bufs = [torch.empty_like(out_local) for _ in range(world)] if rank == dst else None
    dist.gather(out_local, bufs, dst=dst, group=group)
    if rank != dst:
        return None
    return torch.cat([bufs[r][: counts[r]] for r in range(world)])
