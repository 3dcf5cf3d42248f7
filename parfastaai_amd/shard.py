"""Row-block sharding of the AJI matrix over ranks.

Every output pair is independent; the only exchange is the final gather.
Rank r owns a contiguous block of output rows, balanced by a per-row cost
model (split_rows: fixed + width for all-vs-all; equal rows for QT/QSUB),
runs the hot path on it (pfaai_run(row_begin, row_end)) and rank 0 gathers the fp64
AJI blocks -- one torch.distributed.gather, which is an RCCL gather over
xGMI with the "nccl" backend (gloo on CPU in the tests).
"""
from __future__ import annotations


# Device time of an all-vs-all row ~ (fixed + width): every row walks its
# genome's full G lists (P protein iterations, each a latency chain) whatever
# its width, then pays per column.  Measured on MI355X at 10k x 100 SCPs
# (tools/gpu/ab_rows.py --rows): 2000 rows of mean width 9000 take 3.65 ms,
# 2000 rows of mean width 1000 take 1.90 ms, i.e. fixed ~ 0.77 x n columns.
# Balancing by pairs alone would give the last rank (narrow rows) ~3x the
# time of the first.
FIXED_COST_FRACTION = 0.75


def split_rows(n_rows: int, world: int, all_vs_all: bool = True, fixed_cols: float | None = None):
    """-> [(row_begin, row_end)] * world, contiguous, covering [0, n_rows),
    balanced by the row cost model fixed_cols + width (all-vs-all row a has
    width n-1-a; QT/QSUB rows are equal)."""
    if not all_vs_all:
        cuts = [n_rows * r // world for r in range(world + 1)]
        return [(cuts[i], cuts[i + 1]) for i in range(world)]
    n = n_rows
    k = FIXED_COST_FRACTION * n if fixed_cols is None else float(fixed_cols)

    def before(a):  # cost of rows < a: a fixed parts + the pairs of the upper triangle
        return a * k + a * n - a * (a + 1) // 2

    total = before(n)
    cuts = [0]
    for r in range(1, world):
        target = total * r / world
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
