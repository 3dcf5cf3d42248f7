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
# genome's full G lists (P protein iterations, each a latency chain with one
# workgroup barrier) whatever its width, then pays per column.  Fitted on
# MI355X at 10k x 100 SCPs from the 8-way shard times of candidate splits
# (tools/gpu/shard_times.py, SHARD_FRACS): with one KW for every launch,
# fixed = 0.75 n -> slowest shard 1.45 ms, 1.0 n -> 1.36, 1.25 n -> 1.32,
# 1.5 n -> 1.33, 2.0 n -> 1.43 (profiles/r02g_shard_times_10k_x8.txt); since
# each launch takes the counter words its own widest row needs, narrow
# shards got cheaper: 1.25 n -> 1.37, 1.0 n -> 1.29, 1.5 n -> 1.34
# (profiles/r02m_shard_times_10k_x8.txt).  Balancing by pairs alone gives
# the last rank (narrow rows) 2.5 ms.  Round 3's row kernel (G_end, no run
# table in the step) moved the balance toward the wide rows: 1.0 n -> 1.22,
# 0.9 n -> 1.16, 0.8 n -> 1.16, 0.7 n -> 1.15 ms (profiles/r03o/shard_times.txt).
# Round 4 (profiles/r04/shard_*.txt: 8-way shard times of seven splits, each
# block run alone on one MI355X): the narrow rows (<= 2 047 columns) run as
# 512-thread workgroups four per CU, so they cost less than the model said --
# NARROW_COST_FACTOR; the cuts of the measurement-recut split (three rounds
# of re-cutting by measured time, then a search) are met within 40 rows by
# fixed 0.68 n and narrow rows at 0.93 of their cost.
FIXED_COST_FRACTION = 0.68
NARROW_COLS = 2047
NARROW_COST_FACTOR = 0.93
# A shard of m rows runs in rounds of 2 x CUs workgroups (two 1024-thread
# row workgroups per CU), and a round's few last rows cost about half a row
# time whatever their number: at 10k x 8, 1 022 rows measured 0.95 ms and
# 1 029 or 1 044 rows 1.17-1.20 ms for neighbouring blocks (a mean of 1.10).
# With cus given, a cut that leaves a block up to ROUND_TAIL of a round past
# a whole number of rounds moves back to the round boundary (its rows go to
# the next block), and so does a cut up to ROUND_TAIL of a round past the
# first narrow row.
ROUND_TAIL = 0.25


def split_rows(n_rows: int, world: int, all_vs_all: bool = True, fixed_cols: float | None = None,
               cus: int | None = None):
    """-> [(row_begin, row_end)] * world, contiguous, covering [0, n_rows),
    balanced by the row cost model (row_costs: fixed + width for all-vs-all
    row a of width n-1-a, narrow rows scaled; QT/QSUB rows are equal).
    cus (the GPU's compute units): cuts that leave a block a few rows into
    another round of 2 * cus workgroups move back to the round boundary."""
    blocks = split_range(0, n_rows, world, n_rows, all_vs_all, fixed_cols)
    if not (cus and all_vs_all and world > 1):
        return blocks
    S = 2 * int(cus)
    edges = [0]
    for k, (_, b) in enumerate(blocks[:-1]):
        a = edges[-1]
        m = b - a
        tail = m % S
        if m > S and 0 < tail <= ROUND_TAIL * S and n_rows - 1 - (b - 1) > NARROW_COLS:
            b -= tail
        # a cut a few rows past the first narrow row moves back to it: the
        # block's narrow rows would run as their own small launch beside its
        # wide ones (10k x 8: [6460, 7988) 1.11-1.14 ms, [6421, 7952) 1.05-1.06)
        narrow0 = n_rows - 1 - NARROW_COLS
        if 0 < b - narrow0 <= ROUND_TAIL * S:
            b = narrow0
        edges.append(max(a, b))
    edges.append(n_rows)
    return [(edges[i], edges[i + 1]) for i in range(world)]


def split_range(row_lo: int, row_hi: int, parts: int, n_rows: int, all_vs_all: bool = True,
                fixed_cols: float | None = None):
    """split_rows for the sub-range [row_lo, row_hi) of an n_rows matrix
    (e.g. a rank's block cut into pipeline chunks)."""
    if not all_vs_all:
        cuts = [row_lo + (row_hi - row_lo) * r // parts for r in range(parts + 1)]
        return [(cuts[i], cuts[i + 1]) for i in range(parts)]
    import numpy as np

    cum = np.concatenate([[0.0], np.cumsum(row_costs(n_rows, True, fixed_cols))])
    c0, c1 = cum[row_lo], cum[row_hi]
    cuts = [row_lo]
    for r in range(1, parts):
        target = c0 + (c1 - c0) * r / parts
        cuts.append(int(min(max(np.searchsorted(cum, target, side="left"), cuts[-1]), row_hi)))
    cuts.append(row_hi)
    return [(cuts[i], cuts[i + 1]) for i in range(parts)]


def row_costs(n_rows: int, all_vs_all: bool = True, fixed_cols: float | None = None):
    """The model cost of every output row (numpy float64[n_rows]): fixed +
    width for all-vs-all row a (width n-1-a), 1 per row otherwise -- the
    density split_rows cuts into equal shares."""
    import numpy as np

    if not all_vs_all:
        return np.ones(n_rows)
    k = FIXED_COST_FRACTION * n_rows if fixed_cols is None else float(fixed_cols)
    width = n_rows - 1 - np.arange(n_rows, dtype=np.float64)
    c = k + width
    if fixed_cols is None:  # (an explicit fixed cost: the plain model)
        c[width <= NARROW_COLS] *= NARROW_COST_FACTOR
    return c


# Block-cyclic rows (round 6): contiguous blocks end on
# their slowest round (the first 10k/8 block is two rounds of the widest
# rows: 1.07-1.08 ms against a 0.87 ms mean), and the blocks' times sum to
# 1.18x the whole matrix's launch, which overlaps wide and narrow rows.
# Dealing groups of CYCLIC_GROUP consecutive rows round robin -- widest
# first, the direction reversing every round (snake order) -- gives every
# rank the whole matrix's mix of wide and narrow rows in ONE launch over its
# row list (pfaai_set_row_order); a group is the XCD chunk of the row kernel
# (kXcdChunk = 32 consecutive rows per XCD, sharing a clade's runs in L2).
CYCLIC_GROUP = 32


def cyclic_rows(n_rows: int, world: int, group: int = CYCLIC_GROUP):
    """-> [sorted row list] * world: groups of `group` consecutive rows dealt
    in snake order (ranks 0..W-1, then W-1..0, ...), widest (first) rows
    first.  Every row in exactly one list; each list ascending."""
    out = [[] for _ in range(world)]
    ng = (n_rows + group - 1) // group
    for k in range(ng):
        rnd, pos = divmod(k, world)
        r = pos if rnd % 2 == 0 else world - 1 - pos
        out[r].extend(range(k * group, min(n_rows, (k + 1) * group)))
    return out


def row_segments(rows):
    """Maximal runs of consecutive ids in an ascending row list -> [(lo, hi)]."""
    seg = []
    for r in rows:
        if seg and seg[-1][1] == r:
            seg[-1][1] = r + 1
        else:
            seg.append([r, r + 1])
    return [tuple(x) for x in seg]


class PipelinedGather:
    """Row blocks cut into `chunks` pipeline chunks per rank.  Chunk j of every
    rank has its own buffer (padded to the largest rank's chunk j); issue(j)
    starts an asynchronous gather of it to `dst` as soon as it is computed,
    so the transfer of chunk j over xGMI overlaps the computation of chunk
    j + 1 (RCCL runs on its own stream, ordered after the work already on
    the current stream when issue() is called).

    slots > 1 pipelines across steps as well: step i computes into buffer set
    i % slots while the gather of step i - 1 is still in flight; begin(i)
    first makes the current stream wait for the gathers that last read set
    i % slots (so a rank never overwrites a block RCCL is still sending).
    Every step still computes and gathers its whole block; wait() drains
    every outstanding gather.

    counts[r][j]: JAC entries of rank r's chunk j.  Because rank blocks and
    their chunks are contiguous row ranges in row order, and rows map to
    contiguous, increasing JAC spans (all-vs-all, QT), the concatenation
    over (r, j) of the received chunks is the full JAC-ordered vector."""

    def __init__(self, counts, dst=0, device=None, dtype=None, group=None, slots=1):
        import torch
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.dst = dst
        self.counts = counts
        self.slots = max(1, int(slots))
        nchunks = len(counts[0])
        dtype = dtype or torch.float64
        self.slot_bufs = [[torch.zeros(max(1, max(c[j] for c in counts)), dtype=dtype, device=device)
                           for j in range(nchunks)] for _ in range(self.slots)]
        self.slot_recv = [([[torch.empty_like(b) for _ in range(self.world)] for b in bufs]
                           if (self.world > 1 and self.rank == dst) else None) for bufs in self.slot_bufs]
        self.slot_works = [[] for _ in range(self.slots)]
        self.cur = 0

    @property
    def bufs(self):
        """The current step's chunk buffers."""
        return self.slot_bufs[self.cur]

    def begin(self, step):
        """Select buffer set step % slots; its previous gathers must have read it."""
        self.cur = step % self.slots
        for w in self.slot_works[self.cur]:
            w.wait()
        self.slot_works[self.cur] = []

    def issue(self, j):
        if self.world == 1:
            return
        recv = self.slot_recv[self.cur]
        self.slot_works[self.cur].append(
            self.dist.gather(self.slot_bufs[self.cur][j], recv[j] if recv else None, dst=self.dst,
                             group=self.group, async_op=True))

    def wait(self):
        for works in self.slot_works:
            for w in works:
                w.wait()
        self.slot_works = [[] for _ in range(self.slots)]

    def result(self, slot=None):
        """The full vector of buffer set `slot` (default: the current one) on
        dst (after wait()), None elsewhere."""
        import torch

        k = self.cur if slot is None else slot
        bufs = self.slot_bufs[k]
        if self.world == 1:
            return torch.cat([b[: self.counts[0][j]] for j, b in enumerate(bufs)])
        if self.rank != self.dst:
            return None
        recv = self.slot_recv[k]
        return torch.cat([recv[j][r][: self.counts[r][j]]
                          for r in range(self.world) for j in range(len(bufs))])


def jac_segments(n_ids: int, rows):
    """All-vs-all: the JAC-index spans [f, l) of an ascending row list's
    maximal runs of consecutive rows (row a's pairs start at n a - a (a + 1) / 2,
    ds_impl.hpp:83-86)."""
    base = lambda a: n_ids * a - a * (a + 1) // 2  # noqa: E731
    return [(base(lo), base(hi)) for lo, hi in row_segments(rows)]


class SegmentGather:
    """The gather of block-cyclic row lists (cyclic_rows).  Every rank runs
    its list into a full-size JAC-ordered array (the row kernel writes at the
    reference's JAC index), so rank dst's array IS the output: its own rows
    land in place, and every other rank sends the JAC segments of its rows
    straight into it -- grouped point-to-point transfers
    (torch.distributed.batch_isend_irecv: one RCCL group of ncclSend /
    ncclRecv over xGMI with the "nccl" backend, gloo on CPU) -- with no
    packing and no reorder on either side.  slots > 1 double-buffers across
    steps as PipelinedGather does: begin(i) makes the current stream wait
    for the transfers that last read buffer set i % slots.

    segs[r]: rank r's JAC segments [(f, l)]; n: n_pairs."""

    def __init__(self, segs, n, dst=0, device=None, dtype=None, group=None, slots=1):
        import torch
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.dst = dst
        self.segs = segs
        self.slots = max(1, int(slots))
        self.slot_bufs = [torch.zeros(max(1, n), dtype=dtype or torch.float64, device=device)
                          for _ in range(self.slots)]
        self.slot_works = [[] for _ in range(self.slots)]
        self.cur = 0

    @property
    def buf(self):
        """The current step's full-size array."""
        return self.slot_bufs[self.cur]

    def begin(self, step):
        self.cur = step % self.slots
        for w in self.slot_works[self.cur]:
            w.wait()
        self.slot_works[self.cur] = []

    def issue(self):
        if self.world == 1:
            return
        d, b = self.dist, self.slot_bufs[self.cur]
        if self.rank == self.dst:
            ops = [d.P2POp(d.irecv, b[f:l], r, self.group) for r in range(self.world) if r != self.dst
                   for f, l in self.segs[r] if l > f]
        else:
            ops = [d.P2POp(d.isend, b[f:l], self.dst, self.group) for f, l in self.segs[self.rank] if l > f]
        if ops:
            self.slot_works[self.cur].extend(d.batch_isend_irecv(ops))

    def wait(self):
        for works in self.slot_works:
            for w in works:
                w.wait()
        self.slot_works = [[] for _ in range(self.slots)]

    def result(self, slot=None):
        """The full vector of buffer set `slot` (default: the current one) on
        dst (after wait()), None elsewhere."""
        if self.rank != self.dst:
            return None
        return self.slot_bufs[self.cur if slot is None else slot]


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
