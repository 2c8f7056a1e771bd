"""Row sharding of the packed lower triangle across ranks:
`dist` pairs are independent, so rank g computes LT rows [r_g, r_{g+1}) with
ccg_snp_ltd(_dev)'s row range and the blocks are gathered in rank order.
Boundaries equalise the cells per rank (r_g ~ n*sqrt(g/G))."""
from __future__ import annotations

import math

import numpy as np


def lt_cells(r):
    """Cells of LT rows [0, r)."""
    return r * (r - 1) // 2


def lt_row_ranges(n, world):
    """Contiguous row ranges [(r0, r1)] covering rows 1..n-1 with nearly equal
    cell counts per rank (row 0 has no cells)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    total = lt_cells(n)
    bounds = [0]
    for g in range(1, world):
        # smallest r with cells(r) >= g/world * total
        target = total * g / world
        r = int(math.ceil((1 + math.sqrt(1 + 8 * target)) / 2))
        while r > 0 and lt_cells(r - 1) >= target:
            r -= 1
        bounds.append(min(max(r, bounds[-1]), n))
    bounds.append(n)
    return [(bounds[g], bounds[g + 1]) for g in range(world)]


def gather_lt(part, rows, n, dist):
    """All ranks' LT row blocks -> the full packed LT on every rank.
    `part` holds this rank's cells of rows [rows[0], rows[1]) in reference
    order; `dist` is torch.distributed (gloo on CPU, RCCL on GPU)."""
    import torch
    world = dist.get_world_size()
    ranges = lt_row_ranges(n, world)
    assert tuple(rows) == ranges[dist.get_rank()], "rank's rows must follow lt_row_ranges"
    sizes = [lt_cells(r1) - lt_cells(r0) for r0, r1 in ranges]
    width = max(sizes) if sizes else 0
    t = torch.zeros(width, dtype=torch.from_numpy(np.zeros(0, part.dtype)).dtype)
    t[: len(part)] = torch.from_numpy(np.ascontiguousarray(part))
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return np.concatenate([o[:s].numpy() for o, s in zip(out, sizes)])


def reduce_max(x, dist):
    """Max of a float over ranks (bench.py's timed-region reduction)."""
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0])


def reduce_sum(x, dist):
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t[0])
