"""CPU, world_size 2 (gloo): the multi-rank pieces -- LT row sharding of
`dist` with a rank-ordered gather, and bench.py's max/sum reductions.  The
per-rank compute is the oracle here (no GPU); on the box each rank calls
ccg_snp_ltd_dev with the same row range."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, n, L, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from ccphylo_amd import shard
    from oracle import pyoracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(11)
    W = L // 32 + 1
    seqs = rng.integers(0, 2**63, size=(n, W), dtype=np.uint64)
    incs = np.full(W, 0xFFFFFFFF, np.uint32)
    full, _, _ = pyoracle.snp_ltd(seqs, incs, n, L)
    r0, r1 = shard.lt_row_ranges(n, world)[rank]
    part = full[shard.lt_cells(r0):shard.lt_cells(r1)]      # this rank's rows (engine: row_begin/row_end)
    got = shard.gather_lt(part, (r0, r1), n, dist)
    mx = shard.reduce_max(rank + 1.5, dist)
    sm = shard.reduce_sum(rank + 1, dist)
    np.save(os.path.join(out_dir, f"r{rank}.npy"), np.concatenate([got, [mx, sm]]))
    ok = np.array_equal(got, full)
    dist.barrier()
    dist.destroy_process_group()
    if not ok:
        raise SystemExit(1)


@pytest.mark.parametrize("n,world", [(2, 1), (7, 3), (100, 4), (1000, 8)])
def test_row_ranges_cover_and_balance(n, world):
    from ccphylo_amd import shard
    rr = shard.lt_row_ranges(n, world)
    assert rr[0][0] == 0 and rr[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(rr, rr[1:]))
    cells = [shard.lt_cells(r1) - shard.lt_cells(r0) for r0, r1 in rr]
    assert sum(cells) == shard.lt_cells(n)
    if n >= 100:
        assert max(cells) - min(cells) <= 2 * n   # each boundary within one row


def test_gloo_world2_dist_shards(tmp_path):
    n, L, world = 157, 3000, 2
    mp.start_processes(_rank_main, args=(world, _free_port(), n, L, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    r0 = np.load(tmp_path / "r0.npy")
    r1 = np.load(tmp_path / "r1.npy")
    assert np.array_equal(r0, r1)
    assert r0[-2] == 2.5 and r0[-1] == 3.0
