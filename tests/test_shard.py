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


# ---------------------------------------------------------------- sharded tree
def _band_off(r, rank, world, SB=8):
    """Elements before owned row r: owned bands below r's band, then r's
    predecessors in its band (the layout ccg_tree_shard_dev consumes)."""
    acc = 0
    for q in range(r):
        if (q // SB) % world == rank:
            acc += q
    return acc


@pytest.mark.parametrize("world", [1, 2, 3, 4, 5, 8])
def test_shard_layout(world):
    from ccphylo_amd import native as nt
    for n in (3, 7, 8, 9, 16, 17, 64, 65, 100, 257):
        total = 0
        for rank in range(world):
            rows = [r for r in range(n) if nt.shard_owner(r, world) == rank]
            for r in rows:
                assert nt.shard_row_offset(r, rank, world) == _band_off(r, rank, world)
            assert nt.shard_elems(n, rank, world) == sum(rows)
            total += sum(rows)
        assert total == n * (n - 1) // 2


def test_shard_extract_roundtrip():
    from ccphylo_amd import native as nt
    n, world = 131, 3
    D = np.arange(n * (n - 1) // 2, dtype=np.float64)
    parts = [nt.shard_extract(D, n, r, world) for r in range(world)]
    back = np.full_like(D, -1)
    for rank, p in enumerate(parts):
        for r in range(1, n):
            if nt.shard_owner(r, world) == rank:
                o = nt.shard_row_offset(r, rank, world)
                back[r * (r - 1) // 2:r * (r + 1) // 2] = p[o:o + r]
    assert np.array_equal(back, D)


def _coll_main(rank, world, port, out_dir):
    """The host-staged transport exactly as the engine drives it: C function
    pointers of a ccg_coll called on host buffers."""
    import ctypes as C
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from ccphylo_amd import native as nt
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    hc = nt.HostColl(dist)
    n = 301
    line = np.arange(1, n + 1, dtype=np.float64) * 1.25
    # lines i/j exchange: every rank holds the entries of its own bands, zeros elsewhere
    mine = np.array([line[k] if nt.shard_owner(k, world) == rank else 0.0 for k in range(n)])
    buf = np.ascontiguousarray(mine)
    rc = hc.c.allreduce_sum_u8(None, buf.ctypes.data, buf.nbytes, None)
    ok = rc == 0 and np.array_equal(buf, line)
    # row n-1 broadcast from its owner
    root = nt.shard_owner(n - 1, world)
    src = np.arange(n, dtype=np.uint16) * 3
    dst = np.zeros(n, np.uint16)
    rc = hc.c.broadcast(None, src.ctypes.data if rank == root else None, dst.ctypes.data, dst.nbytes, root, None)
    ok = ok and rc == 0 and np.array_equal(dst, src) and not hc.errors
    np.save(os.path.join(out_dir, f"c{rank}.npy"), np.array([ok, hc.calls]))
    dist.barrier()
    dist.destroy_process_group()


def test_host_coll_gloo_world2(tmp_path):
    world = 2
    mp.start_processes(_coll_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    for r in range(world):
        ok, calls = np.load(tmp_path / f"c{r}.npy")
        assert ok and calls == 2
