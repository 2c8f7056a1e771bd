"""GPU parity of the row-sharded NJ and DNJ engines (ccg_tree_shard).

Its joins must be bit-identical to the single-GPU engine's (and so, in exact
mode, to the reference's) for every world size:
- world 1 without a transport;
- world 2 / 3 as separate processes on the one GPU, exchanging over the
  host-staged gloo transport (HostColl);
- world 1 over RCCL (the production transport; more ranks need more GPUs).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import GOLDEN, ROOT, golden_bytes, golden_cases, parse_tree_args

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import ccphylo_amd as cg
    d = cg.Device(0)
    yield d
    d.close()


@pytest.fixture(autouse=True)
def _sharded_kernels_at_world1(monkeypatch):
    """World 1 normally runs the single-GPU engine (nothing to exchange);
    these tests compare the sharded kernels with it, so they force them."""
    monkeypatch.setenv("CCG_SHARD_FORCE", "1")


def _euclid(n, seed, dim=8):
    rng = np.random.default_rng(seed)
    pts = rng.random((n, dim))
    i, j = np.tril_indices(n, -1)
    return np.sqrt(((pts[i] - pts[j]) ** 2).sum(1))


def _snp(n, seed, L=3000):
    rng = np.random.default_rng(seed)
    X = rng.integers(0, 4, (n, L))
    X[rng.random((n, L)) < 0.7] = 0        # shared sites: many equal distances
    i, j = np.tril_indices(n, -1)
    same = sum((X == c).astype(np.float64) @ (X == c).astype(np.float64).T for c in range(4))
    return L - same[i, j]                  # differing sites (exact integers in f64)


def _typed(D, et):
    bs = {8: 1.0, 4: 1.0, 2: 4.0, 1: 1.0}[et]
    if et == 8:
        return D, bs
    if et == 4:
        return D.astype(np.float32), bs
    return np.clip(D * bs + 0.5, 0, 255 if et == 1 else 65535).astype(np.uint8 if et == 1 else np.uint16), bs


def _same(a, b):
    (ja, fa, da), (jb, fb, db) = a, b
    assert (fa, da) == (fb, db)
    assert len(ja) == len(jb)
    assert (ja == jb).all()


def _clade(n, seed, L=4000, clades=24):
    """clade-structured SNP distances (config-3-like): DNJ's minQpair
    qualifies many rows per join, past the LDS replay table"""
    rng = np.random.default_rng(seed)
    roots = rng.integers(0, 4, (clades, L))
    X = roots[rng.integers(0, clades, n)]
    flip = rng.random((n, L)) < 0.01
    X = np.where(flip, rng.integers(0, 4, (n, L)), X)
    same = sum((X == c).astype(np.float64) @ (X == c).astype(np.float64).T for c in range(4))
    i, j = np.tril_indices(n, -1)
    return L - same[i, j]


def _data(kind, n):
    return {"euc": _euclid, "snp": _snp, "clade": _clade}[kind](n, n)


@pytest.mark.parametrize("method", [0, 1, 2], ids=["nj", "dnj", "hnj"])
@pytest.mark.parametrize("n,kind,et,exact", [(600, "euc", 8, True), (600, "euc", 8, False), (1100, "snp", 8, True),
                                             (700, "snp", 4, True), (700, "snp", 2, False), (500, "snp", 1, True),
                                             (2100, "euc", 8, False), (3000, "clade", 8, True)])
def test_shard_world1_matches_single(dev, n, kind, et, exact, method):
    D, bs = _typed(_data(kind, n), et)
    ref = dev.tree(D, n, etype=et, byte_scale=bs, method=method, exact=exact)[:3]
    got = dev.tree_shard(D, n, None, etype=et, byte_scale=bs, method=method, exact=exact)[:3]
    _same(got, ref)


# miss80 and multi.phy's second matrix hold missing entries (CCG_EUNSUP below)
@pytest.mark.parametrize("case", [c for c in golden_cases("tree") if not c["name"].startswith(("miss", "multi"))],
                         ids=lambda c: c["name"])
def test_shard_golden(dev, case):
    import ccphylo_amd as cg
    path, method, et, bs, flags, prec = parse_tree_args(case["args"])

    def run(D, n):
        joins, fn, fd, _ = dev.tree_shard(D, n, None, etype=et, byte_scale=bs, method=method, flags=flags)
        return joins, fn, fd
    trees = cg.newick_from_phylip(path, run, etype=et, byte_scale=bs, flags=flags, precision=prec)
    assert ("\n".join(trees) + "\n").encode() == golden_bytes(case)


def test_shard_refuses_missing(dev):
    """missing (negative) entries: updateD's quirks run on one GPU only"""
    import ccphylo_amd as cg
    n = 50
    D = _euclid(n, 1)
    D[17] = -1.0
    for method in (0, 1, 2):
        with pytest.raises(cg.CcgError, match="not supported"):
            dev.tree_shard(D, n, None, method=method)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, n, kind, et, exact, transport, method, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    import ccphylo_amd as cg
    from ccphylo_amd import native as nt
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["CCG_SHARD_FORCE"] = "1"   # world 1 over RCCL: the sharded kernels, not the single engine
    dist.init_process_group("gloo", rank=rank, world_size=world)
    D, bs = _typed(_data(kind, n), et)
    dev = cg.Device(0)
    coll = nt.HostColl(dist, allgather_native=transport != "gloo-noag") if transport.startswith("gloo") \
        else nt.RcclColl(dev, dist)
    if transport.startswith("gloo"):
        joins, fn, fd, st = dev.tree_shard(D, n, coll, etype=et, byte_scale=bs, method=method, exact=exact)
    else:
        loc = nt.shard_extract(D, n, rank, world)
        p = dev.malloc(max(loc.nbytes, 1))
        dev.h2d(p, loc)
        joins, fn, fd, st = dev.tree_shard_dev(p, n, coll, etype=et, byte_scale=bs, method=method, exact=exact)
        dev.free(p)
        coll.close()
    np.save(os.path.join(out_dir, f"j{rank}.npy"), joins)
    np.save(os.path.join(out_dir, f"f{rank}.npy"), np.array([fn, fd]))
    dev.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n,kind,et,exact,transport,method", [(2, 700, "euc", 8, True, "gloo", 0),
                                                                    (3, 450, "snp", 8, True, "gloo", 0),
                                                                    (2, 400, "snp", 2, False, "gloo", 0),
                                                                    (1, 900, "euc", 8, True, "rccl", 0),
                                                                    (2, 700, "euc", 8, True, "gloo", 1),
                                                                    (3, 500, "snp", 8, True, "gloo", 1),
                                                                    (2, 400, "snp", 2, False, "gloo", 1),
                                                                    (3, 1200, "clade", 4, True, "gloo", 1),
                                                                    # ccg_coll.allgather NULL: emulated by the allreduce
                                                                    (3, 600, "euc", 4, True, "gloo-noag", 1),
                                                                    (2, 700, "euc", 8, True, "gloo-noag", 0),
                                                                    (1, 900, "euc", 8, True, "rccl", 1),
                                                                    # world 8, the driver's node size, rehearsed as 8
                                                                    # processes on the one GPU
                                                                    (8, 1200, "euc", 8, True, "gloo", 1),
                                                                    (8, 800, "snp", 8, True, "gloo", 0),
                                                                    # HNJ (hclust.c:1671) over the row shards
                                                                    (2, 700, "euc", 8, True, "gloo", 2),
                                                                    (3, 450, "snp", 8, True, "gloo", 2),
                                                                    (2, 400, "snp", 2, False, "gloo", 2),
                                                                    (1, 900, "euc", 8, True, "rccl", 2),
                                                                    (8, 800, "snp", 8, True, "gloo", 2)])
def test_shard_multiprocess(dev, tmp_path, world, n, kind, et, exact, transport, method):
    D, bs = _typed(_data(kind, n), et)
    ref_j, ref_fn, ref_fd, _ = dev.tree(D, n, etype=et, byte_scale=bs, method=method, exact=exact)
    mp.start_processes(_rank_main, args=(world, _free_port(), n, kind, et, exact, transport, method, str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    for r in range(world):
        j = np.load(tmp_path / f"j{r}.npy")
        fn, fd = np.load(tmp_path / f"f{r}.npy")
        assert (int(fn), fd) == (ref_fn, ref_fd)
        assert len(j) == len(ref_j) and (j == ref_j).all()


@pytest.mark.parametrize("world,kind,et,mode", [(1, "euc", 8, "9"), (1, "clade", 4, "20"), (3, "euc", 8, "9"),
                                                (2, "clade", 4, "20"), (8, "euc", 8, "9")])
def test_shard_block_bounds(dev, monkeypatch, tmp_path, world, kind, et, mode):
    """The sharded engine's scan under the block lower bounds (a line per
    owned row, kept by k_shd_join / k_shd_requeue; thresholds and the plan's
    band partner-cell bound from the requeue): at small n through
    CCG_LB_MIN_N the joins equal the single engine's (itself equal to the
    oracle with the bounds, test_dnj_block_bounds), and at world 1 the bounded
    scan loads fewer cells than the unbounded one."""
    for k, v in (("CCG_SCAN_WAVE", mode), ("CCG_SEG_MUL", "1"), ("CCG_S_SPLIT_N", "100"), ("CCG_LB_MIN_N", "100")):
        monkeypatch.setenv(k, v)
    n = {1: 2500, 2: 1800, 3: 2000, 8: 1500}[world]   # (every rank process builds D itself: small kinds at world 8)
    D, bs = _typed(_data(kind, n), et)
    monkeypatch.setenv("CCG_SCAN_LB", "0")
    ref = dev.tree(D, n, etype=et, byte_scale=bs, method=1, exact=True)[:3]
    cells = {}
    for lb in ("1", "0"):
        monkeypatch.setenv("CCG_SCAN_LB", lb)
        if world == 1:
            j, fn, fd, st = dev.tree_shard(D, n, None, etype=et, byte_scale=bs, method=1, exact=True, profile=True)
            _same((j, fn, fd), ref)
            cells[lb] = st[1]
        elif lb == "1":
            mp.start_processes(_rank_main, args=(world, _free_port(), n, kind, et, True, "gloo", 1, str(tmp_path)),
                               nprocs=world, join=True, start_method="spawn")
            for r in range(world):
                fn, fd = np.load(tmp_path / f"f{r}.npy")
                _same((np.load(tmp_path / f"j{r}.npy"), int(fn), fd), ref)
    if world == 1:
        assert cells["1"] < cells["0"], cells


@pytest.mark.parametrize("kind,et,n,max_hard", [("snp", 8, 1500, 0), ("clade", 4, 1200, 0), ("snp", 2, 900, 0),
                                                 ("euc", 4, 2000, 100), ("euc", 8, 1600, 1600)])
@pytest.mark.parametrize("method", [0, 1], ids=["nj", "dnj"])
def test_shard_init_exact_columns(dev, kind, et, n, max_hard, method):
    """initSummaD's column parts (nj.c:111) without gathering the matrix:
    integer SNP counts and float distances take the exact per-rank
    statistics path (stats[9+2N]: columns left for the serial gather), only
    %.9f-like doubles need the serial gather; the joins equal the single-GPU
    engine's (exact row sums) either way."""
    import ccphylo_amd as cg
    D, bs = _typed(_data(kind, n), et)
    ref = dev.tree(D, n, etype=et, byte_scale=bs, method=method, exact=True)[:3]
    j, fn, fd, st = dev.tree_shard(D, n, None, etype=et, byte_scale=bs, method=method, exact=True, profile=True)
    _same((j, fn, fd), ref)
    hard, init_bytes = st[9 + 2 * cg.native.NKSTAT], st[8 + 2 * cg.native.NKSTAT]
    assert hard <= max_hard, hard
    if hard == 0:
        assert init_bytes == 28 * n + 16, init_bytes   # row parts + one n x 16 B statistics slot


def test_max_joins_prefix(dev):
    """max_joins stops both engines after a prefix of the same join list."""
    n, k = 500, 37
    D = _euclid(n, 5)
    full = dev.tree(D, n, method=0)[0]
    for fn in (lambda: dev.tree(D, n, method=0, max_joins=k), lambda: dev.tree(D, n, method=1, max_joins=k),
               lambda: dev.tree_shard(D, n, None, method=0, max_joins=k),
               lambda: dev.tree_shard(D, n, None, method=1, max_joins=k)):
        j, fin, fd, _ = fn()
        assert len(j) == k and fin == n - k and fd == -1.0
    j = dev.tree_shard(D, n, None, method=0, max_joins=k)[0]
    assert (j == full[:k]).all()
    fullq = dev.tree(D, n, method=1)[0]
    j = dev.tree_shard(D, n, None, method=1, max_joins=k)[0]
    assert (j == fullq[:k]).all()


def test_shard_hnj_prefix_and_ties(dev):
    """Sharded HNJ (k_sh_hnj_argmin / k_sh_hnj): max_joins prefixes of the
    single engine's join list, and a matrix of equal entries (minQ's `<=`
    rule, hclust.c:353, and the column rules' ties decide every join)."""
    import ccphylo_amd as cg
    n, k = 500, 37
    D = _euclid(n, 5)
    full = dev.tree(D, n, method=cg.CCG_TREE_HNJ)[0]
    j, fin, fd, _ = dev.tree_shard(D, n, None, method=cg.CCG_TREE_HNJ, max_joins=k)
    assert len(j) == k and fin == n - k and fd == -1.0 and (j == full[:k]).all()
    for et in (8, 1):
        E = np.full(300 * 299 // 2, 7.0)
        E, bs = _typed(E, et)
        _same(dev.tree_shard(E, 300, None, etype=et, byte_scale=bs, method=cg.CCG_TREE_HNJ)[:3],
              dev.tree(E, 300, etype=et, byte_scale=bs, method=cg.CCG_TREE_HNJ)[:3])


@pytest.mark.parametrize("method", [0, 1, 2], ids=["nj", "dnj", "hnj"])
def test_shard_world1_runs_single_engine(dev, monkeypatch, method):
    """Without CCG_SHARD_FORCE, world 1 (no transport) is the single-GPU
    engine on the same buffer: missing entries (updateD's quirks,
    nj.c:1021-1030) and -m hnj work, with its joins."""
    monkeypatch.delenv("CCG_SHARD_FORCE")
    n = 300
    D = _euclid(n, 9)
    D[[17, 4000, 9000]] = -1.0
    ref = dev.tree(D, n, method=method, exact=True)[:3]
    got = dev.tree_shard(D, n, None, method=method, exact=True)[:3]
    _same(got, ref)


def _rand_msa(n, L, seed):
    rng = np.random.default_rng(seed)
    W = L // 32 + 1
    base = rng.integers(0, 2 ** 63, size=W, dtype=np.uint64)
    seqs = np.tile(base, (n, 1))
    flip = rng.random((n, W)) < 0.3          # related taxa: distances spread, with ties
    seqs[flip] = rng.integers(0, 2 ** 63, size=int(flip.sum()), dtype=np.uint64)
    nw = (L + 31) // 32
    inc = np.zeros(W, np.uint32)
    inc[:nw] = 0xFFFFFFFF
    inc[3] = 0xF0F0F0F0
    if L % 32:
        inc[nw - 1] = (0xFFFFFFFF << (32 - L % 32)) & 0xFFFFFFFF
    return seqs, inc, W


@pytest.mark.parametrize("n,L,et,norm", [(300, 4000, 8, 0), (1000, 3000, 4, 0), (517, 2049, 2, 100), (129, 1000, 1, 0),
                                         (2300, 1500, 8, 1000), (70, 6_000_000, 8, 0)])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_dist_shard_layout(dev, n, L, et, norm, world):
    """ccg_snp_ltd_shard_dev writes each rank's rows exactly where
    ccg_tree_shard_dev reads them: equal to the band extract of the full LT
    (itself bit-exact vs the oracle elsewhere)."""
    import ccphylo_amd as cg
    from ccphylo_amd import native as nt
    seqs, inc, W = _rand_msa(n, L, n + world)
    dt = cg.ETYPES[et]
    full, _, _ = dev.snp_ltd(seqs, inc, n, L, norm=norm, etype=et, byte_scale=2.0)
    ps, pi = dev.malloc(seqs.nbytes), dev.malloc(inc.nbytes)
    dev.h2d(ps, seqs)
    dev.h2d(pi, inc)
    try:
        for rank in range(world):
            m = nt.shard_elems(n, rank, world)
            pd = dev.malloc(max(m, 1) * et)
            dev.snp_ltd_shard_dev(ps, pi, n, L, W, pd, rank, world, norm=norm, etype=et, byte_scale=2.0)
            got = np.empty(m, dtype=dt)
            if m:
                dev.d2h(got, pd)
            dev.free(pd)
            assert (got == nt.shard_extract(full, n, rank, world)).all()
    finally:
        dev.free(ps)
        dev.free(pi)


def test_dist_shard_to_tree_in_place(dev):
    """configs[4] in miniature on one GPU: dist writes the shard, the sharded
    DNJ consumes it in place; joins equal the single-GPU tree's."""
    import ccphylo_amd as cg
    from ccphylo_amd import native as nt
    n, L = 1500, 6000
    seqs, inc, W = _rand_msa(n, L, 3)
    full, _, _ = dev.snp_ltd(seqs, inc, n, L)
    ref = dev.tree(full, n, method=cg.CCG_TREE_DNJ, exact=True)[:3]
    ps, pi = dev.malloc(seqs.nbytes), dev.malloc(inc.nbytes)
    dev.h2d(ps, seqs)
    dev.h2d(pi, inc)
    pd = dev.malloc(nt.shard_elems(n, 0, 1) * 8)
    dev.snp_ltd_shard_dev(ps, pi, n, L, W, pd, 0, 1)
    got = dev.tree_shard_dev(pd, n, None, method=cg.CCG_TREE_DNJ, exact=True)[:3]
    for p in (ps, pi, pd):
        dev.free(p)
    _same(got, ref)


@pytest.mark.parametrize("n,L,et,proxi", [(300, 4000, 8, 0), (517, 2049, 4, 0), (129, 1000, 2, 0), (260, 3000, 8, 20),
                                          (75, 700, 4, 5)])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("mfma", ["2", "1", "0"])
def test_dist_shard_layout_pair(dev, monkeypatch, n, L, et, proxi, world, mfma):
    """Pair mode (cmpairFsaThrd, fsacmp.c:587; -P: maskProxi fsacmp.c:355)
    into the band shards: each rank's buffer equals the band extract of the
    full pair-mode LT (itself checked against the oracle and goldens), with
    the MFMA (k_snp_mfma2_pair, k_snp_mfma_pair) and VALU (k_snp_tile_pair) band forms."""
    import ccphylo_amd as cg
    monkeypatch.setenv("CCG_DIST_MFMA", mfma)
    from ccphylo_amd import native as nt
    seqs, inc1, W = _rand_msa(n, L, 7 * n + world + proxi)
    rng = np.random.default_rng(n + proxi)
    incs = np.tile(inc1, (n, 1))
    drop = rng.random((n, W, 32)) < 0.1        # per-taxon exclusions
    bits = (drop.astype(np.uint64) << np.arange(31, -1, -1, dtype=np.uint64)).sum(axis=2).astype(np.uint32)
    incs &= ~bits
    ml = int(0.8 * L)
    dt = cg.ETYPES[et]
    full, _, _ = dev.snp_ltd(seqs, incs, n, L, pair=True, min_length=ml, proxi=proxi, etype=et, byte_scale=2.0)
    ps, pi = dev.malloc(seqs.nbytes), dev.malloc(incs.nbytes)
    dev.h2d(ps, seqs)
    dev.h2d(pi, incs)
    try:
        for rank in range(world):
            m = nt.shard_elems(n, rank, world)
            pd = dev.malloc(max(m, 1) * et)
            dev.snp_ltd_shard_dev(ps, pi, n, L, W, pd, rank, world, etype=et, byte_scale=2.0, pair=True,
                                  min_length=ml, proxi=proxi)
            got = np.empty(m, dtype=dt)
            if m:
                dev.d2h(got, pd)
            dev.free(pd)
            assert (got == nt.shard_extract(full, n, rank, world)).all()
    finally:
        dev.free(ps)
        dev.free(pi)


class _DeviceSelfColl:
    """A world-1 ccg_coll with host_staged = 0 whose callbacks move DEVICE
    buffers with hipMemcpyAsync on the engine's stream, as RCCL's enqueue
    does: the non-staged CollRun paths (the allgather or its allreduce
    emulation, the broadcast of row n-1) without RCCL."""

    def __init__(self, native_allgather=True):
        import ctypes as C
        import importlib.util
        from ccphylo_amd import native
        spec = importlib.util.find_spec("torch")
        hip = C.CDLL(os.path.join(list(spec.submodule_search_locations)[0], "lib", "libamdhip64.so"))
        hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
        self.calls = {"allreduce": 0, "broadcast": 0, "allgather": 0}

        def copy(dst, src, nbytes, stream):
            if nbytes and dst != src:
                return int(hip.hipMemcpyAsync(dst, src, nbytes, 3, stream) != 0)   # device to device
            return 0

        def allreduce(user, buf, nbytes, stream):   # one rank: the sum is the buffer
            self.calls["allreduce"] += 1
            return 0

        def broadcast(user, send, recv, nbytes, root, stream):
            self.calls["broadcast"] += 1
            return copy(recv, send, nbytes, stream) if send else 0

        def allgather(user, send, recv, nbytes, stream):
            self.calls["allgather"] += 1
            return copy(recv, send, nbytes, stream)

        self._fns = (native.ALLREDUCE_FN(allreduce), native.BROADCAST_FN(broadcast),
                     native.ALLGATHER_FN(allgather) if native_allgather else native.ALLGATHER_FN())
        self.c = native.Coll(None, 0, 1, 0, *self._fns)


@pytest.mark.parametrize("method", [0, 1], ids=["nj", "dnj"])
@pytest.mark.parametrize("native_allgather", [True, False])
def test_shard_device_transport_world1(dev, method, native_allgather):
    """The sharded kernels over a device-side transport (host_staged = 0) give
    the single engine's joins (exact row sums)."""
    n = 1500
    D = _snp(n, 41) if method else _euclid(n, 41)
    want = dev.tree(D, n, method=method, exact=True)[:3]
    coll = _DeviceSelfColl(native_allgather)
    got = dev.tree_shard(D, n, coll, method=method, exact=True)[:3]
    assert (got[1], got[2]) == (want[1], want[2])
    assert len(got[0]) == len(want[0]) and (got[0] == want[0]).all()
    assert coll.calls["allgather" if native_allgather else "allreduce"] > 0


@pytest.mark.parametrize("world,n,kind,et", [(1, 3000, "euc", 8), (3, 2600, "clade", 4), (8, 2200, "snp", 8)])
def test_shard_multiblock_plan(dev, monkeypatch, tmp_path, world, n, kind, et):
    """The sharded DNJ's k_dnj_plan over a grid of listing blocks with the
    decoupled look-back (the single engine's form past 15361 taxa; round 6):
    CCG_PLAN_FR=1 gives one block per 960 rows at these sizes, with and
    without the band search; the joins equal the single engine's."""
    monkeypatch.setenv("CCG_PLAN_FR", "1")
    D, bs = _typed(_data(kind, n), et)
    ref = dev.tree(D, n, etype=et, byte_scale=bs, method=1, exact=True)[:3]
    monkeypatch.setenv("CCG_SHARD_FORCE", "1")   # world 1: the sharded kernels, not the single engine
    for split in ("16384", "100"):   # plain top-S listing, then band mode
        monkeypatch.setenv("CCG_S_SPLIT_N", split)
        if world == 1:
            _same(dev.tree_shard(D, n, None, etype=et, byte_scale=bs, method=1, exact=True)[:3], ref)
            continue
        mp.start_processes(_rank_main, args=(world, _free_port(), n, kind, et, True, "gloo", 1, str(tmp_path)),
                           nprocs=world, join=True, start_method="spawn")
        for r in range(world):
            fn, fd = np.load(tmp_path / f"f{r}.npy")
            _same((np.load(tmp_path / f"j{r}.npy"), int(fn), fd), ref)
