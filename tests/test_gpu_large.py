"""GPU parity at the BASELINE.json sizes (configs[1]-[3]), against the oracle's
serial restatement (oracle/ccoracle.c, pinned by the reference's golden
vectors; test infrastructure only).

- configs[1], N = 10,000 (the bench matrix: Euclidean U[0,1)^8, seed 1,
  %.9f-quantized): exact DNJ and HNJ, whole trees, joins and branch lengths
  bit-identical; NJ (O(n^3) in the oracle) as a join prefix.  Also an
  integer SNP matrix of 10k taxa (tie-heavy, from the GPU dist on a
  clade-structured alignment): exact DNJ prefix.
- configs[2], 50k taxa x 5 Mbp tree-like alignment: the GPU dist (sampled
  LT cells against orc_fsacmp, fsacmp.c:552) then exact DNJ on that matrix,
  a join prefix against the oracle's prefix on a host copy.
- configs[3], N = 200k float (80 GB) through the row-sharded engine
  (ccg_tree_shard_dev) at world 1: exact DNJ, the first 500 joins.

The sharded / multi-rank paths at smaller n are in test_gpu_shard.py.
Reference rules stressed here: minQpair dnj.c:43-128 (rescans and ties),
the serial row sums nj.c:911 / :1002 (exact mode), initSummaD nj.c:111.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 4)


@pytest.fixture(scope="module")
def dev():
    import ccphylo_amd as cg
    d = cg.Device(0)
    yield d
    d.close()


@pytest.fixture(scope="module")
def d10k():
    from tools.synth import euclid
    return euclid(10_000, seed=1)


def _same_joins(got, ref, what):
    (gj, gfn, gfd), (rj, rfn, rfd) = got, ref
    assert len(gj) == len(rj), (what, len(gj), len(rj))
    bad = np.nonzero((gj["i"] != rj["i"]) | (gj["j"] != rj["j"]))[0]
    assert bad.size == 0, (what, "first differing join", int(bad[0]) if bad.size else None)
    # branch lengths bit-identical (exact row sums are the reference's serial sums)
    assert (gj["Li"] == rj["Li"]).all() and (gj["Lj"] == rj["Lj"]).all(), what
    assert (gfn, gfd) == (rfn, rfd), (what, gfn, gfd, rfn, rfd)


def test_config1_dnj_exact_full(dev, d10k):
    import ccphylo_amd as cg
    from oracle import pyoracle
    n = 10_000
    ref = pyoracle.tree(d10k, n, method=cg.CCG_TREE_DNJ, threads=THREADS)
    got = dev.tree(d10k, n, method=cg.CCG_TREE_DNJ, exact=True)[:3]
    assert len(ref[0]) == n - 2
    _same_joins(got, ref, "dnj 10k exact")


def test_config1_hnj_exact_full(dev, d10k):
    import ccphylo_amd as cg
    from oracle import pyoracle
    n = 10_000
    ref = pyoracle.tree(d10k, n, method=cg.CCG_TREE_HNJ, threads=THREADS)
    got = dev.tree(d10k, n, method=cg.CCG_TREE_HNJ, exact=True)[:3]
    _same_joins(got, ref, "hnj 10k exact")


def test_config1_nj_exact_prefix(dev, d10k):
    """NJ: every join is a full initQ scan (nj.c:182), 5e7 cells at 10k, so
    the oracle runs a prefix; the GPU runs the same prefix (max_joins)."""
    import ccphylo_amd as cg
    from oracle import pyoracle
    n, k = 10_000, 120
    ref = pyoracle.tree(d10k, n, method=cg.CCG_TREE_NJ, max_joins=k, threads=THREADS)
    got = dev.tree(d10k, n, method=cg.CCG_TREE_NJ, exact=True, max_joins=k)
    assert len(ref[0]) == k and len(got[0]) == k
    _same_joins((got[0], 0, 0), (ref[0], 0, 0), "nj 10k exact prefix")


def test_config1_fast_sums_topology(dev, d10k):
    """Fast row sums (--fast_sums, not the default): a fixed-order tree sum of
    the new row instead of the serial one.  On this matrix the tree must be
    the same (same splits); the join order may differ at near-ties."""
    import ccphylo_amd as cg
    from oracle import pyoracle
    from tools.parity_large import splits
    n = 10_000
    ref, rfn, _ = pyoracle.tree(d10k, n, method=cg.CCG_TREE_DNJ, threads=THREADS)
    got, fn, _, _ = dev.tree(d10k, n, method=cg.CCG_TREE_DNJ, exact=False)
    assert splits(got, n, fn) == splits(ref, n, rfn)


def _clade_snp_ltd(dev, torch, n, L, clades, etype=8, seed=3):
    """LT (device tensor) of the SNP distances of a clade-structured packed
    alignment (tools/config3.make_packed), computed by the GPU dist."""
    from tools.config3 import make_packed
    W = L // 32 + 1
    seqs = make_packed(torch, n, W, clades=clades, seed=seed)
    incs = torch.full((W,), -1, dtype=torch.int32, device="cuda")
    incs[::10] = 0
    incs[(L + 31) // 32:] = 0
    if L % 32:
        incs[(L + 31) // 32 - 1] &= ((0xFFFFFFFF << (32 - L % 32)) & 0xFFFFFFFF) - (1 << 32)
    dt = {8: torch.float64, 4: torch.float32}[etype]
    D = torch.empty(n * (n - 1) // 2, dtype=dt, device="cuda")
    torch.cuda.synchronize()
    dev.snp_ltd_dev(seqs.data_ptr(), incs.data_ptr(), n, L, W, D.data_ptr(), etype=etype)
    torch.cuda.synchronize()
    return seqs, incs, D


def test_config1_snp_dnj_exact_prefix(dev):
    """Integer SNP counts at N = 10k (configs[1] (b)): many exactly tied Q
    values, the case minQpair's strict `<` rescans and the tie rules decide."""
    import torch
    import ccphylo_amd as cg
    from oracle import pyoracle
    n, k = 10_000, 1500
    seqs, incs, D = _clade_snp_ltd(dev, torch, n, 100_000, clades=256)
    del seqs, incs
    host = D.cpu().numpy()
    got = dev.tree_dev(D.data_ptr(), n, method=cg.CCG_TREE_DNJ, exact=True, max_joins=k)
    del D
    torch.cuda.empty_cache()
    ref = pyoracle.tree(host, n, method=cg.CCG_TREE_DNJ, max_joins=k, threads=THREADS, copy=False)
    assert len(ref[0]) == k
    _same_joins((got[0], 0, 0), (ref[0], 0, 0), "dnj 10k SNP exact prefix")


def test_config2_dist_and_dnj_prefix(dev):
    """configs[2]: 50k taxa x 5 Mbp (packed 2-bit, 62.5 GB in HBM), the
    non-pair dist into a double LT (10 GB), sampled cells against the
    oracle's fsacmp, then exact DNJ on that matrix (a join prefix)."""
    import torch
    import ccphylo_amd as cg
    from oracle import pyoracle
    n, L, k = 50_000, 5_000_000, 1000
    seqs, incs, D = _clade_snp_ltd(dev, torch, n, L, clades=512)
    lib = pyoracle.lib()
    hinc = incs.cpu().numpy().view(np.uint32).copy()
    rng = np.random.default_rng(2)
    pairs = [(1, 0), (n - 1, 0), (n - 1, n - 2), (n // 2, n // 3)] + \
            [tuple(sorted(rng.choice(n, 2, replace=False).tolist(), reverse=True)) for _ in range(12)]
    for i, j in pairs:
        a = seqs[i].cpu().numpy().view(np.uint64).copy()
        b = seqs[j].cpu().numpy().view(np.uint64).copy()
        want = lib.orc_fsacmp(a.ctypes.data, b.ctypes.data, hinc.ctypes.data, L)
        assert float(D[i * (i - 1) // 2 + j].item()) == float(want), (i, j)
    del seqs, incs
    torch.cuda.empty_cache()
    host = D.cpu().numpy()
    got = dev.tree_dev(D.data_ptr(), n, method=cg.CCG_TREE_DNJ, exact=True, max_joins=k)
    del D
    torch.cuda.empty_cache()
    ref = pyoracle.tree(host, n, method=cg.CCG_TREE_DNJ, max_joins=k, threads=THREADS, copy=False)
    assert len(ref[0]) == k
    _same_joins((got[0], 0, 0), (ref[0], 0, 0), "dnj configs[2] exact prefix")


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _config3_rank(rank, world, port, n, k, out_dir):
    """One rank of the world-8 rehearsal: its own band shard of configs[3]'s
    matrix built on the GPU, the sharded DNJ over gloo (HostColl)."""
    import json
    import sys
    import time
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist
    import ccphylo_amd as cg
    from ccphylo_amd import native as nt
    from tools.synth import euclid_shard_dev
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = cg.Device(0)
    # the ranks build their shards one after another: 8 ranks share the one
    # GPU, and each generator's temporaries (a few GB) should not peak together
    for r in range(world):
        if r == rank:
            loc = euclid_shard_dev(torch, n, rank, world, dtype=torch.float32)
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
        dist.barrier()
    assert loc.numel() == nt.shard_elems(n, rank, world)
    coll = nt.HostColl(dist)
    dist.barrier()
    t0 = time.perf_counter()
    joins, fn, fd, st = dev.tree_shard_dev(loc.data_ptr(), n, coll, etype=4, method=cg.CCG_TREE_DNJ, exact=True,
                                           max_joins=k, profile=True)
    dt = time.perf_counter() - t0
    np.save(os.path.join(out_dir, f"j{rank}.npy"), joins)
    K = nt.NKSTAT
    # device time per join by kernel class (HIP events on this rank's stream;
    # host-staged collectives: the class holds the staging copies, not the host wait)
    names = ["init", "dnj_select", "dnj_scan", "nj_argmin", "update", "dnj_requeue", "nj_pop", "dnj_find", "coll",
             "exact_sum"]
    dev_us = {nm: round(st[5 + 2 * c] / 1e3 / max(len(joins), 1), 2) for c, nm in enumerate(names)
              if st[4 + 2 * c] and nm != "init"}
    with open(os.path.join(out_dir, f"s{rank}.json"), "w") as f:
        json.dump({"rank": rank, "shard_GB": round(loc.numel() * 4 / 1e9, 3), "tree_s": round(dt, 2),
                   "device_us_per_join": dev_us, "device_s": round(st[3] / 1e6, 3),
                   "init_coll_bytes": int(st[8 + 2 * K]), "hard_columns": int(st[9 + 2 * K]),
                   "ref_rows": int(st[10 + 2 * K]), "ref_cells": int(st[11 + 2 * K]),
                   "coll_calls": coll.calls, "coll_bytes": coll.bytes}, f)
    del loc
    dev.close()
    dist.barrier()
    dist.destroy_process_group()


def test_config3_dnj_prefix(dev, monkeypatch, tmp_path):
    """configs[3]: N = 200k Euclidean (seed 4), float (`-p`, 80 GB), exact DNJ
    against the oracle's serial minQpair (threaded rescans, same decisions):
    the single engine's default float path (row-group rescans over the
    compacted enumeration, k_dnj_fold, k_dnj_join_pf, under the block lower
    bounds) over the first 1000 joins; the row-sharded kernels at
    world 1 (band layout = the packed LT) over the first 500; and configs[3]'s
    own world size rehearsed on the one GPU: 8 rank processes,
    each building its 10 GB band shard on the GPU (tools/synth.euclid_shard_dev)
    and running ccg_tree_shard_dev over gloo (HostColl: every exchange of the
    8-GPU run, host-staged), the first 1000 joins, every rank's joins equal to
    the oracle's and to the single engine's.  Reference: dnj.c:985-1052."""
    import json
    import torch
    import torch.multiprocessing as mp
    import ccphylo_amd as cg
    from oracle import pyoracle
    from tools.synth import euclid_shard_dev
    n, k, ks, kw, world = 200_000, 1000, 500, 1000, 8   # (one oracle prefix serves all three; the suite's time)
    got = {}
    for force, kk in (("0", k), ("1", ks)):
        monkeypatch.setenv("CCG_SHARD_FORCE", force)
        loc = euclid_shard_dev(torch, n, 0, 1, dtype=torch.float32)
        if force == "0":
            host = loc.cpu().numpy()
        got[force] = dev.tree_shard_dev(loc.data_ptr(), n, None, etype=4, method=cg.CCG_TREE_DNJ, exact=True,
                                        max_joins=kk)
        del loc
        torch.cuda.empty_cache()
    import gc
    gc.collect()
    torch.cuda.empty_cache()   # this process's cached blocks (earlier tests') back to the device for the 8 ranks
    free_b, total_b = torch.cuda.mem_get_info()
    print(f"device memory before the 8 ranks: {free_b / 2**30:.1f} GiB free of {total_b / 2**30:.1f}", flush=True)
    mp.start_processes(_config3_rank, args=(world, _free_port(), n, kw, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    ref = pyoracle.tree(host, n, etype=4, method=cg.CCG_TREE_DNJ, max_joins=k, threads=THREADS, copy=False)
    assert len(ref[0]) == k
    _same_joins((got["0"][0], 0, 0), (ref[0], 0, 0), "single engine dnj 200k float exact prefix")
    _same_joins((got["1"][0], 0, 0), (ref[0][:ks], 0, 0), "sharded dnj 200k float exact prefix")
    recs = []
    for r in range(world):
        jr = np.load(tmp_path / f"j{r}.npy")
        _same_joins((jr, 0, 0), (ref[0][:kw], 0, 0), f"world-8 rank {r} dnj 200k float exact prefix")
        assert (jr == got["0"][0][:kw]).all()
        recs.append(json.load(open(tmp_path / f"s{r}.json")))
    # every rank counted the same reference-rule rescans (replicated replay)
    assert len({(x["ref_rows"], x["ref_cells"]) for x in recs}) == 1
    rec = {"test": "config3_world8_rehearsal", "n": n, "world": world, "joins": kw, "etype": 4, "exact": True,
           "transport": "gloo (HostColl), 8 processes on one MI355X", "oracle_identical": True, "ranks": recs}
    print(json.dumps(rec))
    if os.environ.get("CCG_CONFIG4_OUT"):
        with open(os.environ["CCG_CONFIG4_OUT"], "a") as f:
            f.write(json.dumps(rec) + "\n")


def test_config3_single_vs_sharded_prefix(dev, monkeypatch):
    """configs[3]'s matrix past the point where a join lists ~10k rows (the
    first 12k joins): the single engine (k_dnj_fold chunk summaries and
    k_dnj_join_pf) against the row-sharded kernels at world 1 (k_shd_pick's
    replay_wave), two independent forms of minQpair's replay: identical joins
    and identical reference-rule rescan counts."""
    import torch
    import ccphylo_amd as cg
    from tools.synth import euclid_shard_dev
    K = cg.native.NKSTAT
    n, k = 200_000, 12_000
    out = []
    for force in ("0", "1"):
        monkeypatch.setenv("CCG_SHARD_FORCE", force)
        loc = euclid_shard_dev(torch, n, 0, 1, dtype=torch.float32)
        out.append(dev.tree_shard_dev(loc.data_ptr(), n, None, etype=4, method=cg.CCG_TREE_DNJ, exact=True,
                                      max_joins=k, profile=True))
        del loc
        torch.cuda.empty_cache()
    (a, _, _, sa), (b, _, _, sb) = out
    assert len(a) == k and len(b) == k
    _same_joins((a, 0, 0), (b, 0, 0), "configs[3] single engine vs sharded kernels")
    assert (sa[10 + 2 * K], sa[11 + 2 * K]) == (sb[10 + 2 * K], sb[11 + 2 * K])
    assert sa[10 + 2 * K] > 10 * k   # long listings: the large-T join path ran


def test_config4_pipeline_200k_world1_exact(dev, monkeypatch):
    """configs[4]'s pipeline at n = 200k x 100 kbp, world 1: the
    tree-like packed alignment in host memory -> ccg_snp_ltd_shard (planes
    streamed into HBM, float band shard = the packed LT at world 1): sampled
    cells against the oracle's fsacmp; then ccg_tree_shard_dev DNJ with EXACT
    row sums in place, a join prefix against the oracle on a host copy.
    Reference: cdist.c:196-390 (dist), dnj.c:985 (the DNJ loop)."""
    import torch
    import ccphylo_amd as cg
    from ccphylo_amd import native as nt
    from oracle import pyoracle
    from tools.config5_rank import make_packed_host
    monkeypatch.setenv("CCG_SHARD_FORCE", "1")   # the sharded kernels (world 1 would run the single engine)
    n, L, k = 200_000, 100_000, 400
    W = L // 32 + 1
    seqs = make_packed_host(torch, n, W)
    incs = np.full(W, 0xFFFFFFFF, dtype=np.uint32)
    incs[::10] = 0
    incs[(L + 31) // 32:] = 0
    if L % 32:
        incs[(L + 31) // 32 - 1] &= (0xFFFFFFFF << (32 - L % 32)) & 0xFFFFFFFF
    elems = nt.shard_elems(n, 0, 1)
    assert elems == n * (n - 1) // 2
    D = torch.empty(elems, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    inc = dev.snp_ltd_shard(seqs, incs, n, L, D.data_ptr(), 0, 1, etype=4)
    assert inc == int(np.unpackbits(incs.view(np.uint8)).sum())
    lib = pyoracle.lib()
    rng = np.random.default_rng(4)
    pairs = [(1, 0), (n - 1, 0), (n - 1, n - 2), (n // 2, n // 3)] + \
            [tuple(sorted(rng.choice(n, 2, replace=False).tolist(), reverse=True)) for _ in range(16)]
    for i, j in pairs:
        want = lib.orc_fsacmp(seqs[i].ctypes.data, seqs[j].ctypes.data, incs.ctypes.data, L)
        assert float(D[i * (i - 1) // 2 + j].item()) == float(want), (i, j)
    del seqs
    host = D.cpu().numpy()
    got = dev.tree_shard_dev(D.data_ptr(), n, None, etype=4, method=cg.CCG_TREE_DNJ, exact=True, max_joins=k)
    del D
    torch.cuda.empty_cache()
    ref = pyoracle.tree(host, n, etype=4, method=cg.CCG_TREE_DNJ, max_joins=k, threads=THREADS, copy=False)
    assert len(ref[0]) == k
    _same_joins((got[0], 0, 0), (ref[0], 0, 0), "configs[4] pipeline 200k exact prefix")


@pytest.mark.parametrize("env", ["", "CCG_SCAN_WAVE=1", "CCG_SCAN_WAVE=0 CCG_PLAN_MULTI=0"])
def test_dnj_large_n_kernels_prefix(dev, monkeypatch, env):
    """The large-n forms of the DNJ search (n > 16384): k_dnj_plan over
    several blocks with the look-back for entry positions, the wave-per-unit
    rescans with 16-byte row loads (default), the scalar wave form, and the
    round-2 forms (one plan block, one unit per block): a 1500-join prefix of
    a 33k Euclidean tree against the oracle (minQpair dnj.c:43-128)."""
    import torch
    import ccphylo_amd as cg
    from oracle import pyoracle
    from tools.synth import euclid_shard_dev
    for kv in env.split():
        k, v = kv.split("=")
        monkeypatch.setenv(k, v)
    n, k = 33_000, 1500
    D = euclid_shard_dev(torch, n, 0, 1, seed=9)   # world 1: the packed LT
    host = D.cpu().numpy()
    got = dev.tree_dev(D.data_ptr(), n, method=cg.CCG_TREE_DNJ, exact=True, max_joins=k)
    del D
    torch.cuda.empty_cache()
    ref = pyoracle.tree(host, n, method=cg.CCG_TREE_DNJ, max_joins=k, threads=THREADS, copy=False)
    assert len(ref[0]) == k
    _same_joins((got[0], 0, 0), (ref[0], 0, 0), f"dnj 33k prefix [{env}]")


@pytest.fixture(scope="module")
def msa_1e6():
    """configs[4]'s alignment: n = 1e6 taxa x L = 100 kbp, tree-like (512
    clades), packed in HOST memory (25 GB; every rank holds it and streams it
    into its bit planes), every 10th word excluded."""
    import torch
    from tools.config5_rank import make_packed_host
    n, L = 1_000_000, 100_000
    W = L // 32 + 1
    seqs = make_packed_host(torch, n, W)
    incs = np.full(W, 0xFFFFFFFF, dtype=np.uint32)
    incs[::10] = 0
    incs[(L + 31) // 32:] = 0
    if L % 32:
        incs[(L + 31) // 32 - 1] &= (0xFFFFFFFF << (32 - L % 32)) & 0xFFFFFFFF
    yield n, L, seqs, incs
    del seqs


@pytest.mark.parametrize("rank", [0, 7])
def test_config4_rank_1e6(dev, msa_1e6, rank):
    """configs[4] (n = 1e6, world 8) for one rank on one MI355X: the rank's
    dist straight into its 250 GB float band shard (ccg_snp_ltd_shard, the
    alignment streamed from host memory into compacted bit planes), sampled
    cells against the oracle's fsacmp (fsacmp.c:552), the dist's HBM peak
    within 280 GB; then, with the planes freed, the rank's whole tree-phase
    state (ccg_tree_shard_bytes: every buffer ccg_tree_shard_dev allocates
    beside the shard for DNJ at this n) allocated next to the shard.  The
    cross-rank exchange of the tree needs the 8-GPU node."""
    import json
    import torch
    from ccphylo_amd import native as nt
    from oracle import pyoracle
    n, L, seqs, incs = msa_1e6
    world = 8
    torch.cuda.empty_cache()
    free0, total = torch.cuda.mem_get_info()
    elems = nt.shard_elems(n, rank, world)
    Dloc = dev.malloc(elems * 4)
    tree_b = None
    try:
        import threading
        import time
        # the dist's HBM high-water mark, sampled: a side thread
        # polls hipMemGetInfo while ccg_snp_ltd_shard runs (ctypes drops the GIL)
        low = [free0]
        stop = threading.Event()

        def poll():
            while not stop.is_set():
                f, _ = torch.cuda.mem_get_info()
                low[0] = min(low[0], f)
                time.sleep(0.002)
        th = threading.Thread(target=poll, daemon=True)
        th.start()
        t0 = time.perf_counter()
        try:
            inc = dev.snp_ltd_shard(seqs, incs, n, L, Dloc, rank, world, etype=4)
        finally:
            dist_s = time.perf_counter() - t0
            stop.set()
            th.join()
        assert inc == int(np.unpackbits(incs.view(np.uint8)).sum())
        # the planes the dist held beside the shard: kept words (compacted) x 2 bits, rows padded to 256
        Wc = int((incs[:(L + 31) // 32] != 0).sum())
        planes = -(-n // 256) * 256 * (-(-Wc // 16) * 16) * 8
        planned = elems * 4 + planes + (256 << 20)
        peak = free0 - low[0]   # measured: HBM this test held at the lowest free sample (shard included)
        assert peak >= elems * 4, (peak, elems * 4)
        assert peak <= 280e9, peak
        lib = pyoracle.lib()
        rng = np.random.default_rng(rank + 1)
        host = np.empty(1, dtype=np.float32)
        rows = [r for r in (n - 1, n // 2 + 3, 8 * world * 3 + rank * 8 + 5, 8 * rank + 1)
                if r >= 1 and nt.shard_owner(r, world) == rank]
        rows += [int(b) * 8 + int(rng.integers(0, 8)) for b in rng.integers(0, n // 8, 64) if b % world == rank][:8]
        checked = 0
        for i in rows:
            if i >= n or i < 1:
                continue
            for j in sorted({0, i // 2, i - 1, int(rng.integers(0, i))}):
                want = lib.orc_fsacmp(seqs[i].ctypes.data, seqs[j].ctypes.data, incs.ctypes.data, L)
                dev.d2h(host, Dloc + 4 * (nt.shard_row_offset(i, rank, world) + j))
                assert float(host[0]) == float(want), (rank, i, j)
                checked += 1
        assert checked >= 20
        # the tree phase: its whole device state beside the shard
        tree_b, gather_b = nt.tree_shard_bytes(n, 4, 1, world)
        free1, _ = torch.cuda.mem_get_info()
        Tb = dev.malloc(tree_b)
        free2, _ = torch.cuda.mem_get_info()
        dev.free(Tb)
        rec = {"n": n, "L": L, "world": world, "rank": rank, "dist_s": round(dist_s, 3), "rank_cells": elems,
               "rank_taxa_pairs_per_s": round(elems / dist_s, 1), "shard_GB": round(elems * 4 / 1e9, 2),
               "kept_words": Wc, "planes_GB": round(planes / 1e9, 2), "dist_peak_GB_measured": round(peak / 1e9, 2),
               "dist_peak_GB_planned": round(planned / 1e9, 2),
               "peak_source": "hipMemGetInfo polled every 2 ms on a side thread during ccg_snp_ltd_shard",
               "tree_phase_state_GB": round(tree_b / 1e9, 3),
               "tree_phase_total_GB": round((elems * 4 + tree_b) / 1e9, 2),
               "init_gather_bound_GB": round(gather_b / 1e9, 2),
               "hbm_total_GB": round(total / 1e9, 2), "hbm_free_before_GB": round(free0 / 1e9, 2),
               "hbm_free_after_shard_GB": round(free1 / 1e9, 2),
               "hbm_free_with_tree_state_GB": round(free2 / 1e9, 2), "checked_cells": checked}
        print(json.dumps(rec))
        if os.environ.get("CCG_CONFIG4_OUT"):
            with open(os.environ["CCG_CONFIG4_OUT"], "a") as f:
                f.write(json.dumps(rec) + "\n")
        # the tree phase leaves the init's gather room too (used only by hard columns)
        assert free2 > 1e9
    finally:
        dev.free(Dloc)


@pytest.mark.skipif(not os.environ.get("CCG_HEADLINE_PIN"),
                    reason="opt-in: CCG_HEADLINE_PIN=1 (about 6 minutes with 16 host cores; run with -s)")
def test_config2_headline_whole_tree_vs_oracle(tmp_path):
    """The bench's own configs[2] matrix (50k x 5 Mbp, seed 3, GPU dist), 64
    LT cells against orc_fsacmp, then the engine's whole exact DNJ tree
    against the oracle's serial-decision DNJ on the same LT (host threads):
    every join, both branch lengths, the final pair (tools/parity_headline.py;
    profiles/r06_parity_headline.jsonl).  Reference: dnj.c:43-128, :985-1052."""
    import json
    import subprocess
    import sys
    out = tmp_path / "pin.jsonl"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-u", os.path.join(root, "tools", "parity_headline.py"), "--start", "0",
                        "--budget", "1e9", "--threads", str(THREADS), "--out", str(out)], cwd=root, timeout=1500)
    assert p.returncode == 0
    rec = json.loads(out.read_text().splitlines()[-1])
    assert rec["cells_identical"] and rec["joins_identical"] and rec["final_identical"], rec
    assert rec["joins_compared"] == 49_998
