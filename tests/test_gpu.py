"""GPU parity: the gfx950 engine through the C-ABI (ctypes) and through the
`ccphylo` CLI, against the golden vectors and the oracle.  Bit-exact for the
integer SNP counts / LT matrices and for exact-mode trees; fast-mode trees
must have the same topology with branch lengths within 1e-9 relative."""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, golden_bytes, golden_cases, parse_dist_args, parse_tree_args, print_phylip

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import ccphylo_amd as cg
    d = cg.Device(0)
    yield d
    d.close()


def test_device_is_gfx950(dev):
    assert "gfx950" in dev.info()


@pytest.mark.parametrize("case", golden_cases("tree"), ids=lambda c: c["name"])
def test_tree_golden_engine(dev, case):
    import ccphylo_amd as cg
    path, method, et, bs, flags, prec = parse_tree_args(case["args"])

    def run(D, n):
        joins, fn, fd, _ = dev.tree(D, n, etype=et, byte_scale=bs, method=method, flags=flags, exact=True)
        return joins, fn, fd
    trees = cg.newick_from_phylip(path, run, etype=et, byte_scale=bs, flags=flags, precision=prec)
    assert ("\n".join(trees) + "\n").encode() == golden_bytes(case)


@pytest.mark.parametrize("case", golden_cases("tree") + golden_cases("dist") + golden_cases("fsafiles"),
                         ids=lambda c: c["name"])
def test_cli_golden(case):
    import ccphylo_amd as cg
    args = list(case["args"])
    p = subprocess.run([cg.CLI_PATH] + args, cwd=GOLDEN, capture_output=True, timeout=300)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    assert p.stdout == golden_bytes(case)


@pytest.mark.parametrize("case", [c for c in golden_cases("dist")], ids=lambda c: c["name"])
def test_dist_golden_engine(dev, case):
    import ccphylo_amd as cg
    o = parse_dist_args(case["args"])
    heads, seqs, incs, L, minLength = cg.load_msa(o["inp"], o["flag"], o["minLength"], o["minCov"], o["proxi"])
    n = len(heads)
    pair = bool(o["flag"] & 2)
    out = b""
    if n > 1:
        D, N, inc = dev.snp_ltd(seqs, incs, n, L, pair=pair, norm=o["norm"], min_length=minLength, etype=o["et"],
                                byte_scale=o["bs"], proxi=o["proxi"] if pair else 0, want_n=o["nout"])
        out = print_phylip(D, n, heads, o["flag"], o["prec"], o["et"], o["bs"])
        if N is not None:
            out += print_phylip(N, n, heads, o["flag"], o["prec"], o["et"], o["bs"])
    assert out == golden_bytes(case)


def _euclid(n, seed, dim=8):
    rng = np.random.default_rng(seed)
    pts = rng.random((n, dim))
    i, j = np.tril_indices(n, -1)
    return np.sqrt(((pts[i] - pts[j]) ** 2).sum(1))


def _snp(n, seed, L=4000):
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 4, L)
    anc = [base]
    rows = []
    for t in range(n):
        p = anc[rng.integers(len(anc))].copy()
        m = rng.random(L) < 0.01
        p[m] = rng.integers(0, 4, m.sum())
        if rng.random() < 0.3:
            anc.append(p)
        rows.append(p)
    X = np.array(rows)
    i, j = np.tril_indices(n, -1)
    # differing sites = L - sites equal, the equal ones counted per code by a
    # matrix product (exact integers in f64; the pairwise compare took seconds)
    same = sum((X == c).astype(np.float64) @ (X == c).astype(np.float64).T for c in range(4))
    return L - same[i, j]


@pytest.mark.parametrize("n,kind,method", [(600, "euc", 1), (600, "euc", 0), (1500, "snp", 1), (1500, "snp", 0),
                                          (2500, "euc", 1)])
def test_tree_exact_vs_oracle(dev, n, kind, method):
    from oracle import pyoracle
    D = _euclid(n, n) if kind == "euc" else _snp(n, n)
    joins, fn, fd, st = dev.tree(D, n, method=method, exact=True)
    rj, rfn, rfd = pyoracle.tree(D, n, method=method)
    assert (fn, fd) == (rfn, rfd)
    assert len(joins) == len(rj)
    assert (joins["i"] == rj["i"]).all() and (joins["j"] == rj["j"]).all()
    assert (joins["Li"] == rj["Li"]).all() and (joins["Lj"] == rj["Lj"]).all()


@pytest.mark.parametrize("et", [4, 2, 1])
def test_tree_types_vs_oracle(dev, et):
    from oracle import pyoracle
    n = 700
    D = _snp(n, 11)
    bs = {4: 1.0, 2: 4.0, 1: 1.0}[et]
    if et == 4:
        Dt = D.astype(np.float32)
    else:
        Dt = np.clip(D * bs + 0.5, 0, 255 if et == 1 else 65535).astype(np.uint8 if et == 1 else np.uint16)
    for method in (0, 1):
        joins, fn, fd, _ = dev.tree(Dt, n, etype=et, byte_scale=bs, method=method, exact=True)
        rj, rfn, rfd = pyoracle.tree(Dt, n, etype=et, byte_scale=bs, method=method)
        assert (fn, fd) == (rfn, rfd)
        assert (joins == rj).all()


def test_tree_fast_sums_topology(dev):
    """--fast_sums: same join sequence, limb lengths within 1e-9 relative (stated tolerance)."""
    from oracle import pyoracle
    n = 2000
    D = _euclid(n, 3)
    joins, fn, fd, _ = dev.tree(D, n, method=1, exact=False)
    rj, rfn, rfd = pyoracle.tree(D, n, method=1)
    assert fn == rfn and (joins["i"] == rj["i"]).all() and (joins["j"] == rj["j"]).all()
    for f in ("Li", "Lj"):
        np.testing.assert_allclose(joins[f], rj[f], rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("n,L,pair,et,norm", [(257, 5000, False, 8, 0), (300, 4097, True, 8, 0),
                                              (130, 70000, False, 4, 1000), (129, 3000, True, 2, 100),
                                              (200, 1024, False, 1, 0)])
def test_dist_random_vs_oracle(dev, n, L, pair, et, norm):
    from oracle import pyoracle
    rng = np.random.default_rng(n + L)
    W = L // 32 + 1
    seqs = rng.integers(0, 2 ** 63, size=(n, W), dtype=np.uint64) | (rng.integers(0, 2, size=(n, W), dtype=np.uint64) << np.uint64(63))
    nw = (L + 31) // 32
    def mask():
        m = rng.integers(0, 2 ** 32, size=W, dtype=np.uint64).astype(np.uint32) | np.uint32(0xF7FFFFFF)
        m[nw:] = 0
        if L % 32:
            m[nw - 1] &= np.uint32((0xFFFFFFFF << (32 - L % 32)) & 0xFFFFFFFF)
        return m
    incs = np.stack([mask() for _ in range(n)]) if pair else mask()
    ml = int(0.9 * L) if pair else 1
    Dg, Ng, _ = dev.snp_ltd(seqs, incs, n, L, pair=pair, norm=norm, min_length=ml, etype=et, byte_scale=2.0,
                            want_n=pair)
    Do, No, _ = pyoracle.snp_ltd(seqs, incs, n, L, pair=pair, norm=norm, min_length=ml, etype=et, byte_scale=2.0,
                                 want_n=pair)
    assert (Dg == Do).all()
    if pair:
        assert (Ng == No).all()


def _related_msa(rng, n, L, rate, nrate=0.02):
    """Packed taxa that differ from one random reference at `rate` (2-bit codes
    MSB-first, qseqs.c:60) and per-taxon include masks with ~nrate holes."""
    W = L // 32 + 1
    base = rng.integers(0, 4, L)
    codes = np.tile(base, (n, 1))
    mut = rng.random((n, L)) < rate
    codes[mut] = rng.integers(0, 4, int(mut.sum()))
    codes[:, L - 1] = np.arange(n) % 4          # a SNP at the last position (the sentinel case, fsacmp.c:367)
    pad = np.zeros((n, W * 32), np.uint64)
    pad[:, :L] = codes
    sh = np.uint64(62) - np.uint64(2) * (np.arange(32, dtype=np.uint64))
    seqs = (pad.reshape(n, W, 32) << sh).sum(2, dtype=np.uint64)
    inc = np.zeros((n, W * 32), np.uint64)
    inc[:, :L] = rng.random((n, L)) >= nrate
    incs = (inc.reshape(n, W, 32) << (np.uint64(31) - np.arange(32, dtype=np.uint64))).sum(2, dtype=np.uint64)
    return seqs, incs.astype(np.uint32)


@pytest.mark.parametrize("n,L,et,rows,pair", [(300, 1000, 8, None, False), (1000, 20000, 4, None, False),
                                              (777, 4097, 2, (100, 650), False), (2100, 33, 1, None, False),
                                              (129, 700000, 8, (5, 129), False), (300, 1000, 8, None, True),
                                              (900, 30000, 4, None, True), (555, 4100, 2, (50, 400), True),
                                              (1100, 65, 8, None, True), (70, 6_000_000, 8, None, False),
                                              (40, 5_800_000, 4, None, True),
                                              # enough 256 x 256 tiles that k_snp_mfma2 runs without split-K
                                              (24000, 640, 4, None, False), (20000, 1000, 8, (3000, 17001), False),
                                              # and k_snp_mfma2_pair (column halves of 256 x 256 tiles) likewise
                                              (17000, 640, 8, None, True), (16500, 300, 4, (2000, 16001), True)])
def test_dist_mfma_equals_valu(dev, monkeypatch, n, L, et, rows, pair):
    """The MFMA forms of fsacmp / fsacmpair (k_snp_mfma / k_snp_mfma2 / k_snp_mfma3, k_snp_mfma_pair /
    k_snp_mfma2_pair:
    tetrahedron +-1 vectors in MX-fp4, dist = (3 L - dot) / 4, in pair mode
    masked with n from a fourth component) give the VALU tile kernels'
    matrices (and N) bit for bit: odd sizes, row ranges, split-K slices, every element type (the
    default path, MFMA, is checked against the oracle by the tests above)."""
    import torch
    rng = np.random.default_rng(n + L)
    W = L // 32 + 1
    seqs = rng.integers(-2**62, 2**62, (n, W), dtype=np.int64)
    seqs[:, : W // 3] = seqs[0, : W // 3]
    inc = np.full((n, W) if pair else W, -1, dtype=np.int32)
    inc[..., (L + 31) // 32:] = 0
    if L % 32:
        inc[..., (L + 31) // 32 - 1] = ((0xFFFFFFFF << (32 - L % 32)) & 0xFFFFFFFF) - (1 << 32)
    inc[..., W // 2] &= 0x0F0F0F0F
    if pair:   # per-taxon masks: ~1/8 of the positions excluded, differently per taxon
        inc &= (rng.integers(-2**31, 2**31, inc.shape, dtype=np.int64) | 0x77777777).astype(np.int32)
    out = {}
    # VALU tiles, k_snp_mfma (128 x 128), k_snp_mfma2 (256 x 256, register-staged), k_snp_mfma3 (256 x 256,
    # LDS-DMA staged through 4 stages: the non-pair default)
    for mode in ("0", "1", "2", "3"):
        monkeypatch.setenv("CCG_DIST_MFMA", "2" if mode == "3" else mode)
        monkeypatch.setenv("CCG_DIST_GLDS", "1" if mode == "3" else "0")
        s_d = torch.from_numpy(seqs).cuda()
        i_d = torch.from_numpy(inc).cuda()
        m = n * (n - 1) // 2
        D = torch.zeros(m, dtype={8: torch.float64, 4: torch.float32, 2: torch.int16, 1: torch.uint8}[et],
                        device="cuda")
        Nd = torch.zeros_like(D) if pair else None
        kw = dict(etype=et, pair=pair, N_ptr=Nd.data_ptr() if pair else None)
        if rows:
            kw["row_range"] = rows
        dev.snp_ltd_dev(s_d.data_ptr(), i_d.data_ptr(), n, L, W, D.data_ptr(), **kw)
        torch.cuda.synchronize()
        out[mode] = (D.cpu().numpy(), Nd.cpu().numpy() if pair else None)
    for mode in ("1", "2", "3"):
        assert (out["0"][0].view(np.uint8) == out[mode][0].view(np.uint8)).all(), mode
        if pair:
            assert (out["0"][1].view(np.uint8) == out[mode][1].view(np.uint8)).all(), mode
    assert out["2"][0].any()


@pytest.mark.parametrize("n,L,proxi,rate,et,norm", [(70, 3000, 10, 0.05, 8, 0), (65, 4097, 2, 0.3, 8, 1000),
                                                    (40, 20000, 40, 0.01, 4, 0), (33, 2048, 100, 0.02, 2, 100),
                                                    (50, 9000, 1, 0.7, 1, 100), (20, 70000, 33, 0.002, 8, 0),
                                                    (30, 1000, 5000, 0.01, 8, 0)])
def test_dist_pair_proxi_vs_oracle(dev, n, L, proxi, rate, et, norm):
    """Pair mode with -P (maskProxi, fsacmp.c:355): bit-exact (dist, n) and the
    A7 epilogue vs the oracle, from dense to sparse SNPs, proxi spanning words."""
    from oracle import pyoracle
    rng = np.random.default_rng(n * L + proxi)
    seqs, incs = _related_msa(rng, n, L, rate)
    ml = int(0.5 * L)
    Dg, Ng, _ = dev.snp_ltd(seqs, incs, n, L, pair=True, norm=norm, min_length=ml, etype=et, byte_scale=2.0,
                            proxi=proxi, want_n=True)
    Do, No, _ = pyoracle.snp_ltd(seqs, incs, n, L, pair=True, norm=norm, min_length=ml, proxi=proxi, etype=et,
                                 byte_scale=2.0, want_n=True)
    assert (Dg == Do).all() and (Ng == No).all()
    D0, _, _ = pyoracle.snp_ltd(seqs, incs, n, L, pair=True, norm=norm, min_length=ml, etype=et, byte_scale=2.0)
    assert not (D0 == Do).all()     # the masking did something


def test_dist_pair_proxi_row_range(dev):
    from oracle import pyoracle
    rng = np.random.default_rng(11)
    n, L = 90, 5000
    seqs, incs = _related_msa(rng, n, L, 0.03)
    Do, _, _ = pyoracle.snp_ltd(seqs, incs, n, L, pair=True, proxi=8)
    for rb, re_ in [(0, 31), (31, 64), (64, 90)]:
        Dg, _, _ = dev.snp_ltd(seqs, incs, n, L, pair=True, proxi=8, row_range=(rb, re_))
        lo, hi = rb * (rb - 1) // 2, re_ * (re_ - 1) // 2
        assert (Dg[lo:hi] == Do[lo:hi]).all()


def test_dist_row_range(dev):
    from oracle import pyoracle
    rng = np.random.default_rng(5)
    n, L = 300, 3000
    W = L // 32 + 1
    seqs = rng.integers(0, 2 ** 63, size=(n, W), dtype=np.uint64)
    incs = np.zeros(W, np.uint32)
    incs[: (L + 31) // 32] = 0xFFFFFFFF
    incs[(L + 31) // 32 - 1] = (0xFFFFFFFF << (32 - L % 32)) & 0xFFFFFFFF
    Do, _, _ = pyoracle.snp_ltd(seqs, incs, n, L)
    parts = [(0, 77), (77, 200), (200, 300)]
    acc = np.zeros_like(Do)
    for rb, re_ in parts:
        Dg, _, _ = dev.snp_ltd(seqs, incs, n, L, row_range=(rb, re_))
        lo, hi = rb * (rb - 1) // 2, re_ * (re_ - 1) // 2
        assert (Dg[lo:hi] == Do[lo:hi]).all()
        acc[lo:hi] = Dg[lo:hi]
    assert (acc == Do).all()


@pytest.mark.parametrize("et", [8, 4, 2, 1])
@pytest.mark.parametrize("n", [70, 300])
@pytest.mark.parametrize("method", [0, 1], ids=["nj", "dnj"])
def test_tree_all_ties(dev, monkeypatch, et, n, method):
    """A matrix of one repeated value: every Q and every D ties, so only the
    reference's tie rules (initHNJ hclust.c:110-115, initQ `<=`, minQpair) pick
    the joins.  Guards the tie branch ROCm 7.2 miscompiled in k_init_hnj for
    u8 elements (P stayed at column 63)."""
    from oracle import pyoracle
    dt = {8: np.float64, 4: np.float32, 2: np.uint16, 1: np.uint8}[et]
    D = np.full(n * (n - 1) // 2, 200, dtype=dt)
    got, fn, fd, _ = dev.tree(D, n, etype=et, byte_scale=1.0, method=method, exact=True)
    ref, rfn, rfd = pyoracle.tree(D, n, method=method, etype=et, byte_scale=1.0)
    assert (fn, fd) == (rfn, rfd)
    assert len(got) == len(ref) and (got["i"] == ref["i"]).all() and (got["j"] == ref["j"]).all()
    assert (got["Li"] == ref["Li"]).all() and (got["Lj"] == ref["Lj"]).all()
    monkeypatch.setenv("CCG_SHARD_FORCE", "1")   # the sharded kernels, not the world-1 single engine
    sh, sfn, sfd, _ = dev.tree_shard(D, n, None, etype=et, byte_scale=1.0, method=method, exact=True)
    assert (sfn, sfd) == (rfn, rfd) and (sh == got).all()


def _clade_ltd(n, seed, L=3000, clades=16):
    rng = np.random.default_rng(seed)
    X = rng.integers(0, 4, (clades, L))[rng.integers(0, clades, n)]
    X = np.where(rng.random((n, L)) < 0.01, rng.integers(0, 4, (n, L)), X)
    same = sum((X == c).astype(np.float64) @ (X == c).astype(np.float64).T for c in range(4))
    i, j = np.tril_indices(n, -1)
    return L - same[i, j]


@pytest.mark.parametrize("kind,n,env", [("euc", 1500, "1,8,3,0"), ("euc", 2500, "2,16,2,0"),
                                        ("clade", 1500, "2,8,4,0"), ("clade", 2500, "1,4,1,0"),
                                        ("clade", 3000, "0,2048,8,0"), ("euc", 3000, "1,2048,1,0")])
def test_dnj_large_n_modes(dev, monkeypatch, kind, n, env):
    """The large-n settings of the DNJ search at small n: rescan units of
    several SEG (CCG_SEG_MUL), each rest row's units folded once by k_dnj_fold
    (CCG_PREFOLD_N=0) and scan grids far smaller than the units
    (CCG_SCAN_MAX: many grid waves), with the chunk-summary join kernel
    k_dnj_join_pf (CCG_JOIN_PF=1), its block-0 replay path forced (2) or the
    per-block replay (0).  Joins bit-identical to the serial reference (exact
    row sums), single GPU and sharded."""
    from oracle import pyoracle
    if kind == "euc":
        rng = np.random.default_rng(n)
        pts = rng.random((n, 8))
        i, j = np.tril_indices(n, -1)
        D = np.sqrt(((pts[i] - pts[j]) ** 2).sum(1))
    else:
        D = _clade_ltd(n, n)
    jpf, scan, segm, pf = env.split(",")
    monkeypatch.setenv("CCG_JOIN_PF", jpf)
    monkeypatch.setenv("CCG_SCAN_MAX", scan)
    monkeypatch.setenv("CCG_SEG_MUL", segm)
    monkeypatch.setenv("CCG_PREFOLD_N", pf)
    got, fn, fd, st = dev.tree(D, n, method=1, exact=True)
    ref, rfn, rfd = pyoracle.tree(D, n, method=1)
    assert (fn, fd) == (rfn, rfd)
    assert len(got) == len(ref) and (got == ref).all()
    monkeypatch.setenv("CCG_SHARD_FORCE", "1")   # the sharded kernels, not the world-1 single engine
    sh = dev.tree_shard(D, n, None, method=1, exact=True)[0]
    assert (sh == got).all()


@pytest.mark.parametrize("kind,n,top,bands", [("euc", 2000, 16, 64), ("clade", 2500, 8, 32), ("euc", 3000, 1, 127),
                                               ("clade", 1800, 16, 64)])
def test_dnj_band_mode_small_n(dev, monkeypatch, kind, n, top, bands):
    """The large-n choice of S (top rows + one min-Q row per band, per-slot
    bounds in k_dnj_plan's listing, CCG_S_SPLIT_N) at small n: joins
    bit-identical to the serial reference (exact row sums), single GPU and
    sharded at world 1."""
    from oracle import pyoracle
    if kind == "euc":
        rng = np.random.default_rng(n + top)
        pts = rng.random((n, 8))
        i, j = np.tril_indices(n, -1)
        D = np.sqrt(((pts[i] - pts[j]) ** 2).sum(1))
    else:
        D = _clade_ltd(n, n + 7)
    monkeypatch.setenv("CCG_S_SPLIT_N", "100")
    monkeypatch.setenv("CCG_S_TOP", str(top))
    monkeypatch.setenv("CCG_S_BANDS", str(bands))
    got, fn, fd, st = dev.tree(D, n, method=1, exact=True)
    ref, rfn, rfd = pyoracle.tree(D, n, method=1)
    assert (fn, fd) == (rfn, rfd)
    assert len(got) == len(ref) and (got == ref).all()
    monkeypatch.setenv("CCG_SHARD_FORCE", "1")   # the sharded kernels, not the world-1 single engine
    sh = dev.tree_shard(D, n, None, method=1, exact=True)[0]
    assert (sh == got).all()


def _missing_ltd(n, seed, frac=0.05):
    """Euclidean distances with a fraction of cells set to -1 (missing,
    nj.c:111 initSummaD skips them; updateD's quirky branches run)."""
    D = _euclid(n, seed)
    rng = np.random.default_rng(seed + 1)
    D[rng.random(D.size) < frac] = -1.0
    return D


@pytest.mark.parametrize("n,kind", [(600, "euc"), (1500, "snp"), (2500, "euc"), (3000, "clade"), (400, "miss"),
                                    (1100, "miss")])
def test_hnj_vs_oracle(dev, n, kind):
    """-m hnj (hclust.c:1671): joins bit-identical to the serial reference
    restatement in exact mode, including updatePrevQ's row-0 / last-row
    quirks, the column-j `P == i || P == j` rule and HNJ_popArrange's
    `P < pos || q < Q` rule; matrices with missing entries take the general
    updateD."""
    from oracle import pyoracle
    D = {"euc": lambda: _euclid(n, n), "snp": lambda: _snp(n, n), "clade": lambda: _clade_ltd(n, n),
         "miss": lambda: _missing_ltd(n, n)}[kind]()
    got, fn, fd, _ = dev.tree(D, n, method=2, exact=True)
    ref, rfn, rfd = pyoracle.tree(D, n, method=2)
    assert (fn, fd) == (rfn, rfd)
    assert len(got) == len(ref) and (got == ref).all()


@pytest.mark.parametrize("et", [4, 2, 1])
def test_hnj_types_vs_oracle(dev, et):
    from oracle import pyoracle
    n = 700
    D = _snp(n, 17)
    bs = {4: 1.0, 2: 4.0, 1: 1.0}[et]
    Dt = D.astype(np.float32) if et == 4 else np.clip(D * bs + 0.5, 0, 255 if et == 1 else 65535).astype(
        np.uint8 if et == 1 else np.uint16)
    got, fn, fd, _ = dev.tree(Dt, n, etype=et, byte_scale=bs, method=2, exact=True)
    ref, rfn, rfd = pyoracle.tree(Dt, n, etype=et, byte_scale=bs, method=2)
    assert (fn, fd) == (rfn, rfd) and (got == ref).all()


@pytest.mark.parametrize("et", [8, 1])
def test_hnj_all_ties(dev, et):
    from oracle import pyoracle
    n = 300
    D = np.full(n * (n - 1) // 2, 200, dtype=np.float64 if et == 8 else np.uint8)
    got, fn, fd, _ = dev.tree(D, n, etype=et, byte_scale=1.0, method=2, exact=True)
    ref, rfn, rfd = pyoracle.tree(D, n, method=2, etype=et, byte_scale=1.0)
    assert (fn, fd) == (rfn, rfd) and (got == ref).all()


def test_hnj_fast_sums(dev):
    """--fast_sums: same joins, lengths within 1e-9 relative (stated tolerance)."""
    from oracle import pyoracle
    n = 2000
    D = _euclid(n, 5)
    got, fn, fd, _ = dev.tree(D, n, method=2, exact=False)
    ref, rfn, rfd = pyoracle.tree(D, n, method=2)
    assert fn == rfn and (got["i"] == ref["i"]).all() and (got["j"] == ref["j"]).all()
    for f in ("Li", "Lj"):
        np.testing.assert_allclose(got[f], ref[f], rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("method", [0, 1, 2], ids=["nj", "dnj", "hnj"])
@pytest.mark.parametrize("n", [3, 4, 5, 17, 65, 257])
def test_tree_small_n(dev, method, n):
    """Smallest matrices (the loop runs n - 2 joins down to the final pair) and
    sizes around the wave / block edges, every method, vs the oracle."""
    from oracle import pyoracle
    for seed in range(3):
        D = _euclid(n, 100 * n + seed)
        got, fn, fd, _ = dev.tree(D, n, method=method, exact=True)
        ref, rfn, rfd = pyoracle.tree(D, n, method=method)
        assert (fn, fd) == (rfn, rfd) and len(got) == len(ref) and (got == ref).all()


@pytest.mark.parametrize("L,proxi", [(1, 1), (31, 3), (32, 40), (33, 1), (64, 63), (65, 2)])
def test_dist_pair_proxi_short(dev, L, proxi):
    """Pair mode with -P on alignments shorter than or just past one word (the
    sentinel lastSNP = len + proxi reaches past the counted words)."""
    from oracle import pyoracle
    rng = np.random.default_rng(L * 7 + proxi)
    n = 9
    seqs, incs = _related_msa(rng, n, L, 0.3, nrate=0.1)
    Dg, Ng, _ = dev.snp_ltd(seqs, incs, n, L, pair=True, proxi=proxi, want_n=True)
    Do, No, _ = pyoracle.snp_ltd(seqs, incs, n, L, pair=True, proxi=proxi, want_n=True)
    assert (Dg == Do).all() and (Ng == No).all()


@pytest.mark.parametrize("n,kind", [(2000, "euc"), (1200, "snp")])
def test_nj_fast_sums(dev, n, kind):
    """-m nj with fast (fixed-order) row sums: same joins as the reference;
    lengths within 1e-9 relative (the stated tolerance; on SNP data the
    averaged distances grow dyadic denominators until sums round, so fast
    and serial sums differ in the last bits there too).  On clade-structured
    data with exact Q ties those last bits can reorder tied joins, which is
    why the CLI default is the exact (serial) sum and --fast_sums is opt-in."""
    from oracle import pyoracle
    D = {"euc": lambda: _euclid(n, 7), "snp": lambda: _snp(n, 9), "clade": lambda: _clade_ltd(n, 3)}[kind]()
    got, fn, fd, _ = dev.tree(D, n, method=0, exact=False)
    ref, rfn, rfd = pyoracle.tree(D, n, method=0)
    assert fn == rfn and len(got) == len(ref)
    assert (got["i"] == ref["i"]).all() and (got["j"] == ref["j"]).all()
    for f in ("Li", "Lj"):
        np.testing.assert_allclose(got[f], ref[f], rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("et", [4, 2, 1])
def test_nj_fast_sums_types(dev, et):
    n = 600
    D = _snp(n, 21)
    bs = {4: 1.0, 2: 4.0, 1: 1.0}[et]
    Dt = D.astype(np.float32) if et == 4 else np.clip(D * bs + 0.5, 0, 255 if et == 1 else 65535).astype(
        np.uint8 if et == 1 else np.uint16)
    fast = dev.tree(Dt, n, etype=et, byte_scale=bs, method=0, exact=False)
    exact = dev.tree(Dt, n, etype=et, byte_scale=bs, method=0, exact=True)
    assert fast[1] == exact[1] and (fast[0]["i"] == exact[0]["i"]).all() and (fast[0]["j"] == exact[0]["j"]).all()
    for f in ("Li", "Lj"):
        np.testing.assert_allclose(fast[0][f], exact[0][f], rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("kind,n,band", [("euc", 1500, False), ("clade", 2000, False), ("snp", 1200, False),
                                         ("euc", 2000, True), ("clade", 2500, True)])
def test_dnj_reference_rule_counters(dev, monkeypatch, kind, n, band):
    """stats[10/11 + 2 NKSTAT]: the rows and cells the reference's minQpair
    rescans (dnj.c:78), counted from the engine's replay decisions, equal the
    oracle's serial count (SURVEY 8(d)'s DNJ unit); single GPU and sharded
    kernels, with the small-n and the band choice of S."""
    from oracle import pyoracle
    from ccphylo_amd import native
    K = native.NKSTAT
    D = _euclid(n, n) if kind == "euc" else _clade_ltd(n, n) if kind == "clade" else _snp(n, n)
    if band:
        monkeypatch.setenv("CCG_S_SPLIT_N", "1000")
    ref, rfn, rfd, rst = pyoracle.tree(D, n, method=1, stats=True)
    got, fn, fd, st = dev.tree(D, n, method=1, exact=True, profile=True)
    assert len(got) == len(ref) and (got == ref).all()
    assert (st[10 + 2 * K], st[11 + 2 * K]) == (int(rst[0]), int(rst[1]))
    assert st[1] >= st[11 + 2 * K]   # the engine rescans a superset
    monkeypatch.setenv("CCG_SHARD_FORCE", "1")
    sh = dev.tree_shard(D, n, None, method=1, exact=True, profile=True)
    assert (sh[0] == got).all()
    assert (sh[3][10 + 2 * K], sh[3][11 + 2 * K]) == (int(rst[0]), int(rst[1]))


@pytest.mark.parametrize("n,jpf", [(900, "1"), (1400, "2"), (1400, "0")])
def test_dnj_missing_large_n_join(dev, monkeypatch, n, jpf):
    """Missing entries (updateD's general body, k_update_general) through the
    large-n join forms at small n: k_dnj_fold's chunk summaries with
    k_dnj_join_pf (1), its block-0 replay path (2), the per-block replay (0);
    joins bit-identical to the serial reference."""
    from oracle import pyoracle
    monkeypatch.setenv("CCG_PREFOLD_N", "0")
    monkeypatch.setenv("CCG_JOIN_PF", jpf)
    D = _missing_ltd(n, n)
    got, fn, fd, _ = dev.tree(D, n, method=1, exact=True)
    ref, rfn, rfd = pyoracle.tree(D, n, method=1)
    assert (fn, fd) == (rfn, rfd)
    assert len(got) == len(ref) and (got == ref).all()


@pytest.mark.parametrize("mode", ["20", "21"])
@pytest.mark.parametrize("kind,n,et", [("euc", 2500, 8), ("clade", 3000, 8), ("euc", 2000, 4), ("clade", 2500, 2),
                                       ("clade", 2000, 1)])
def test_dnj_scan_row_groups(dev, monkeypatch, mode, kind, n, et):
    """The row-group rescan (k_dnj_scan_g: G rows per wave sharing the sD
    loads of a column range; the default past 16384 taxa for float, u16 and
    u8 rows) at small n with the large-n fold and join: joins bit-identical
    to the serial reference."""
    from oracle import pyoracle
    monkeypatch.setenv("CCG_SCAN_WAVE", mode)
    monkeypatch.setenv("CCG_PREFOLD_N", "0")
    monkeypatch.setenv("CCG_SEG_MUL", "1")
    D = _euclid(n, n) if kind == "euc" else _clade_ltd(n, n)
    bs = {8: 1.0, 4: 1.0, 2: 4.0, 1: 0.1}[et]
    if et == 4:
        D = D.astype(np.float32)
    elif et in (2, 1):   # dtouc(d, 0.5) stores (bytescale.c)
        D = np.clip(D * bs + 0.5, 0, 255 if et == 1 else 65535).astype(np.uint8 if et == 1 else np.uint16)
    got, fn, fd, _ = dev.tree(D, n, etype=et, byte_scale=bs, method=1, exact=True)
    ref, rfn, rfd = pyoracle.tree(D, n, etype=et, byte_scale=bs, method=1)
    assert (fn, fd) == (rfn, rfd)
    assert len(got) == len(ref) and (got == ref).all()


def _state_equal(g, r, n):
    """An engine checkpoint (ccg_dnj_state + its device LT) against the
    oracle's DnjState after the same joins: every vector bit for bit."""
    assert g["n"] == r.n == n
    assert g["cand"] == r.cand
    assert (g["sD"] == r.sD[:n]).all() and (g["Q"] == r.Q[:n]).all()
    assert (g["N"] == r.N[:n]).all() and (g["P"] == r.P[:n]).all()


@pytest.mark.parametrize("kind,n,et,cuts", [("clade", 2500, 8, (300, 1100)), ("euc", 2000, 4, (1, 700)),
                                            ("miss", 1500, 8, (200, 900)), ("snp", 1800, 8, (1, 1000))])
def test_dnj_checkpoint_vs_oracle(dev, kind, n, et, cuts):
    """ccg_tree_dev_state: the engine's DNJ loop state after k joins (D, sD, Q,
    N, P and minPos's candidate, dnj.c:985-1052) equals the oracle's after the
    same k joins bit for bit; the run resumed from it (and the oracle resumed
    from the engine's state) continue with the uninterrupted run's joins."""
    import torch
    from oracle import pyoracle
    D = {"euc": lambda: _euclid(n, n), "snp": lambda: _snp(n, n), "clade": lambda: _clade_ltd(n, n),
         "miss": lambda: _missing_ltd(n, n)}[kind]()
    D = D.astype(np.float32) if et == 4 else D
    whole, wfn, wfd = pyoracle.tree(D, n, etype=et, method=1)
    ost = pyoracle.dnj_init(D.copy(), n, etype=et)
    Dd = torch.from_numpy(np.ascontiguousarray(D)).cuda()
    torch.cuda.synchronize()
    state, done, m = None, [], n
    for k in list(cuts) + [0]:
        got, fn, fd, _, st = dev.tree_dev_state(Dd.data_ptr(), m, etype=et, max_joins=k, state=state)
        ref, rfn, rfd = pyoracle.dnj_resume(ost, max_joins=k)
        assert len(got) == len(ref) and (got == ref).all(), (kind, k)
        done.append(got)
        if k:
            _state_equal(st, ost, m - k)
            mm = m - k
            cells = Dd[:mm * (mm - 1) // 2].cpu().numpy()
            assert (cells == ost.D[:mm * (mm - 1) // 2]).all()
            # the oracle continues 150 joins from the ENGINE's state
            gst = pyoracle.DnjState(cells.copy(), mm, st["sD"].copy(), st["Q"].copy(), st["N"].copy(),
                                    st["P"].copy(), st["cand"], etype=et)
            ref2 = pyoracle.dnj_resume(gst, max_joins=150)[0]
            assert (ref2 == whole[sum(len(x) for x in done):][:150]).all()
            m, state = mm, st
        else:
            assert (fn, fd) == (wfn, wfd) and (rfn, rfd) == (wfn, wfd)
    assert (np.concatenate(done) == whole).all()


def test_dnj_checkpoint_large_n(dev):
    """The checkpoint at n > 16384 (band rows of S, k_dnj_fold, k_dnj_join_pf):
    20k Euclidean doubles, state after 400 joins against the oracle's, then
    400 more joins from it on both sides."""
    import torch
    from oracle import pyoracle
    n, k = 20_000, 400
    D = _euclid(n, 3)
    Dd = torch.from_numpy(D).cuda()
    torch.cuda.synchronize()
    got, _, _, _, st = dev.tree_dev_state(Dd.data_ptr(), n, max_joins=k)
    ost = pyoracle.dnj_init(D, n, threads=8)
    ref = pyoracle.dnj_resume(ost, max_joins=k, threads=8)[0]
    assert (got == ref).all()
    _state_equal(st, ost, n - k)
    got2 = dev.tree_dev_state(Dd.data_ptr(), n - k, max_joins=k, state=st, want_state=False)[0]
    ref2 = pyoracle.dnj_resume(ost, max_joins=k, threads=8)[0]
    assert (got2 == ref2).all()


@pytest.mark.parametrize("n,L,et,excl,norm", [(300, 5000, 8, 10, 0), (777, 4097, 4, 3, 0), (2100, 3200, 8, 7, 1000),
                                              (129, 64, 2, 1, 0), (500, 100, 1, 100, 0), (257, 9000, 8, 0, 0)])
def test_dist_compacted_words(dev, monkeypatch, n, L, et, excl, norm):
    """Non-pair dist keeps only the words the global mask does not exclude
    entirely in its bit planes (fsacmp.c:552 counts included positions only):
    the matrix equals the uncompacted planes' (CCG_DIST_NOCOMPACT=1) and the
    oracle's bit for bit; every `excl`-th word excluded, partial words kept
    masked, all words excluded (excl = 1), none (0); the device-, host- and
    shard-input paths."""
    from oracle import pyoracle
    from tools.synth import clade_packed
    seqs, incs = clade_packed(n, L, 8, seed=n, every=excl)
    incs[1::5] &= np.uint32(0x0FF0F00F)   # partial words
    bs = {8: 1.0, 4: 1.0, 2: 4.0, 1: 0.05}[et]
    want = pyoracle.snp_ltd(seqs, incs, n, L, norm=norm, etype=et, byte_scale=bs)[0]
    got = dev.snp_ltd(seqs, incs, n, L, norm=norm, etype=et, byte_scale=bs)[0]
    monkeypatch.setenv("CCG_DIST_NOCOMPACT", "1")
    whole = dev.snp_ltd(seqs, incs, n, L, norm=norm, etype=et, byte_scale=bs)[0]
    monkeypatch.delenv("CCG_DIST_NOCOMPACT")
    assert (got.view(np.uint8) == want.view(np.uint8)).all()
    assert (whole.view(np.uint8) == want.view(np.uint8)).all()
    if et in (8, 4):   # the band shard from host memory (ccg_snp_ltd_shard), world 3
        import torch
        from ccphylo_amd import native as nt
        for rank in range(3):
            elems = nt.shard_elems(n, rank, 3)
            Dl = torch.zeros(max(elems, 1), dtype=torch.float64 if et == 8 else torch.float32, device="cuda")
            dev.snp_ltd_shard(seqs, incs, n, L, Dl.data_ptr(), rank, 3, etype=et, norm=norm)
            loc = Dl.cpu().numpy()
            for r in range(1, n):
                if nt.shard_owner(r, 3) == rank:
                    o = nt.shard_row_offset(r, rank, 3)
                    assert (loc[o:o + r] == want[r * (r - 1) // 2:r * (r - 1) // 2 + r]).all(), (rank, r)


@pytest.mark.parametrize("kind,n,et,mode", [("euc", 2500, 8, "9"), ("clade", 3000, 8, "4"), ("euc", 2000, 4, "20"),
                                            ("clade", 2200, 8, "1"), ("miss", 1400, 8, "1"), ("snp", 1800, 2, "20")])
def test_dnj_scan_tail_fold(dev, monkeypatch, kind, n, et, mode):
    """The fold of each entry's unit partials and the 64-entry chunk
    summaries at the scan's last arrivals (FoldTail, the default past 16384
    taxa) instead of a k_dnj_fold pass, at small n through CCG_PREFOLD_N=0
    and small rescan units (many units per row, many arrivals per entry):
    wave scans with 16-byte loads (9, 4), row groups (20), the GEN wave scan
    with missing entries (1); joins bit-identical to the serial reference and
    to CCG_SCAN_FOLD=0 (k_dnj_fold)."""
    from oracle import pyoracle
    monkeypatch.setenv("CCG_SCAN_WAVE", mode)
    monkeypatch.setenv("CCG_PREFOLD_N", "0")
    monkeypatch.setenv("CCG_SEG_MUL", "1")
    D = {"euc": lambda: _euclid(n, n + 1), "snp": lambda: _snp(n, n), "clade": lambda: _clade_ltd(n, n + 2),
         "miss": lambda: _missing_ltd(n, n)}[kind]()
    bs = {8: 1.0, 4: 1.0, 2: 4.0}[et]
    if et == 4:
        D = D.astype(np.float32)
    elif et == 2:
        D = np.clip(D * bs + 0.5, 0, 65535).astype(np.uint16)
    ref, rfn, rfd = pyoracle.tree(D, n, etype=et, byte_scale=bs, method=1)
    for fold in ("1", "0"):
        monkeypatch.setenv("CCG_SCAN_FOLD", fold)
        got, fn, fd, _ = dev.tree(D, n, etype=et, byte_scale=bs, method=1, exact=True)
        assert (fn, fd) == (rfn, rfd), fold
        assert len(got) == len(ref) and (got == ref).all(), fold


@pytest.mark.parametrize("kind,n,et,mode,bands", [("clade", 3000, 8, "9", 64), ("euc", 2500, 8, "9", 64),
                                                  ("clade", 2600, 4, "20", 64), ("euc", 2200, 4, "20", 32),
                                                  ("snp", 2000, 2, "20", 64), ("clade", 2400, 8, "4", 120),
                                                  ("clade", 2000, 1, "21", 64)])
def test_dnj_scan_prune(dev, monkeypatch, kind, n, et, mode, bands):
    """Band mode's in-scan pruning: the scan rescans S (top + band rows) first,
    builds the bound table from their exact fresh minima (max(fresh, Q),
    prefix-min from m0), and an entry whose stale Q is not below it at its row
    (so minQpair skips it, dnj.c:78) loads nothing.  At small n through
    CCG_S_SPLIT_N / CCG_PREFOLD_N: joins and the reference-rule counters equal
    the serial oracle's, CCG_SCAN_PRUNE=0 gives the same joins, and the
    pruned run loads no more cells; with the requeue's V block minima
    (CCG_SCAN_VBLK, the bound from every row above) fewer still."""
    from oracle import pyoracle
    from ccphylo_amd import native
    K = native.NKSTAT
    monkeypatch.setenv("CCG_SCAN_WAVE", mode)
    monkeypatch.setenv("CCG_PREFOLD_N", "0")
    monkeypatch.setenv("CCG_SEG_MUL", "1")
    monkeypatch.setenv("CCG_S_SPLIT_N", "100")
    monkeypatch.setenv("CCG_S_BANDS", str(bands))
    monkeypatch.setenv("CCG_PRUNE_CELLS", "0")   # prune every join (not only while the listings are long)
    D = {"euc": lambda: _euclid(n, n + 3), "snp": lambda: _snp(n, n + 1), "clade": lambda: _clade_ltd(n, n + 4)}[kind]()
    bs = {8: 1.0, 4: 1.0, 2: 4.0, 1: 0.1}[et]
    if et == 4:
        D = D.astype(np.float32)
    elif et in (2, 1):
        D = np.clip(D * bs + 0.5, 0, 255 if et == 1 else 65535).astype(np.uint8 if et == 1 else np.uint16)
    ref, rfn, rfd, rst = pyoracle.tree(D, n, etype=et, byte_scale=bs, method=1, stats=True)
    cells = {}
    # prune 1: the S phase inside the scan (with its fold at the last arrivals);
    # prune 2: S rescanned by k_dnj_sphase, its own launch (wave scans only)
    for prune, vblk, fold in (("1", "1", "1"), ("1", "0", "1"), ("2", "1", "0"), ("2", "0", "0"), ("0", "0", "0")):
        monkeypatch.setenv("CCG_SCAN_PRUNE", prune)
        monkeypatch.setenv("CCG_SCAN_VBLK", vblk)   # + the requeue's V block minima
        monkeypatch.setenv("CCG_SCAN_FOLD", fold)
        got, fn, fd, st = dev.tree(D, n, etype=et, byte_scale=bs, method=1, exact=True, profile=True)
        assert (fn, fd) == (rfn, rfd), (prune, vblk)
        assert len(got) == len(ref) and (got == ref).all(), (prune, vblk)
        assert (st[10 + 2 * K], st[11 + 2 * K]) == (int(rst[0]), int(rst[1])), (prune, vblk)
        cells[prune + vblk] = st[1]
    assert int(rst[1]) <= cells["11"] <= cells["10"] <= cells["00"]
    # the split form (the plan's helpers + k_dnj_sphase; for row groups the
    # compacted group scan k_dnj_scan_gc over the survivors) prunes exactly as
    # the in-scan one
    assert (cells["21"], cells["20"]) == (cells["11"], cells["10"])
    # without the compacted enumeration: the wave scan rechecks the table and
    # k_dnj_sphase alone counts the pruned cells; row groups then
    # run unpruned (k_dnj_scan_g)
    monkeypatch.setenv("CCG_SCAN_PRUNE", "2")
    monkeypatch.setenv("CCG_SCAN_VBLK", "1")
    monkeypatch.setenv("CCG_SCAN_FOLD", "0")
    monkeypatch.setenv("CCG_SCAN_CMP", "0")
    got, fn, fd, st = dev.tree(D, n, etype=et, byte_scale=bs, method=1, exact=True, profile=True)
    assert (fn, fd) == (rfn, rfd) and (got == ref).all()
    assert (st[10 + 2 * K], st[11 + 2 * K]) == (int(rst[0]), int(rst[1]))
    assert st[1] == (cells["21"] if int(mode) < 20 else cells["00"])


@pytest.mark.parametrize("kind,n,et,mode", [("clade", 3000, 8, "9"), ("euc", 2500, 8, "9"), ("euc", 2600, 4, "20"),
                                             ("snp", 2000, 2, "20"), ("clade", 2200, 1, "9"), ("euc", 3000, 8, "4"),
                                             ("snp", 2400, 8, "9")])
def test_dnj_block_bounds(dev, monkeypatch, kind, n, et, mode):
    """The scan under the block lower bounds (TreeBufs::lbm, lb_unit): a
    64-column block is skipped when ((n-2) m_d - sD_r) - M_sD exceeds the q at
    the row's partner cell, with the bounds kept conservatively by the join
    (row j, column j) and the requeue (row i, column i, the sD maxima).  At
    small n through CCG_LB_MIN_N: joins, lengths and the reference-rule
    counters equal the serial oracle's with pruning on and off, and the
    bounded scan loads fewer cells than the unbounded one."""
    from oracle import pyoracle
    from ccphylo_amd import native
    K = native.NKSTAT
    for k, v in (("CCG_SCAN_WAVE", mode), ("CCG_PREFOLD_N", "0"), ("CCG_SEG_MUL", "1"), ("CCG_S_SPLIT_N", "100"),
                 ("CCG_PRUNE_CELLS", "0"), ("CCG_LB_MIN_N", "100")):
        monkeypatch.setenv(k, v)
    D = {"euc": lambda: _euclid(n, n + 7), "snp": lambda: _snp(n, n + 5), "clade": lambda: _clade_ltd(n, n + 6)}[kind]()
    bs = {8: 1.0, 4: 1.0, 2: 4.0, 1: 0.1}[et]
    if et == 4:
        D = D.astype(np.float32)
    elif et in (2, 1):
        D = np.clip(D * bs + 0.5, 0, 255 if et == 1 else 65535).astype(np.uint8 if et == 1 else np.uint16)
    ref, rfn, rfd, rst = pyoracle.tree(D, n, etype=et, byte_scale=bs, method=1, stats=True)
    for prune in ("2", "0"):
        monkeypatch.setenv("CCG_SCAN_PRUNE", prune)
        cells = {}
        # row-group modes unpruned: the bounded row groups (lb_unit_g, "1g") and one bounded row per wave ("1")
        forms = ("1g", "1", "0") if int(mode) >= 20 and prune == "0" else ("1", "0")
        for lb in forms:
            monkeypatch.setenv("CCG_SCAN_LB", lb[0])
            monkeypatch.setenv("CCG_LB_GROUPS", "1" if lb == "1g" else "0")
            got, fn, fd, st = dev.tree(D, n, etype=et, byte_scale=bs, method=1, exact=True, profile=True)
            assert (fn, fd) == (rfn, rfd), (prune, lb)
            assert len(got) == len(ref) and (got == ref).all(), (prune, lb)
            assert (st[10 + 2 * K], st[11 + 2 * K]) == (int(rst[0]), int(rst[1])), (prune, lb)
            cells[lb] = st[1]
        assert cells["1"] < cells["0"], (prune, cells)
        if "1g" in cells:   # each row loads exactly the blocks lb_unit loads for it
            assert cells["1g"] == cells["1"], cells


@pytest.mark.parametrize("allpre", ["1", "0"])
@pytest.mark.parametrize("kind", ["euc", "clade"])
def test_exact_walk_forms(dev, monkeypatch, allpre, kind):
    """The exact row sum's walk over the binade records (xs_walk_blocks), with
    every block's records loaded at once (CCG_XS_ALLPRE=1) and block by block
    (the default): whole exact DNJ trees equal the serial oracle's."""
    from oracle import pyoracle
    monkeypatch.setenv("CCG_XS_ALLPRE", allpre)
    n = 2500
    D = _euclid(n, n + 11) if kind == "euc" else _clade_ltd(n, n + 12)
    ref, rfn, rfd = pyoracle.tree(D, n, method=1)
    got, fn, fd, _ = dev.tree(D, n, method=1, exact=True)
    assert (fn, fd) == (rfn, rfd)
    assert len(got) == len(ref) and (got == ref).all()


@pytest.mark.parametrize("withhold", ["1", "2"])
def test_dnj_plan_wait_timeout_is_an_error(dev, monkeypatch, withhold):
    """A bounded wait of k_dnj_plan that gives up stops the tree with an
    error, never a silently different tree: CCG_TEST_WITHHOLD=1 makes block 0
    withhold its entry count (the other listing blocks' look-back), =2 the S
    header's tag (the helper blocks' wait for S).  CCG_PLAN_FR=1 gives several
    listing blocks at n = 3000, band mode with pruning brings the helpers."""
    from ccphylo_amd import CcgError
    n = 3000
    for k, v in (("CCG_SCAN_WAVE", "9"), ("CCG_PREFOLD_N", "0"), ("CCG_SEG_MUL", "1"), ("CCG_S_SPLIT_N", "100"),
                 ("CCG_PRUNE_CELLS", "0"), ("CCG_PLAN_FR", "1")):
        monkeypatch.setenv(k, v)
    D = _clade_ltd(n, 5)
    got, fn, _, _ = dev.tree(D, n, method=1, exact=True)   # the same settings without the knob: a tree
    assert fn == 2 and len(got) == n - 2
    monkeypatch.setenv("CCG_TEST_WITHHOLD", withhold)
    with pytest.raises(CcgError):
        dev.tree(D, n, method=1, exact=True)
