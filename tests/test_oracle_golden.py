"""CPU: the oracle (oracle/ccoracle.c) + the product host layer reproduce every
golden vector the reference binary produced (tests/golden/golden.json)."""
import pytest

from conftest import golden_bytes, golden_cases, parse_dist_args, parse_kma_args, parse_tree_args, print_phylip


@pytest.mark.parametrize("case", golden_cases("tree"), ids=lambda c: c["name"])
def test_tree_oracle_matches_reference(case):
    from oracle import pyoracle
    import ccphylo_amd as cg
    path, method, et, bs, flags, prec = parse_tree_args(case["args"])
    trees = cg.newick_from_phylip(path, lambda D, n: pyoracle.tree(D, n, etype=et, byte_scale=bs, method=method,
                                                                    flags=flags),
                                  etype=et, byte_scale=bs, flags=flags, precision=prec)
    assert ("\n".join(trees) + "\n").encode() == golden_bytes(case)


@pytest.mark.parametrize("case", golden_cases("dist"), ids=lambda c: c["name"])
def test_dist_oracle_matches_reference(case):
    from oracle import pyoracle
    import ccphylo_amd as cg
    o = parse_dist_args(case["args"])
    heads, seqs, incs, L, minLength = cg.load_msa(o["inp"], o["flag"], o["minLength"], o["minCov"], o["proxi"])
    n = len(heads)
    pair = bool(o["flag"] & 2)
    D, N, inc = pyoracle.snp_ltd(seqs, incs, n, L, pair=pair, norm=o["norm"], min_length=minLength,
                                 min_cov=0.0, proxi=o["proxi"] if pair else 0, etype=o["et"], byte_scale=o["bs"],
                                 want_n=o["nout"] and pair)
    out = b""
    if n > 1:
        out = print_phylip(D, n, heads, o["flag"], o["prec"], o["et"], o["bs"])
        if N is not None:
            out += print_phylip(N, n, heads, o["flag"], o["prec"], o["et"], o["bs"])
    assert out == golden_bytes(case)


def kma_phylip(o, D, N, include, n):
    """The bytes `ccphylo dist` prints for a KMA run (dist.c:175-179)."""
    names = [f for f in o["files"]]
    out = b""
    if n > 1:
        out = print_phylip(D, n, names, o["flag"], o["prec"], o["et"], o["bs"], include=include, comment=o["tmpl"])
        if N is not None:
            out += print_phylip(N, n, names, o["flag"], o["prec"], o["et"], o["bs"], include=include,
                                comment=o["tmpl"])
    return out


@pytest.mark.parametrize("case", golden_cases("kma"), ids=lambda c: c["name"])
def test_kma_oracle_matches_reference(case):
    from oracle import pyoracle
    o = parse_kma_args(case["args"])
    D, N, inc, n = pyoracle.kma_dist(o["files"], o["tmpl"], metric=o["metric"], norm=o["norm"],
                                     min_depth=o["minDepth"], min_length=o["minLength"], min_cov=o["minCov"],
                                     etype=o["et"], byte_scale=o["bs"], want_n=o["nout"])
    assert kma_phylip(o, D, N, inc, n) == golden_bytes(case)


@pytest.mark.parametrize("method", [0, 1, 2])
@pytest.mark.parametrize("et", [8, 4, 2])
def test_oracle_threaded_init_and_prefix(method, et):
    """orc_tree_ex (the large-n checker of tests/test_gpu_large.py): the
    threaded initSummaD / initHNJ give the serial run bit for bit, and a
    max_joins run is a prefix of the full run (missing entries included)."""
    import numpy as np
    from oracle import pyoracle
    from tools.synth import euclid
    n = 1500
    D = euclid(n, 5)
    D[::97] = -1.0
    bs = 1.0
    if et == 4:
        D = D.astype(np.float32)
    elif et == 2:
        bs = 100.0
        D = np.where(D < 0, 65535, np.round(D * bs)).astype(np.uint16)
    full = pyoracle.tree(D, n, etype=et, byte_scale=bs, method=method)
    par = pyoracle.tree(D, n, etype=et, byte_scale=bs, method=method, threads=5)
    pre = pyoracle.tree(D, n, etype=et, byte_scale=bs, method=method, threads=3, max_joins=40)
    assert (full[0] == par[0]).all() and full[1:] == par[1:]
    assert len(pre[0]) == 40 and (pre[0] == full[0][:40]).all()


def _snp_clade_ltd(n, L, clades, seed=5):
    """An integer SNP-count LT with many exact ties (clade-structured random
    packed alignment through the oracle's fsacmp)."""
    import numpy as np
    from oracle import pyoracle
    from tools.synth import clade_packed
    seqs, incs = clade_packed(n, L, clades, seed)
    D, _, _ = pyoracle.snp_ltd(seqs, incs, n, L)
    return D


@pytest.mark.parametrize("kind", ["euc", "snp"])
def test_oracle_parallel_min_q_pair(monkeypatch, kind):
    """min_q_pair_par (threaded speculative rescans + the serial loop's own
    accept order, the large-n checker) equals min_q_pair (dnj.c:43-128) bit
    for bit: joins, lengths, final pair and the reference-rule counters."""
    import numpy as np
    from oracle import pyoracle
    from tools.synth import euclid
    monkeypatch.setenv("ORC_PAR_CELLS", "0")   # every batch through the threads
    n = 1200
    D = euclid(n, 7) if kind == "euc" else _snp_clade_ltd(n, 600, 24)
    ser = pyoracle.tree(D, n, method=1, stats=True)
    par = pyoracle.tree(D, n, method=1, stats=True, threads=4)
    assert (ser[0] == par[0]).all() and ser[1:3] == par[1:3]
    assert (ser[3] == par[3]).all()


@pytest.mark.parametrize("threads", [1, 3])
def test_oracle_dnj_resume_chain(monkeypatch, threads):
    """orc_dnj_init + orc_dnj_resume in three legs (state carried between
    them: D, sD, Q, N, P and minPos's candidate) give the one-run tree."""
    import numpy as np
    from oracle import pyoracle
    monkeypatch.setenv("ORC_PAR_CELLS", "0")
    n = 900
    D = _snp_clade_ltd(n, 800, 16, seed=8)
    whole = pyoracle.tree(D, n, method=1, stats=True)
    st = pyoracle.dnj_init(D.copy(), n, threads=threads)
    parts, cells = [], np.zeros(2, dtype=np.int64)
    for k in (150, 400, 0):
        j, fn, fd, s = pyoracle.dnj_resume(st, max_joins=k, threads=threads, stats=True)
        parts.append(j)
        cells += s
    got = np.concatenate(parts)
    assert (got == whole[0]).all() and (fn, fd) == whole[1:3]
    assert (cells == whole[3]).all()


def test_oracle_threaded_snp_ltd():
    """orc_snp_ltd_ex over row-interleaved pthreads = the serial fill, both
    modes (pair mode with -P)."""
    import numpy as np
    from oracle import pyoracle
    from tools.synth import clade_packed
    n, L = 300, 700
    seqs, incs = clade_packed(n, L, 8, 3)
    a = pyoracle.snp_ltd(seqs, incs, n, L)[0]
    b = pyoracle.snp_ltd(seqs, incs, n, L, threads=4)[0]
    assert (a == b).all()
    W = L // 32 + 1
    pinc = np.tile(incs, (n, 1))
    pinc[::7, 3] = 0
    a = pyoracle.snp_ltd(seqs, pinc, n, L, pair=True, proxi=5, want_n=True)
    b = pyoracle.snp_ltd(seqs, pinc, n, L, pair=True, proxi=5, want_n=True, threads=3)
    assert (a[0] == b[0]).all() and (a[1] == b[1]).all()
