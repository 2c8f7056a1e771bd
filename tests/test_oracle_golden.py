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
