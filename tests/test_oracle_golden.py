"""CPU: the oracle (oracle/ccoracle.c) + the product host layer reproduce every
golden vector the reference binary produced (tests/golden/golden.json)."""
import pytest

from conftest import golden_bytes, golden_cases, parse_dist_args, parse_tree_args, print_phylip


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
