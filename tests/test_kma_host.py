"""CPU: the product's KMA loader (ccq_load_kma) against the oracle.

The GPU kernel compares the loader's two views per pair (rec1 of the row
sample after stripMat, rec2 of the column sample), so a direct evaluation of
cmpMats (matcmp.c:448) over those views -- sequential, in Python -- must give
the oracle's matrix bit for bit.  This pins the loader (parsing, the
stripMat stride quirk, inclusion rules, lengths) without a GPU."""
import glob
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN

FILES = sorted(glob.glob(os.path.join(GOLDEN, "kma*.mat*")))


def _i32(x):
    return (x + 2**31) % 2**32 - 2**31


def _cos(x, y):
    d = 0.0
    c1 = c2 = 0
    for k in range(5):
        d += _i32(int(x[k]) * int(y[k]))
        c1 += _i32(int(x[k]) ** 2) % 2**64
        c2 += _i32(int(y[k]) ** 2) % 2**64
    c1 %= 2**64
    c2 %= 2**64
    if not c1 or not c2:
        return -1.0
    d = 1 - d / (math.sqrt(float(c1)) * math.sqrt(float(c2)))
    return 0.0 if d < 0 else d


def _l1(x, y):
    return float(sum(abs(int(x[k]) - int(y[k])) for k in range(5)))


def view_matrix(K, metric, min_depth=15, min_length=1, min_cov=0.5):
    n = K["n"]
    out = []
    f = {"cos": _cos, "l1": _l1}[metric]
    for i in range(1, n):
        for j in range(i):
            l1, l2 = int(K["len1"][i]), int(K["len2"][j])
            if l2 > l1:
                out.append(-1.0)
                continue
            dist, inc, nn = 0.0, 0, 0
            for r in range(l2):
                x, y = K["rec1"][i, r], K["rec2"][j, r]
                t1 = int(x[6]) | int(x[7]) << 16
                t2 = int(y[6]) | int(y[7]) << 16
                if min_depth <= t2:
                    nn += 1
                    if min_depth <= t1:
                        d = f(x, y)
                        if d >= 0:
                            dist += d
                            inc += 1
            assert not (nn < min_length or nn < min_cov * l2)
            out.append(-1.0 if (inc < min_length or inc < min_cov * l2) else dist)
    return np.array(out)


@pytest.mark.parametrize("tmpl,metric", [("tmpl_one", "cos"), ("tmpl_two", "cos"), ("tmpl_two", "l1")])
def test_loader_views_match_oracle(tmpl, metric):
    import ccphylo_amd as cg
    from oracle import pyoracle
    K = cg.native.load_kma(FILES, tmpl)
    D, _, inc, n = pyoracle.kma_dist(FILES, tmpl, metric=metric)
    assert K["n"] == n and (K["include"] == inc).all()
    got = view_matrix(K, metric)
    assert np.array_equal(got, D)


def test_loader_missing_file():
    import ccphylo_amd as cg
    with pytest.raises(cg.CcgError):
        cg.native.load_kma(FILES[:2] + ["/nonexistent.mat.gz"], "tmpl_one")
