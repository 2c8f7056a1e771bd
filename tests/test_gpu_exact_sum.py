"""GPU: the exact-mode row sum (ccg_tree_common.h exact_sum_block) equals the
reference's serial sum s = ((0 + c0) + c1) + ... (nj.c:911 / :1002) bit for
bit, and the parallel binade-segmented form (not the serial fallback chain)
produces it on ordinary inputs: uniform, %.9f-quantized, wide-range, dyadic
(many exact half-ulp ties), leading and scattered zeros, n = 1 .. 300k."""
import math
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["block1024", "block256"])
def dev(request):
    """The 1024-thread k_exact_sum of the single-GPU engine, and the per-block
    (256-thread) form the sharded engines run."""
    if request.param == "block256":
        os.environ["CCG_SELFTEST_TB256"] = "1"
    else:
        os.environ.pop("CCG_SELFTEST_TB256", None)
    import ccphylo_amd as cg
    d = cg.Device(0)
    yield d
    d.close()
    os.environ.pop("CCG_SELFTEST_TB256", None)


def _serial(c):
    s = 0.0
    for x in c.tolist():
        s += x
    return s


def _case(kind, n, rng):
    if kind == "uniform":
        c = rng.random(n)
    elif kind == "phylip":
        c = np.round(rng.random(n) * 1e9) / 1e9
    elif kind == "dyadic":   # sums of few bits: exact ties at many ulps
        c = rng.integers(0, 9, n) * np.ldexp(1.0, -rng.integers(0, 61, n))
    elif kind == "wide":
        c = rng.random(n) * 10.0 ** rng.integers(-6, 6, n)
    elif kind == "zeros":
        c = rng.random(n)
        c[rng.random(n) < 0.3] = 0.0
        c[: n // 10] = 0.0
    else:   # "integers": provable in any order, still through the same code
        c = rng.integers(0, 5000, n).astype(np.float64)
    return c


@pytest.mark.parametrize("kind", ["uniform", "phylip", "dyadic", "wide", "zeros", "integers"])
def test_exact_sum_matches_serial(dev, kind):
    rng = np.random.default_rng(abs(hash(kind)) % 2 ** 32)
    par_used = 0
    sizes = [1, 2, 3, 7, 64, 255, 256, 257, 1000, 4097, 9998, 30000]
    for n in sizes:
        for rep in range(3):
            c = _case(kind, n, rng)
            got, par = dev.selftest_row_sum(c)
            want = _serial(c)
            assert got == want and math.copysign(1, got) == math.copysign(1, want), (kind, n, rep, got, want)
            par_used += par
    # the parallel form must carry ordinary inputs (the chain is the rare
    # fallback); dyadic inputs at large n hold more half-ulp ties than the
    # tie list (XS_CAP) and fall back by design
    assert par_used >= (0.6 if kind == "dyadic" else 0.9) * 3 * len(sizes), (kind, par_used)


def test_exact_sum_large_n(dev):
    rng = np.random.default_rng(11)
    c = np.round(rng.random(300_000) * 1e9) / 1e9
    got, par = dev.selftest_row_sum(c)
    assert par and got == _serial(c)


def test_exact_sum_declines_bad_input(dev):
    """Negative or non-finite contributions cannot occur in updateD's clamped
    sums; the parallel form declines them and the chain gives IEEE's answer."""
    rng = np.random.default_rng(5)
    c = rng.random(300)
    c[150] = -0.5          # past the serially summed head (XS_HEAD = 64)
    got, par = dev.selftest_row_sum(c)
    assert not par and got == _serial(c)
    c[150] = np.inf
    got, par = dev.selftest_row_sum(c)
    assert not par and got == np.inf
    c = np.array([1.0, -0.5, 2.0, 3.0])   # inside the head: summed serially as given
    got, par = dev.selftest_row_sum(c)
    assert got == _serial(c)
