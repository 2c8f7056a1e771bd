"""GPU parity of count-matrix (KMA *.mat) distances, ccg_kma_ltd:
bit-exact against the reference's golden vectors and the oracle, through the
C-ABI and through the CLI.  l<n> / nl<n> go through pow(), which the GPU
math library does not round like glibc (parity of pow itself is unpinned):
l<n> compares within 1e-12 relative.  nl<n> raises the FIRST difference
without |.| (matcmp.c:113), so a position's sum can cancel to about +-1e-20,
where a one-ulp difference of pow decides between a cube root of ~1e-7 and
NaN (excluded): nl<n> compares within 1e-6 relative."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, golden_bytes, golden_cases, parse_kma_args

pytestmark = pytest.mark.gpu
sys.path.insert(0, GOLDEN)


def _pow_metric(m):
    return m[0] == "l" and m[1:].isdigit() or m.startswith("nl") and m[2:].isdigit()


def _pow_rtol(m):
    return 1e-6 if m.startswith("nl") else 1e-12


@pytest.fixture(scope="module")
def dev():
    import ccphylo_amd as cg
    d = cg.Device(0)
    yield d
    d.close()


def _phylip_values(text):
    vals = []
    for line in text.decode().splitlines()[1:]:
        vals += [float(v) for v in line.split("\t")[1:]]
    return np.array(vals)


@pytest.mark.parametrize("case", golden_cases("kma"), ids=lambda c: c["name"])
def test_kma_golden_engine(dev, case):
    import ccphylo_amd as cg
    from test_oracle_golden import kma_phylip
    o = parse_kma_args(case["args"])
    K = cg.native.load_kma(o["files"], o["tmpl"], min_depth=o["minDepth"], min_length=o["minLength"],
                           min_cov=o["minCov"])
    D, N, fatal = dev.kma_ltd(K, metric=o["metric"], norm=o["norm"], min_depth=o["minDepth"],
                              min_length=o["minLength"], min_cov=o["minCov"], etype=o["et"], byte_scale=o["bs"],
                              want_n=o["nout"])
    assert fatal == -1
    got = kma_phylip(o, D, N, K["include"], K["n"])
    if _pow_metric(o["metric"]):
        np.testing.assert_allclose(_phylip_values(got), _phylip_values(golden_bytes(case)),
                                   rtol=_pow_rtol(o["metric"]))
    else:
        assert got == golden_bytes(case)


@pytest.mark.parametrize("case", golden_cases("kma"), ids=lambda c: c["name"])
def test_kma_golden_cli(case):
    import ccphylo_amd as cg
    p = subprocess.run([cg.CLI_PATH] + case["args"], cwd=GOLDEN, capture_output=True, timeout=300)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    m = parse_kma_args(case["args"])["metric"]
    if _pow_metric(m):
        np.testing.assert_allclose(_phylip_values(p.stdout), _phylip_values(golden_bytes(case)), rtol=_pow_rtol(m))
    else:
        assert p.stdout == golden_bytes(case)


@pytest.mark.parametrize("nsamp,L,metric,et", [(41, 20000, "cos", 8), (37, 9000, "c", 4), (70, 4000, "nbc", 8),
                                               (33, 6000, "chi2", 2), (35, 5000, "nchi2", 8), (40, 5000, "l2", 8)])
def test_kma_random_vs_oracle(dev, tmp_path, nsamp, L, metric, et):
    """More samples than one 32 x 32 tile, insertion rows, low-depth rows."""
    import random
    import ccphylo_amd as cg
    from gen_golden import kma_sample
    from oracle import pyoracle
    rng = random.Random(nsamp * L)
    ref = "".join(rng.choice("ACGT") for _ in range(L))
    files = []
    for k in range(nsamp):
        f = str(tmp_path / f"r{k}.mat.gz")
        kma_sample(f, [("x", ref)], seed=1000 + k, depth=20 if k % 5 else 12, ins=0.003 if k % 7 == 3 else 0.0)
        files.append(f)
    bs = 10.0 if et <= 2 else 1.0
    D0, N0, inc, n = pyoracle.kma_dist(files, "x", metric=metric, etype=et, byte_scale=bs, want_n=True)
    K = cg.native.load_kma(files, "x")
    D, N, fatal = dev.kma_ltd(K, metric=metric, etype=et, byte_scale=bs, want_n=True)
    assert fatal == -1 and K["n"] == n and (K["include"] == inc).all()
    assert np.array_equal(D, D0) and np.array_equal(N, N0)


def test_kma_fatal_pair(dev, tmp_path):
    """A later sample whose rows with ref != '-' fail the thresholds that its
    rows with '-' passed: the reference exits(1) at the first such pair."""
    import ccphylo_amd as cg
    from gen_golden import kma_sample
    ref = "ACGT" * 200
    files = []
    for k in range(4):
        f = str(tmp_path / f"f{k}.mat.gz")
        kma_sample(f, [("x", ref)], seed=k, depth=30, ins=0.0)
        files.append(f)
    # sample 1: shallow rows + deep insertion rows (counted by FileBuffLoadMat's nNucs only)
    with open(str(tmp_path / "f1.mat"), "w") as fh:
        fh.write("#x\n")
        for b in ref:
            fh.write(b + "\t1\t0\t0\t0\t0\t0\n-\t40\t0\t0\t0\t0\t0\n")
        fh.write("\n")
    files[1] = str(tmp_path / "f1.mat")
    K = cg.native.load_kma(files, "x")
    _, _, fatal = dev.kma_ltd(K)
    assert fatal >= 0
    p = subprocess.run([cg.CLI_PATH, "dist", "-i"] + files + ["-r", "x"], capture_output=True, timeout=120)
    assert p.returncode == 1 and p.stdout == b""
    assert b"did not exceed threshold" in p.stderr
