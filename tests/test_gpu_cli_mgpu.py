"""GPU: the multi-GPU CLI (host/mgpu.c).
- `ccphylo tree --gpus G` shards the matrix over G ranks (one host thread
  per rank): the Newick bytes equal the golden reference outputs and the
  one-GPU CLI's, for G = 1 over RCCL and G = 1, 2, 3, 8 over the host
  transport (several ranks per device on a one-GPU box).
- `ccphylo dist MSA --tree FILE` (dist and tree in HBM, no Phylip text)
  writes the Newick that `ccphylo dist MSA | ccphylo tree` writes.
ref: tree.c:146 main_tree (call sites tree.c:89-93), dist.c:473 main_dist."""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, golden_bytes, golden_cases

pytestmark = pytest.mark.gpu


def cli(args, **kw):
    import ccphylo_amd as cg
    p = subprocess.run([cg.CLI_PATH] + args, capture_output=True, timeout=600, **kw)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    return p.stdout


TREE_CASES = [c for c in golden_cases("tree")
              if not c["name"].startswith(("miss", "multi")) and "hnj" not in c["args"]
              and ("-m" not in c["args"] or c["args"][c["args"].index("-m") + 1] in ("nj", "dnj"))]


@pytest.mark.parametrize("case", TREE_CASES, ids=lambda c: c["name"])
@pytest.mark.parametrize("gpus,transport", [(1, "rccl"), (2, "host"), (3, "host")])
def test_cli_tree_gpus_golden(case, gpus, transport):
    args = case["args"] + ["--gpus", str(gpus), "--transport", transport]
    assert cli(args, cwd=GOLDEN) == golden_bytes(case)


def _write_phylip(path, D, n):
    from ccphylo_amd import native
    native.write_phylip(str(path), D, n, [f"t{k}" for k in range(n)])


@pytest.mark.parametrize("method", ["dnj", "nj"])
@pytest.mark.parametrize("fast", [False, True])
def test_cli_tree_gpus8_matches_one_gpu(tmp_path, method, fast):
    """8 ranks (the driver's node size) on the one GPU through the host
    transport: the same bytes as the single-GPU engine."""
    from tools.synth import euclid
    n = 1500
    path = tmp_path / "m.phy"
    _write_phylip(path, euclid(n, seed=4), n)
    extra = ["--fast_sums"] if fast else []
    one = cli(["tree", "-i", str(path), "-m", method] + extra)
    eight = cli(["tree", "-i", str(path), "-m", method, "--gpus", "8", "--transport", "host"] + extra)
    assert eight == one


def test_cli_tree_gpus_refuses_hnj(tmp_path):
    import ccphylo_amd as cg
    p = subprocess.run([cg.CLI_PATH, "tree", "-i", os.path.join(GOLDEN, "test.phy.gz"), "-m", "hnj", "--gpus", "2",
                        "--transport", "host"], capture_output=True, timeout=120)
    assert p.returncode == 1 and b"hnj" in p.stderr


DIST_MSAS = ["msa64.fsa", "msa300.fsa", "msa_crlf.fsa", "msa_odd.fsa", "msa_word.fsa"]


@pytest.mark.parametrize("msa", DIST_MSAS)
@pytest.mark.parametrize("gpus,transport,method", [(1, "rccl", "dnj"), (2, "host", "dnj"), (3, "host", "nj")])
def test_cli_dist_tree_fused(tmp_path, msa, gpus, transport, method):
    src = os.path.join(GOLDEN, msa)
    phy = tmp_path / "d.phy"
    with open(phy, "wb") as f:
        f.write(cli(["dist", "-i", src]))
    two_step = cli(["tree", "-i", str(phy), "-m", method])
    out = tmp_path / "t.nwk"
    cli(["dist", "-i", src, "--tree", str(out), "--tree_method", method, "--gpus", str(gpus), "--transport",
         transport])
    assert out.read_bytes() == two_step


def test_cli_dist_tree_fused_large(tmp_path):
    """A clade-structured MSA with many equal distances (tie-heavy joins)."""
    rng = np.random.default_rng(8)
    n, L = 700, 3000
    lut = np.frombuffer(b"ACGT", np.uint8)
    base = rng.integers(0, 4, L)
    clades = [np.where(rng.random(L) < 0.02, rng.integers(0, 4, L), base) for _ in range(12)]
    src = tmp_path / "c.fsa"
    with open(src, "wb") as f:
        for k in range(n):
            s = clades[k % 12].copy()
            flip = rng.random(L) < 0.003
            s[flip] = rng.integers(0, 4, int(flip.sum()))
            f.write(b">s%d\n" % k + lut[s].tobytes() + b"\n")
    phy = tmp_path / "d.phy"
    with open(phy, "wb") as f:
        f.write(cli(["dist", "-i", str(src)]))
    two_step = cli(["tree", "-i", str(phy)])
    out = tmp_path / "t.nwk"
    cli(["dist", "-i", str(src), "--tree", str(out), "--gpus", "3", "--transport", "host"])
    assert out.read_bytes() == two_step


@pytest.mark.parametrize("msa,extra", [("msa64.fsa", ["-f", "3"]), ("msa_odd.fsa", ["-f", "3", "-P", "2"]),
                                       ("msa_word.fsa", ["-f", "3"]), ("msa_crlf.fsa", ["-f", "3"])])
@pytest.mark.parametrize("gpus,transport", [(1, "rccl"), (3, "host")])
def test_cli_dist_tree_fused_pair(tmp_path, msa, extra, gpus, transport):
    """Pair-mode distances (-f 2: cmpairFsaThrd, fsacmp.c:587; -P maskProxi)
    written into the rank bands: the same Newick as `dist -f 3 | tree`."""
    src = os.path.join(GOLDEN, msa)
    phy = tmp_path / "d.phy"
    with open(phy, "wb") as f:
        f.write(cli(["dist", "-i", src] + extra))
    two_step = cli(["tree", "-i", str(phy)])
    out = tmp_path / "t.nwk"
    cli(["dist", "-i", src, "--tree", str(out), "--gpus", str(gpus), "--transport", transport] + extra)
    assert out.read_bytes() == two_step


def test_cli_dist_tree_fused_pair_missing(tmp_path):
    """msa64 with -f 3 -P 10 leaves pairs below the minimum length (-1
    entries): the sharded tree refuses them (CCG_EUNSUP) and says how to run
    them on one GPU, rather than building a different tree."""
    import ccphylo_amd as cg
    p = subprocess.run([cg.CLI_PATH, "dist", "-i", os.path.join(GOLDEN, "msa64.fsa"), "-f", "3", "-P", "10", "--tree",
                        str(tmp_path / "t.nwk")], capture_output=True, timeout=120)
    assert p.returncode == 1 and b"missing entries" in p.stderr
