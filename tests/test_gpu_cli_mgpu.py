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
              if not c["name"].startswith(("miss", "multi"))
              and ("-m" not in c["args"] or c["args"][c["args"].index("-m") + 1] in ("nj", "dnj", "hnj"))]


@pytest.mark.parametrize("case", TREE_CASES, ids=lambda c: c["name"])
@pytest.mark.parametrize("gpus,transport", [(1, "rccl"), (2, "host"), (3, "host")])
def test_cli_tree_gpus_golden(case, gpus, transport):
    args = case["args"] + ["--gpus", str(gpus), "--transport", transport]
    assert cli(args, cwd=GOLDEN) == golden_bytes(case)


def _write_phylip(path, D, n):
    from ccphylo_amd import native
    native.write_phylip(str(path), D, n, [f"t{k}" for k in range(n)])


@pytest.mark.parametrize("method", ["dnj", "nj", "hnj"])
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


def test_cli_dist_tree_fused_hnj(tmp_path):
    """`dist --tree --tree_method hnj` over 3 ranks: the Newick of `dist | tree -m hnj`."""
    src = os.path.join(GOLDEN, "msa300.fsa")
    phy = tmp_path / "d.phy"
    with open(phy, "wb") as f:
        f.write(cli(["dist", "-i", src]))
    two_step = cli(["tree", "-i", str(phy), "-m", "hnj"])
    out = tmp_path / "t.nwk"
    cli(["dist", "-i", src, "--tree", str(out), "--tree_method", "hnj", "--gpus", "3", "--transport", "host"])
    assert out.read_bytes() == two_step


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
    entries).  With one GPU the fused path runs the single-GPU engine, whose
    updateD keeps the missing-entry quirks (nj.c:1021-1030): the Newick of
    `dist -f 3 -P 10 | tree`.  The sharded tree (--gpus > 1) still refuses
    such matrices (CCG_EUNSUP) and says to use one GPU."""
    import ccphylo_amd as cg
    src = os.path.join(GOLDEN, "msa64.fsa")
    extra = ["-f", "3", "-P", "10"]
    phy = tmp_path / "d.phy"
    with open(phy, "wb") as f:
        f.write(cli(["dist", "-i", src] + extra))
    assert b"-1" in phy.read_bytes()
    for method in ("dnj", "nj", "hnj"):
        two_step = cli(["tree", "-i", str(phy), "-m", method])
        out = tmp_path / f"t_{method}.nwk"
        cli(["dist", "-i", src, "--tree", str(out), "--tree_method", method, "--gpus", "1"] + extra)
        assert out.read_bytes() == two_step, method
    p = subprocess.run([cg.CLI_PATH, "dist", "-i", src, "--tree", str(tmp_path / "t.nwk"), "--gpus", "2",
                        "--transport", "host"] + extra, capture_output=True, timeout=120)
    assert p.returncode == 1 and b"missing entries" in p.stderr


@pytest.mark.parametrize("msa,extra", [("msa64.fsa", ["-W", "1000"]), ("msa300.fsa", ["-W", "7", "-x", "4"]),
                                       ("msa64.fsa", ["-W", "1000", "-p"]), ("msa_odd.fsa", ["-f", "3", "-W", "3"])])
@pytest.mark.parametrize("gpus", [1, 3])
def test_cli_dist_tree_fused_norm(tmp_path, msa, extra, gpus):
    """-W normalised distances are not integral: `dist -W | tree` rounds them
    to -x digits in the Phylip text (printphy phy.c:117, strtod phy.c:469);
    the fused path rounds them in HBM the same way (ccg_round_decimal_dev)."""
    src = os.path.join(GOLDEN, msa)
    phy = tmp_path / "d.phy"
    with open(phy, "wb") as f:
        f.write(cli(["dist", "-i", src] + extra))
    tx = ["-x", extra[extra.index("-x") + 1]] if "-x" in extra else []
    tp = ["-p"] if "-p" in extra else []
    two_step = cli(["tree", "-i", str(phy)] + tx + tp)
    out = tmp_path / "t.nwk"
    cli(["dist", "-i", src, "--tree", str(out), "--gpus", str(gpus), "--transport", "host"] + extra)
    assert out.read_bytes() == two_step


def test_round_decimal_dev():
    """ccg_round_decimal_dev against Python's own %.*f / float() round trip
    (correctly rounded both ways, as glibc's printf / strtod are)."""
    import torch
    import ccphylo_amd as cg
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.random(20000) * 10.0 ** rng.integers(-6, 6, 20000), np.arange(50.0),
                        np.array([0.5e-9, 1.5e-9, 2.5e-9, 0.1, 0.7, 123456.7890123455, 1e-12, 4.4e5]),
                        # |x 10^p| in [2^52, 2^53) at p = 9: the integral-hi branch
                        4.6e6 + rng.random(4000) * 4.3e6, -(4.6e6 + rng.random(500) * 4.3e6)])
    dev = cg.Device(0)
    try:
        for p in (9, 4, 0, 12):
            for dt, et in ((np.float64, 8), (np.float32, 4)):
                h = x.astype(dt)
                h = h[(h == np.trunc(h)) | (np.abs(h.astype(np.float64)) * 10.0 ** p < 2.0 ** 53 * 0.999)]
                t = torch.from_numpy(h.copy()).cuda()
                rc = dev.lib.ccg_round_decimal_dev(dev.h, C_void(t.data_ptr()), C_i64(len(h)), et, p)
                assert rc == 0, (p, et)
                torch.cuda.synchronize()
                want = np.array([v if v == int(v) else dt(float("%.*f" % (p, v))) for v in h.astype(np.float64)],
                                dtype=dt)
                assert (t.cpu().numpy() == want).all(), (p, et)
        # more significant digits than a double holds: refused, not rounded wrongly
        t = torch.tensor([123456.5, 1.25], dtype=torch.float64, device="cuda")
        assert dev.lib.ccg_round_decimal_dev(dev.h, C_void(t.data_ptr()), C_i64(2), 8, 15) == -5
    finally:
        dev.close()


def C_void(p):
    import ctypes
    return ctypes.c_void_p(p)


def C_i64(v):
    import ctypes
    return ctypes.c_int64(v)


@pytest.mark.parametrize("where", ["setup:1", "run:2"])
def test_cli_mgpu_rank_failure_exits(tmp_path, where):
    """One rank failing -- in its setup, or leaving instead of running its
    tree while its peers sit in their collectives -- makes the CLI exit with
    an error instead of hanging (host transport)."""
    import ccphylo_amd as cg
    env = dict(os.environ, CCQ_MGPU_FAIL=where)
    p = subprocess.run([cg.CLI_PATH, "dist", "-i", os.path.join(GOLDEN, "msa300.fsa"), "--tree",
                        str(tmp_path / "t.nwk"), "--gpus", "3", "--transport", "host"], capture_output=True,
                       timeout=120, env=env)
    assert p.returncode == 1, p.stderr.decode()[-1000:]
    assert b"injected" in p.stderr
    p = subprocess.run([cg.CLI_PATH, "tree", "-i", os.path.join(GOLDEN, "test.phy.gz"), "--gpus", "3",
                        "--transport", "host"], capture_output=True, timeout=120, env=env)
    assert p.returncode == 1 and b"injected" in p.stderr


@pytest.mark.parametrize("method", ["dnj", "nj"])
def test_cli_dist_tree_world8_20k(tmp_path, method):
    """configs[4] rehearsal on one GPU (formerly
    tools/rehearse_world8.py): a clade-structured 20k x 3 kbp MSA through
    `dist --tree --gpus 8 --transport host` (8 rank threads, dist straight into
    the band shards, the sharded tree) against `--gpus 1` (the single-GPU
    engine on the full LT): the same Newick bytes."""
    from tools.rehearse_world8 import write_fasta
    fa = tmp_path / "m.fsa"
    write_fasta(str(fa), 20000, 3000)
    outs = {}
    for g in (1, 8):
        out = tmp_path / f"{method}{g}.nwk"
        cli(["dist", "-i", str(fa), "--tree", str(out), "--tree_method", method, "--gpus", str(g), "--transport",
             "host"])
        outs[g] = out.read_bytes()
    assert outs[8] == outs[1] and len(outs[1]) > 20000


def _devices():
    import ccphylo_amd as cg
    return cg.Device.count()


@pytest.mark.parametrize("method", ["dnj", "nj"])
def test_cli_tree_rccl_multi_gpu(tmp_path, method):
    """RCCL with one rank per GPU (the configuration of the driver's 8-GPU
    node): `tree --gpus G --transport rccl` for G = 2 and every visible GPU,
    against the one-GPU CLI.  Skipped on a one-GPU box, where several ranks
    cannot share a device over RCCL (the host transport covers those worlds)."""
    ndev = _devices()
    if ndev < 2:
        pytest.skip(f"{ndev} GPU(s) visible: RCCL with world > 1 needs one GPU per rank")
    from tools.synth import euclid
    n = 3000
    path = tmp_path / "m.phy"
    _write_phylip(path, euclid(n, seed=6), n)
    one = cli(["tree", "-i", str(path), "-m", method])
    for g in sorted({2, ndev}):
        assert cli(["tree", "-i", str(path), "-m", method, "--gpus", str(g), "--transport", "rccl"]) == one, g
