"""CPU: the parallel MSA loader (host/fasta_par.c, ccq_load_msa_par) returns
the serial loader's result (ccq_load_msa, itself pinned by the dist goldens)
byte for byte: headers, packed rows, include masks, length, minLength and the
Included / Excluded lines, for every golden dist case and for generated
FASTA with the reference parser's edge cases (seqparse.c:28: '>' inside
headers and residues, CRLF, empty sequences, a last header without residues
or without a newline, IUPAC / lowercase / gap codes, excluded taxa), at
several thread counts and window sizes small enough to cut records."""
import os

import numpy as np
import pytest

from conftest import golden_cases, parse_dist_args


def both(path, flag, min_length, min_cov, proxi, threads, tmp_path, window=None):
    import ccphylo_amd as cg
    ls, lp = str(tmp_path / "serial.log"), str(tmp_path / "par.log")
    s = cg.load_msa(path, flag, min_length, min_cov, proxi, log_path=ls)
    old = os.environ.get("CCQ_FASTA_WINDOW")
    if window:
        os.environ["CCQ_FASTA_WINDOW"] = str(window)
    try:
        p = cg.load_msa(path, flag, min_length, min_cov, proxi, threads=threads, log_path=lp)
    finally:
        if window:
            if old is None:
                del os.environ["CCQ_FASTA_WINDOW"]
            else:
                os.environ["CCQ_FASTA_WINDOW"] = old
    return s, p, open(ls, "rb").read(), open(lp, "rb").read()


def assert_same(s, p, slog, plog):
    assert s[0] == p[0]                      # headers
    assert s[1].shape == p[1].shape and (s[1] == p[1]).all()
    assert np.asarray(s[2]).shape == np.asarray(p[2]).shape and (np.asarray(s[2]) == np.asarray(p[2])).all()
    assert s[3:] == p[3:]                    # len, minLength
    assert slog == plog


@pytest.mark.parametrize("case", [c for c in golden_cases("dist") if parse_dist_args(c["args"])["inp"].endswith(".fsa")],
                         ids=lambda c: c["name"])
@pytest.mark.parametrize("threads", [1, 3, 16])
def test_par_loader_golden(case, threads, tmp_path):
    o = parse_dist_args(case["args"])
    assert_same(*both(o["inp"], o["flag"], o["minLength"], o["minCov"], o["proxi"], threads, tmp_path))


def synth_fasta(path, rng, n, L, crlf=False, odd=True):
    """Random MSA text with the parser's corner cases."""
    alphabet = np.frombuffer(b"ACGTACGTACGTACGTNn-RYacgtuU", dtype=np.uint8)
    lines = []
    for k in range(n):
        hdr = f">t{k}"
        if odd and k % 7 == 3:
            hdr += " desc > with > marks"    # '>' inside a header is part of it
        if odd and k % 11 == 5:
            hdr += "  \t "                    # trailing white space is trimmed
        seq = alphabet[rng.integers(0, len(alphabet), L)].tobytes()
        if odd and k % 13 == 7:               # mostly N: excluded by minLength
            seq = b"N" * (L - 3) + b"ACG"
        width = int(rng.integers(7, 80))
        body = [seq[i:i + width] for i in range(0, L, width)]
        if odd and k % 17 == 9:
            body.insert(1, b"**12 ")          # bytes the table drops (codes >= 8)
        nl = b"\r\n" if crlf else b"\n"
        lines.append(hdr.encode() + nl + nl.join(body) + nl)
    with open(path, "wb") as f:
        f.write(b"".join(lines))


@pytest.mark.parametrize("flag", [1, 3, 9, 33, 11])
@pytest.mark.parametrize("proxi", [0, 3])
@pytest.mark.parametrize("window", [None, 257, 4096])
def test_par_loader_synthetic(flag, proxi, window, tmp_path):
    rng = np.random.default_rng(flag * 100 + proxi)
    path = str(tmp_path / "m.fsa")
    synth_fasta(path, rng, 90, 333, crlf=flag == 9)
    for threads in (1, 4, 16):
        assert_same(*both(path, flag, 10, 0.5, proxi, threads, tmp_path, window=window))


@pytest.mark.parametrize("tail", [b">last\n", b">last", b">last\n" + b"ACGT" * 16, b"", b">x\n" + b"GT" * 32 + b"\n>y\n"])
def test_par_loader_input_end(tail, tmp_path):
    """A final header without residues or newline ends the input without a
    record (FileBuffgetFsa returns 0); residues that run to the end of the
    input without a newline are a record."""
    rng = np.random.default_rng(5)
    path = str(tmp_path / "e.fsa")
    synth_fasta(path, rng, 12, 64, odd=False)
    with open(path, "ab") as f:
        f.write(tail)
    for window in (None, 64):
        for threads in (1, 5):
            assert_same(*both(path, 1, 1, 0.0, 0, threads, tmp_path, window=window))


def test_par_loader_first_excluded(tmp_path):
    """Leading sequences below minLength: each re-sets the length and ratchets
    minLength (cdist.c:287-321) until one is usable."""
    path = str(tmp_path / "x.fsa")
    with open(path, "wb") as f:
        f.write(b">a\n" + b"N" * 50 + b"\n>b\n" + b"N" * 90 + b"AC\n>c\n" + b"ACGT" * 25 + b"\n")
        rng = np.random.default_rng(9)
        for k in range(20):
            f.write(b">r%d\n" % k + np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, 100)].tobytes() + b"\n")
    for threads in (1, 7):
        assert_same(*both(path, 1, 5, 0.6, 0, threads, tmp_path, window=300))


def test_par_loader_gz(tmp_path):
    import gzip
    rng = np.random.default_rng(3)
    raw = str(tmp_path / "g.fsa")
    synth_fasta(raw, rng, 40, 500)
    gz = raw + ".gz"
    with open(raw, "rb") as a, gzip.open(gz, "wb") as b:
        b.write(a.read())
    assert_same(*both(gz, 1, 10, 0.5, 2, 6, tmp_path, window=1000))


MISMATCH = """
import sys
sys.path.insert(0, {root!r})
import ccphylo_amd as cg
cg.load_msa({path!r}, 1, 1, 0.0, 0, threads={threads}, log_path={log!r})
"""


@pytest.mark.parametrize("window", [None, 100])
def test_par_loader_length_mismatch(window, tmp_path):
    """A sequence of another length: the reference prints the lines of the
    records before it, then 'Sequences does not match: <header>' and exits 1
    (cdist.c:264-267); both loaders do the same (run in child processes)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = str(tmp_path / "mm.fsa")
    with open(path, "wb") as f:
        for k in range(9):
            f.write(b">s%d\n" % k + b"ACGT" * (10 if k != 6 else 11) + b"\n")
    outs = []
    for threads in (0, 4):
        log = str(tmp_path / f"mm{threads}.log")
        env = dict(os.environ)
        if window:
            env["CCQ_FASTA_WINDOW"] = str(window)
        p = subprocess.run([sys.executable, "-c", MISMATCH.format(root=root, path=path, threads=threads, log=log)],
                           capture_output=True, env=env, timeout=120)
        outs.append((p.returncode, p.stderr.decode().strip().splitlines()[-1], open(log, "rb").read()))
    assert outs[0] == outs[1]
    assert outs[0][0] == 1 and outs[0][1] == "Sequences does not match: >s6"
