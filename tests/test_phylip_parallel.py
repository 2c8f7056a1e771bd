"""CPU: the parallel Phylip reader (ccq_load_phy for n >= 512)
loads exactly what the serial reader (CCQ_SERIAL_PHY=1, the restatement of
phy.c:251 loadPhy) loads: names (with their buffer capacities) and every cell
bit for bit, over the formats a Phylip matrix can hold."""
import gzip
import os
import random

import numpy as np
import pytest


def _write(path, n, fmt, seed, full=False, empties=False, sep="\t", gz=False, tail=True, trailing_junk=False):
    rng = random.Random(seed)
    op = gzip.open if gz else open
    with op(path, "wt") as f:
        f.write("#comment line\n%10d\n" % n)
        for i in range(n):
            cells = []
            for j in range(n if full else i):
                x = rng.random() * 10 ** rng.randint(-3, 4)
                if fmt == "f9":
                    s = "%.9f" % x
                elif fmt == "int":
                    s = str(int(x))
                elif fmt == "mixed":
                    s = rng.choice(["%.9f" % x, "%g" % x, "%.17g" % x, "%e" % x, str(int(x)), "-1", "+%.3f" % x,
                                    "%.25f" % x, "0.%s" % ("3" * 25)])
                cells.append(s)
                if empties and rng.random() < 0.05:
                    cells.append("")
            row = [f"taxon_{i}" + ("_" * (i % 37))] + cells
            if trailing_junk:
                row.append("junk")
            line = sep.join(row)
            if i < n - 1 or tail:
                line += "\n"
            f.write(line)


def _load(path, et=8, bs=1.0, serial=False):
    import ccphylo_amd as cg
    if serial:
        os.environ["CCQ_SERIAL_PHY"] = "1"
    try:
        return cg.native.load_phylip(path, etype=et, byte_scale=bs)
    finally:
        os.environ.pop("CCQ_SERIAL_PHY", None)


@pytest.mark.parametrize("fmt,kw", [("f9", {}), ("int", {"gz": True}), ("mixed", {}), ("f9", {"full": True}),
                                    ("mixed", {"empties": True}), ("f9", {"tail": False}),
                                    ("int", {"trailing_junk": True})])
def test_parallel_reader_matches_serial(tmp_path, fmt, kw):
    path = str(tmp_path / ("m.phy.gz" if kw.get("gz") else "m.phy"))
    _write(path, 700, fmt, 7, **kw)
    for et, bs in ((8, 1.0), (4, 1.0), (2, 100.0)):
        a = _load(path, et, bs)
        b = _load(path, et, bs, serial=True)
        # a last row cut by EOF inside its last distance is an error for both
        assert len(a) == len(b) == (1 if kw.get("tail", True) else 0)
        if not a:
            continue
        assert a[0][0] == b[0][0]
        assert a[0][1].dtype == b[0][1].dtype and np.array_equal(a[0][1].view(np.uint8), b[0][1].view(np.uint8))


def test_parallel_reader_two_matrices(tmp_path):
    """Bytes after the first matrix go back to the reader for the second."""
    p1, p2 = str(tmp_path / "a.phy"), str(tmp_path / "b.phy")
    _write(p1, 600, "f9", 1)
    _write(p2, 530, "mixed", 2)
    both = str(tmp_path / "ab.phy")
    with open(both, "w") as f:
        f.write(open(p1).read() + open(p2).read())
    a = _load(both)
    b = _load(both, serial=True)
    assert [x[0] for x in a] == [x[0] for x in b]
    assert all(np.array_equal(x[1], y[1]) for x, y in zip(a, b))
    assert len(a) == 2


@pytest.mark.parametrize("flag,et", [(1, 8), (0, 8), (5, 4), (1, 2)])
def test_parallel_writer_matches_one_thread(tmp_path, flag, et):
    """ccq_print_phy splits rows over threads; the bytes equal a 1-thread run
    (the reference's printphy loop), incl. quoted names, dirs and include."""
    from conftest import print_phylip
    rng = np.random.default_rng(3)
    n_all = 900
    include = (rng.random(n_all) > 0.1).astype(np.uint8)
    n = int(include.sum())
    m = n * (n - 1) // 2
    D = rng.random(m) * 100
    D[rng.random(m) < 0.3] = np.floor(D[rng.random(m) < 0.3 * 1.0][: int((rng.random(m) < 0.3).sum())].mean())
    D[::7] = np.round(D[::7])
    D[::11] = -1.0
    bs = 10.0 if et == 2 else 1.0
    Dt = {8: D, 4: D.astype(np.float32), 2: np.clip(D * bs + 0.5, 0, 65535).astype(np.uint16)}[et]
    names = [(f'"dir/q{k}"' if k % 5 == 0 else f"path/to/taxon_{k}_long_name") for k in range(n_all)]
    outs = []
    for threads in ("1", "8"):
        os.environ["OMP_NUM_THREADS"] = threads
        try:
            outs.append(print_phylip(Dt, n, list(names), flag, 9, et, bs, include=include, comment="tmpl"))
        finally:
            os.environ.pop("OMP_NUM_THREADS", None)
    assert outs[0] == outs[1]
