"""CPU: the Newick replay at scale.

`ccq_replay_newick` replays only (capacity, length) per name slot, then writes
the string once; `ccq_replay_newick_strings` edits the strings join by join as
nwck.c:35 formNode does.  Both must give the same bytes and leave every name
buffer with the same capacity (the next matrix in the file reuses them,
tree.c:61-66, and capacities decide child order, nwck.c:45)."""
import ctypes as C
import time

import numpy as np
import pytest

import ccphylo_amd.native as nat


def _lib():
    import ccphylo_amd as cg
    lib = cg.host_lib()
    lib.ccq_replay_newick_strings.argtypes = lib.ccq_replay_newick.argtypes
    return lib


def _table(lib, names, sizes):
    T = lib.ccq_names_new(len(names), 64)
    tb = nat._Names.from_address(T)
    for k, (nm, sz) in enumerate(zip(names, sizes)):
        s = tb.names[k].contents
        addr = C.c_void_p.from_address(C.addressof(s) + nat._Str.seq.offset).value
        C.memmove(addr, nm + b"\0", len(nm) + 1)
        s.len = len(nm)
        s.size = sz
    return T, tb


def _state(tb, n):
    return [(tb.names[k].contents.size) for k in range(n)]


def _joins(rng, n, shape, njoins, neg):
    import ccphylo_amd as cg
    J = np.zeros(njoins, dtype=cg.JOIN_DTYPE)
    m = n
    for k in range(njoins):
        if shape == "caterpillar":
            i, j = m - 1, 0
        elif shape == "ladder":
            i, j = m - 1, m - 2
        else:
            i = int(rng.integers(1, m))
            j = int(rng.integers(0, i))
        J[k]["i"], J[k]["j"] = i, j
        J[k]["Li"], J[k]["Lj"] = rng.random() * 10, rng.random() * 1e-3
        if neg and rng.random() < 0.3:
            J[k]["Li"] = -1.0
            if rng.random() < 0.5:
                J[k]["Lj"] = -2.0
        m -= 1
    return J


@pytest.mark.parametrize("n,shape,flags,prec,stop,neg", [
    (3, "random", 0, 9, False, False), (4, "random", 1, 9, False, True), (50, "random", 0, 4, False, True),
    (777, "random", 0, 9, False, False), (500, "caterpillar", 1, 9, False, False), (300, "ladder", 0, 9, True, False),
    (400, "random", 1, 6, True, True), (64, "caterpillar", 0, 0, True, True)])
def test_replay_matches_string_editing(n, shape, flags, prec, stop, neg):
    lib = _lib()
    rng = np.random.default_rng(n + flags + prec)
    names = [("t%d_" % k).encode() + b"x" * int(rng.integers(0, 30)) for k in range(n)]
    sizes = [int(rng.choice([4, 8, 16, 32, 64])) for _ in range(n)]
    sizes = [max(s, len(nm) + 1) for s, nm in zip(sizes, names)]
    tables = [_table(lib, names, sizes) for _ in range(2)]
    try:
        # two trees in a row on the same tables: the second sees the first's capacities
        for rep in range(2):
            njoins = n - 2 if not stop else max(0, n - 2 - int(rng.integers(1, 4)))
            J = _joins(rng, n, shape, njoins, neg)
            fn = n - njoins
            fd = float(rng.random()) if fn == 2 else -1.0
            outs = []
            for fnc, (T, tb) in zip((lib.ccq_replay_newick, lib.ccq_replay_newick_strings), tables):
                fnc(T, n, J.ctypes.data, len(J), fn, fd, flags, prec)
                outs.append((tb.names[0].contents.seq, _state(tb, n)))
            assert outs[0][0] == outs[1][0]
            assert outs[0][1] == outs[1][1]
            if rep == 0:
                for T, tb in tables:    # the next matrix's names, read into the same buffers
                    for k in range(n):
                        s = tb.names[k].contents
                        nm = names[k][:max(0, s.size - 1)]
                        addr = C.c_void_p.from_address(C.addressof(s) + nat._Str.seq.offset).value
                        C.memmove(addr, nm + b"\0", len(nm) + 1)
                        s.len = len(nm)
    finally:
        for T, _ in tables:
            lib.ccq_names_free(T)


def test_replay_caterpillar_at_scale():
    """200k-taxon caterpillar: the string-editing replay shifts the whole
    growing string per join (O(N^2) bytes); the symbolic replay is linear."""
    lib = _lib()
    rng = np.random.default_rng(1)
    n = 200_000
    names = [b"taxon%d" % k for k in range(n)]
    T, tb = _table(lib, names, [16] * n)
    try:
        J = _joins(rng, n, "caterpillar", n - 2, False)
        t0 = time.perf_counter()
        lib.ccq_replay_newick(T, n, J.ctypes.data, len(J), 2, 0.5, 0, 9)
        dt = time.perf_counter() - t0
        s = tb.names[0].contents.seq
        assert s.count(b"(") == s.count(b")") == n - 2
        assert s.count(b",") == n - 1
        assert dt < 5.0, dt
    finally:
        lib.ccq_names_free(T)
