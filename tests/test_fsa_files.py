"""CPU: multi-file FASTA input with -r (cdist.c:36 ltdFsaMatrix_get) restated
over the oracle's primitives (code table, packing, masks, fsacmp), including
cmpFsaThrd's pair order (fsacmpthrd.c:192-218: the skip test is `&&`, so a
pair with one excluded file still fills the next cell), against the reference's
golden vectors."""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden_bytes, golden_cases, print_phylip


def parse_args(args):
    o = dict(files=[], tmpl=None, flag=1, norm=0, minLength=1, minCov=0.5, et=8, bs=1.0, prec=9, nout=False, proxi=0)
    k = 1
    while k < len(args):
        a, nxt = args[k], (args[k + 1] if k + 1 < len(args) else None)
        if a == "-i":
            while k + 1 < len(args) and not args[k + 1].startswith("-"):
                o["files"].append(os.path.join(GOLDEN, args[k + 1]))
                k += 1
        elif a == "-r": o["tmpl"] = nxt; k += 1
        elif a == "-f": o["flag"] = int(nxt); k += 1
        elif a == "-W": o["norm"] = int(nxt); k += 1
        elif a == "-n": o["nout"] = True; k += 1
        elif a == "-P": o["proxi"] = int(nxt); k += 1
        elif a == "-s":
            o["et"] = 2
            if nxt and not nxt.startswith("-"):
                o["bs"] = float(nxt); k += 1
        k += 1
    return o


def cell_pairs(include, cells):
    """cmpFsaThrd's (i, j) for LT cells 0, 1, ... (fsacmpthrd.c:147-218)."""
    n = len(include)
    first = next(i for i in range(n) if include[i])
    si, sj, out = first + 1, 0, []
    for _ in range(cells):
        i, j = si, sj
        while not include[i] and not include[j]:
            while i < n and not include[i]:
                i += 1
            while j < i and not include[j]:
                j += 1
            if i == j:
                i, j = i + 1, 0
        out.append((i, j))
        si, sj = i, j + 1
        if si == sj:
            si, sj = si + 1, 0
    return out


def load(o):
    from oracle import pyoracle
    L = pyoracle.lib()
    table = (C.c_uint8 * 256)()
    L.orc_code_table(o["flag"], table)
    tab = np.frombuffer(bytes(table), np.uint8)
    variant = 32 if o["flag"] & 32 else 8 if o["flag"] & 8 else 0
    pair = bool(o["flag"] & 2)
    seqs, incs, include = {}, {}, []
    gmask, ref, length, minL = None, None, 0, o["minLength"]
    for f in o["files"]:
        entry, name, buf = None, None, []
        for line in open(f, "rb").read().split(b"\n"):
            if line.startswith(b">"):
                if name == o["tmpl"]:
                    break
                name, buf = line[1:].rstrip().decode(), []
            else:
                buf.append(line)
        if name == o["tmpl"]:
            codes = tab[np.frombuffer(b"".join(buf), np.uint8)]
            entry = np.ascontiguousarray(codes[codes < 8])
        if entry is None:
            include.append(0)
            continue
        if ref is None:
            length = len(entry)
            minL = max(minL, int(o["minCov"] * length))
        W = length // 32 + 1
        packed = np.zeros(W, np.uint64)
        nN = L.orc_pack(entry.ctypes.data, length, packed.ctypes.data)
        seqs[len(include)] = packed
        if ref is None or pair:
            m = np.zeros(W, np.uint32)
            L.orc_init_inc(m.ctypes.data, length)
            L.orc_inc_update(m.ctypes.data, entry.ctypes.data, entry.ctypes.data, length, 0, variant)
            inc = L.orc_npos(m.ctypes.data, length)
        else:
            inc = length - nN
        if inc < minL:
            include.append(0)
            continue
        include.append(1)
        if pair:
            incs[len(include) - 1] = m
        elif ref is None:
            gmask = m
        else:
            L.orc_inc_update(gmask.ctypes.data, entry.ctypes.data, ref.ctypes.data, length, 0, variant)
        if ref is None:
            ref = entry
    return seqs, incs, gmask, include, length, minL, pair


@pytest.mark.parametrize("case", golden_cases("fsafiles"), ids=lambda c: c["name"])
def test_fsa_files_oracle_matches_reference(case):
    from oracle import pyoracle
    o = parse_args(case["args"])
    seqs, incs, gmask, include, length, minL, pair = load(o)
    Dn = sum(include)
    W = length // 32 + 1
    idx = [k for k in range(len(include)) if include[k]]
    if pair:
        S = np.stack([seqs[k] for k in idx])
        I = np.stack([incs[k] for k in idx])
        D, N, _ = pyoracle.snp_ltd(S, I, Dn, length, pair=True, norm=o["norm"], min_length=minL, etype=o["et"],
                                   byte_scale=o["bs"], proxi=o["proxi"], want_n=o["nout"])
    else:
        L = pyoracle.lib()
        inc = L.orc_npos(gmask.ctypes.data, length)
        nf = o["norm"] / inc if o["norm"] else 1.0
        zero = np.zeros(W, np.uint64)
        vals = []
        for i, j in cell_pairs(include, Dn * (Dn - 1) // 2):
            a, b = seqs.get(i, zero), seqs.get(j, zero)
            vals.append(nf * L.orc_fsacmp(a.ctypes.data, b.ctypes.data, gmask.ctypes.data, length))
        D, N = np.array(vals, dtype=np.float64), None
        assert o["et"] == 8
    names = o["files"]
    out = print_phylip(D, Dn, names, o["flag"], o["prec"], o["et"], o["bs"], include=include, comment=o["tmpl"])
    if N is not None:
        out += print_phylip(N, Dn, names, o["flag"], o["prec"], o["et"], o["bs"], include=include,
                            comment=o["tmpl"])
    assert out == golden_bytes(case)
