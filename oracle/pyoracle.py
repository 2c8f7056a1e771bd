"""ctypes view of oracle/_build/liboracle.so (the CPU restatement, ccoracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker -- never by ccphylo_amd/.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")
REF_BIN = os.path.join(HERE, "_ref", "ccphylo")
ETYPES = {8: np.float64, 4: np.float32, 2: np.uint16, 1: np.uint8}
JOIN_DTYPE = np.dtype([("i", np.int32), ("j", np.int32), ("Li", np.float64), ("Lj", np.float64)])

_lib = None


def build():
    """Builds liboracle.so (and, where /root/reference exists, the reference binary)."""
    targets = ["oracle"] + (["all"] if os.path.isdir("/root/reference") else [])
    subprocess.run(["make", "-s", "-C", HERE] + targets, check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        L.orc_tree.argtypes = [C.c_int, C.c_int, C.c_double, C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                               C.POINTER(C.c_int), C.POINTER(C.c_double), C.c_void_p]
        L.orc_tree_ex.argtypes = [C.c_int, C.c_int, C.c_double, C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                                  C.POINTER(C.c_int), C.POINTER(C.c_double), C.c_void_p, C.c_int, C.c_int]
        L.orc_snp_ltd.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_uint, C.c_uint, C.c_double,
                                  C.c_uint, C.c_int, C.c_double, C.c_void_p, C.c_void_p]
        L.orc_snp_ltd_ex.argtypes = L.orc_snp_ltd.argtypes + [C.c_int]
        L.orc_dnj_init.argtypes = [C.c_int, C.c_int, C.c_double, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                   C.c_void_p, C.c_int]
        L.orc_dnj_resume.argtypes = [C.c_int, C.c_int, C.c_double, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.POINTER(C.c_int),
                                     C.POINTER(C.c_double), C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_int)]
        L.orc_pack.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.orc_init_inc.argtypes = [C.c_void_p, C.c_int]
        L.orc_inc_update.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_uint, C.c_int]
        L.orc_npos.argtypes = [C.c_void_p, C.c_int]
        L.orc_fsacmp.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.orc_fsacmp.restype = C.c_uint32
        L.orc_fsacmpair.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.orc_fsacmpair.restype = C.c_uint64
        L.orc_code_table.argtypes = [C.c_uint, C.c_void_p]
        L.orc_init_sums.argtypes = [C.c_int, C.c_int, C.c_double, C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_kma_dist.argtypes = [C.c_int, C.c_void_p, C.c_char_p, C.c_int, C.c_uint, C.c_uint, C.c_uint, C.c_uint,
                                   C.c_double, C.c_int, C.c_double, C.c_void_p, C.c_void_p, C.c_void_p,
                                   C.POINTER(C.c_int)]
        _lib = L
    return _lib


def tree(D, n, etype=8, byte_scale=1.0, method=1, flags=0, stats=False, max_joins=0, threads=1, copy=True):
    """Serial NJ (method 0) / DNJ (method 1) / HNJ (method 2) exactly as the reference.
    max_joins > 0 stops after that many joins (a prefix of the same run);
    threads > 1 runs the O(n^2) initSummaD / initHNJ passes and DNJ's
    minQpair rescans on pthreads (same order / decisions, bit-identical).  copy=False destroys D in place (it must
    then be a writable contiguous array of the element type: large n).
    Returns (joins, final_n, final_d[, stats])."""
    if copy:
        D = np.array(D, dtype=ETYPES[etype], copy=True)
    else:
        assert D.dtype == ETYPES[etype] and D.flags.c_contiguous and D.flags.writeable
    cap = min(n, max_joins) if max_joins > 0 else n
    joins = np.zeros(max(cap, 1), dtype=JOIN_DTYPE)
    fn = C.c_int(0)
    fd = C.c_double(0)
    st = np.zeros(2, dtype=np.int64)
    nj = lib().orc_tree_ex(n, etype, byte_scale, D.ctypes.data, method, flags, joins.ctypes.data, C.byref(fn),
                           C.byref(fd), st.ctypes.data, max_joins, threads)
    res = (joins[:nj], fn.value, fd.value)
    return res + (st,) if stats else res


class DnjState:
    """A DNJ loop state (dnj.c:985-1052 between two joins): the LT of the
    current n rows, the per-row vectors minQpair reads and its candidate row."""

    def __init__(self, D, n, sD, Q, N, P, cand, etype=8, byte_scale=1.0):
        self.D, self.n, self.sD, self.Q, self.N, self.P = D, int(n), sD, Q, N, P
        self.cand, self.etype, self.byte_scale = int(cand), etype, byte_scale


def dnj_init(D, n, etype=8, byte_scale=1.0, threads=1):
    """initSummaD + initHNJ + the first candidate: the state a whole DNJ run
    starts from.  D is taken over (the state's matrix is D itself)."""
    D = np.ascontiguousarray(D, dtype=ETYPES[etype])
    sD, Q = np.zeros(n), np.zeros(n)
    N, P = np.zeros(n, dtype=np.int32), np.zeros(n, dtype=np.int32)
    cand = lib().orc_dnj_init(n, etype, byte_scale, D.ctypes.data, sD.ctypes.data, Q.ctypes.data, N.ctypes.data,
                              P.ctypes.data, threads)
    return DnjState(D, n, sD, Q, N, P, cand, etype, byte_scale)


def dnj_resume(state, max_joins=0, flags=0, threads=1, stats=False):
    """Continues the DNJ loop from `state` (updated in place) for max_joins
    joins (0: to the end).  Returns (joins, final_n, final_d[, stats])."""
    s = state
    for a, dt in ((s.sD, np.float64), (s.Q, np.float64), (s.N, np.int32), (s.P, np.int32)):
        assert a.dtype == dt and a.flags.c_contiguous and a.flags.writeable and len(a) >= s.n
    assert s.D.dtype == ETYPES[s.etype] and s.D.flags.c_contiguous and s.D.flags.writeable
    assert s.D.size >= s.n * (s.n - 1) // 2
    cap = min(s.n, max_joins) if max_joins > 0 else s.n
    joins = np.zeros(max(cap, 1), dtype=JOIN_DTYPE)
    fn, fd, nc = C.c_int(0), C.c_double(0), C.c_int(0)
    st = np.zeros(2, dtype=np.int64)
    nj = lib().orc_dnj_resume(s.n, s.etype, s.byte_scale, s.D.ctypes.data, s.sD.ctypes.data, s.Q.ctypes.data,
                              s.N.ctypes.data, s.P.ctypes.data, s.cand, flags, joins.ctypes.data, C.byref(fn),
                              C.byref(fd), st.ctypes.data, max_joins, threads, C.byref(nc))
    s.n, s.cand = fn.value, nc.value
    res = (joins[:nj], fn.value, fd.value)
    return res + (st,) if stats else res


def snp_ltd(seqs, incs, n, length, pair=False, norm=0, min_length=1, min_cov=0.0, proxi=0, etype=8,
            byte_scale=1.0, want_n=False, threads=1):
    seqs = np.ascontiguousarray(seqs, dtype=np.uint64)
    incs = np.ascontiguousarray(incs, dtype=np.uint32)
    W = length // 32 + 1
    assert seqs.shape[1] == W
    m = n * (n - 1) // 2
    D = np.zeros(max(m, 1), dtype=ETYPES[etype])
    N = np.zeros(max(m, 1), dtype=ETYPES[etype]) if want_n else None
    inc = lib().orc_snp_ltd_ex(n, length, seqs.ctypes.data, incs.ctypes.data, int(pair), norm, min_length, min_cov,
                               proxi, etype, byte_scale, D.ctypes.data, N.ctypes.data if N is not None else None,
                               threads)
    return D[:m], (N[:m] if N is not None else None), inc


KMA_METRICS = {"cos": 0, "chi2": 2, "nchi2": 3, "nc": 4, "c": 5, "nbc": 8, "bc": 9, "nl1": 10, "nl2": 11,
               "nlinf": 12, "l1": 13, "l2": 14, "linf": 15}


def kma_metric(name):
    """-d name -> (metric id, n of ln / nln) as dist.c:736-790 parses it."""
    if name in KMA_METRICS:
        return KMA_METRICS[name], 0
    if name.startswith("nl") and name[2:].isdigit():
        return 17, int(name[2:])
    if name.startswith("l") and name[1:].isdigit():
        return 16, int(name[1:])
    raise ValueError(name)


def kma_dist(files, tmpl, metric="cos", norm=0, min_depth=15, min_length=1, min_cov=0.5, etype=8,
             byte_scale=1.0, want_n=False):
    """KMA *.mat distances (ltdMatrixThrd).  Returns (D, N, include, n) or
    raises RuntimeError where the reference exits."""
    mid, ln = kma_metric(metric)
    nf = len(files)
    arr = (C.c_char_p * nf)(*[f.encode() for f in files])
    m = max(nf * (nf - 1) // 2, 1)
    D = np.zeros(m, dtype=ETYPES[etype])
    N = np.zeros(m, dtype=ETYPES[etype]) if want_n else None
    inc = np.zeros(nf, dtype=np.uint8)
    n = C.c_int(0)
    rc = lib().orc_kma_dist(nf, arr, tmpl.encode(), mid, ln, norm, min_depth, min_length, min_cov, etype,
                            byte_scale, D.ctypes.data, N.ctypes.data if N is not None else None, inc.ctypes.data,
                            C.byref(n))
    if rc:
        raise RuntimeError(f"orc_kma_dist: {rc}")
    k = n.value * (n.value - 1) // 2
    return D[:k], (N[:k] if N is not None else None), inc, n.value
