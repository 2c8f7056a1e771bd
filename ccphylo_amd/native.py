"""ctypes bindings of the two in-tree shared libraries.

- ``lib/libccphylo_amd.so``  -- the gfx950 engine, C-ABI ``include/ccphylo_amd.h``
  (replaces ``fsaCmpThreadOut`` fsacmpthrd.h:49 and ``dnj_thread``/``nj_thread``
  dnj.c:1054 / nj.c:1612 of the reference).
- ``lib/libccphylo_host.so`` -- Phylip / Newick / FASTA host layer,
  ``include/ccphylo_host.h`` (ref phy.c, nwck.c, seqparse.c, fsacmp.c masks).

There is deliberately no CPU fallback: every GPU entry point raises
``CcgError`` when the engine library is missing or no gfx950 device exists.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIBDIR = os.path.join(HERE, "lib")
# CCPHYLO_AMD_ENGINE: alternative engine build (e.g. the phase-stamp diagnostic one)
ENGINE_PATH = os.environ.get("CCPHYLO_AMD_ENGINE") or os.path.join(LIBDIR, "libccphylo_amd.so")
HOST_PATH = os.path.join(LIBDIR, "libccphylo_host.so")
CLI_PATH = os.path.join(HERE, "bin", "ccphylo")

ETYPES = {8: np.float64, 4: np.float32, 2: np.uint16, 1: np.uint8}

CCG_TREE_NJ = 0
CCG_TREE_DNJ = 1
CCG_TREE_HNJ = 2
NKSTAT = 10
KSTAT_NAMES = ["init", "dnj_select", "dnj_scan", "nj_argmin", "update", "dnj_requeue", "nj_pop", "dnj_find", "coll",
               "exact_sum"]
SHARD_BAND = 8
RCCL_ID_BYTES = 128


class CcgError(RuntimeError):
    pass


class SnpArgs(C.Structure):
    _fields_ = [
        ("n", C.c_int), ("len", C.c_int), ("stride", C.c_int),
        ("seqs", C.c_void_p), ("incs", C.c_void_p),
        ("pair", C.c_int), ("norm", C.c_uint), ("minLength", C.c_uint), ("proxi", C.c_uint),
        ("etype", C.c_int), ("byteScale", C.c_double),
        ("row_begin", C.c_int64), ("row_end", C.c_int64),
    ]


class KmaArgs(C.Structure):
    _fields_ = [
        ("n", C.c_int), ("metric", C.c_int), ("lnorm", C.c_uint), ("norm", C.c_uint), ("minDepth", C.c_uint),
        ("minLength", C.c_uint), ("minCov", C.c_double), ("etype", C.c_int), ("byteScale", C.c_double),
        ("stride1", C.c_int64), ("rec1", C.c_void_p), ("len1", C.c_void_p),
        ("stride2", C.c_int64), ("rec2", C.c_void_p), ("len2", C.c_void_p),
    ]


# -d names of `ccphylo dist` on count matrices (dist.c:736-790) -> CCG_KMA_*
KMA_METRICS = {"cos": 0, "chi2": 2, "nchi2": 3, "nc": 4, "c": 5, "nbc": 8, "bc": 9, "nl1": 10, "nl2": 11,
               "nlinf": 12, "l1": 13, "l2": 14, "linf": 15}


def kma_metric(name):
    """-d name -> (CCG_KMA_* id, n of l<n> / nl<n>)."""
    if name in KMA_METRICS:
        return KMA_METRICS[name], 0
    if name.startswith("nl") and name[2:].isdigit():
        return 17, int(name[2:])
    if name.startswith("l") and name[1:].isdigit():
        return 16, int(name[1:])
    raise ValueError(f"distance method {name!r} is not on the GPU engine")


class TreeArgs(C.Structure):
    _fields_ = [
        ("n", C.c_int), ("etype", C.c_int), ("byteScale", C.c_double),
        ("method", C.c_int), ("flags", C.c_int), ("exact", C.c_int), ("profile", C.c_int),
        ("max_joins", C.c_int),
    ]


class Join(C.Structure):
    _fields_ = [("i", C.c_int32), ("j", C.c_int32), ("Li", C.c_double), ("Lj", C.c_double)]


# ccg_coll (include/ccphylo_amd.h): the sharded tree loop's collectives
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p)
BROADCAST_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p)


class DnjState(C.Structure):
    """ccg_dnj_state: a DNJ loop state between two joins (host arrays)."""
    _fields_ = [("n", C.c_int), ("cand", C.c_int), ("sD", C.c_void_p), ("Q", C.c_void_p), ("N", C.c_void_p),
                ("P", C.c_void_p)]


class Coll(C.Structure):
    _fields_ = [("user", C.c_void_p), ("rank", C.c_int), ("world", C.c_int), ("host_staged", C.c_int),
                ("allreduce_sum_u8", ALLREDUCE_FN), ("broadcast", BROADCAST_FN), ("allgather", ALLGATHER_FN)]


CCG_CTX_NOSYNC = 1
JOIN_DTYPE = np.dtype([("i", np.int32), ("j", np.int32), ("Li", np.float64), ("Lj", np.float64)])

# every symbol of include/ccphylo_amd.h
ENGINE_SYMBOLS = [
    "ccg_init", "ccg_device_count", "ccg_destroy", "ccg_strerror", "ccg_device_info",
    "ccg_snp_ltd", "ccg_snp_ltd_dev", "ccg_tree", "ccg_tree_dev",
    "ccg_malloc", "ccg_free", "ccg_memcpy_h2d", "ccg_memcpy_d2h", "ccg_synchronize",
    "ccg_shard_owner", "ccg_shard_row_offset", "ccg_shard_elems",
    "ccg_rccl_unique_id", "ccg_rccl_open", "ccg_rccl_close", "ccg_rccl_abort", "ccg_tree_shard", "ccg_tree_shard_dev",
    "ccg_kma_ltd", "ccg_kma_ltd_dev", "ccg_snp_ltd_shard_dev", "ccg_snp_ltd_shard", "ccg_selftest_row_sum",
    "ccg_round_decimal_dev", "ccg_last_dist_ms", "ccg_tree_dev_state", "ccg_tree_shard_bytes", "ccg_ctx_configure",
    "ccg_shutdown",
]
# every symbol of include/ccphylo_host.h
HOST_SYMBOLS = [
    "ccq_new", "ccq_free", "ccq_open", "ccq_close", "ccq_peek",
    "ccq_ltd_new", "ccq_ltd_free", "ccq_ltd_reserve", "ccq_ltd_get", "ccq_ltd_set",
    "ccq_names_new", "ccq_names_free", "ccq_names_set", "ccq_load_phy", "ccq_print_phy",
    "ccq_replay_newick", "ccq_replay_newick_strings", "ccq_newick_pair",
    "ccq_code_table", "ccq_read_fasta", "ccq_pack", "ccq_init_inc", "ccq_inc_update", "ccq_npos",
    "ccq_load_msa", "ccq_load_msa_par", "ccq_msa_free", "ccq_load_fsa_files", "ccq_load_kma", "ccq_kma_free",
]

_engine = None
_host = None


def _preload_torch_hip():
    """PyTorch ships its own libamdhip64 (SONAME libamdhip64.so.7, loaded by
    libtorch_hip as "libamdhip64.so").  Loading it first makes the engine bind
    to the same HIP runtime, whichever of torch / the engine comes first in the
    process: one runtime, so device pointers, streams and
    hipDeviceSynchronize are shared with torch (two runtimes in one process
    leave torch without a device)."""
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    p = os.path.join(list(spec.submodule_search_locations)[0], "lib", "libamdhip64.so")
    if os.path.exists(p):
        C.CDLL(p, mode=C.RTLD_GLOBAL)


def engine_lib():
    """Loads libccphylo_amd.so (raises if it was not built)."""
    global _engine
    if _engine is None:
        if not os.path.exists(ENGINE_PATH):
            raise CcgError(f"{ENGINE_PATH} missing: run __graft_entry__.build() (no CPU fallback)")
        _preload_torch_hip()
        lib = C.CDLL(ENGINE_PATH)
        lib.ccg_init.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
        lib.ccg_destroy.argtypes = [C.c_void_p]
        lib.ccg_destroy.restype = None
        lib.ccg_ctx_configure.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.c_int, C.c_int]
        lib.ccg_strerror.argtypes = [C.c_int]
        lib.ccg_strerror.restype = C.c_char_p
        lib.ccg_device_info.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
        lib.ccg_snp_ltd.argtypes = [C.c_void_p, C.POINTER(SnpArgs), C.c_void_p, C.c_void_p, C.POINTER(C.c_int)]
        lib.ccg_snp_ltd_dev.argtypes = lib.ccg_snp_ltd.argtypes
        lib.ccg_tree.argtypes = [C.c_void_p, C.POINTER(TreeArgs), C.c_void_p, C.c_void_p, C.POINTER(C.c_int),
                                 C.POINTER(C.c_int), C.POINTER(C.c_double), C.POINTER(C.c_int64)]
        lib.ccg_tree_dev.argtypes = lib.ccg_tree.argtypes
        lib.ccg_tree_dev_state.argtypes = [C.c_void_p, C.POINTER(TreeArgs), C.c_void_p, C.POINTER(DnjState),
                                           C.POINTER(DnjState), C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                           C.POINTER(C.c_double), C.POINTER(C.c_int64)]
        lib.ccg_malloc.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.c_size_t]
        lib.ccg_free.argtypes = [C.c_void_p, C.c_void_p]
        lib.ccg_memcpy_h2d.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
        lib.ccg_memcpy_d2h.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
        lib.ccg_synchronize.argtypes = [C.c_void_p]
        lib.ccg_shard_owner.argtypes = [C.c_int64, C.c_int]
        lib.ccg_shard_row_offset.argtypes = [C.c_int64, C.c_int, C.c_int]
        lib.ccg_shard_row_offset.restype = C.c_int64
        lib.ccg_shard_elems.argtypes = [C.c_int64, C.c_int, C.c_int]
        lib.ccg_shard_elems.restype = C.c_int64
        lib.ccg_rccl_unique_id.argtypes = [C.c_void_p]
        lib.ccg_rccl_open.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.POINTER(Coll)]
        lib.ccg_rccl_close.argtypes = [C.POINTER(Coll)]
        lib.ccg_rccl_abort.argtypes = [C.POINTER(Coll)]
        lib.ccg_tree_shard.argtypes = [C.c_void_p, C.POINTER(TreeArgs), C.POINTER(Coll), C.c_void_p, C.c_void_p,
                                       C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_double),
                                       C.POINTER(C.c_int64)]
        lib.ccg_tree_shard_dev.argtypes = lib.ccg_tree_shard.argtypes
        lib.ccg_tree_shard_bytes.argtypes = [C.c_int64, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int64),
                                             C.POINTER(C.c_int64)]
        lib.ccg_kma_ltd.argtypes = [C.c_void_p, C.POINTER(KmaArgs), C.c_void_p, C.c_void_p, C.POINTER(C.c_int64)]
        lib.ccg_kma_ltd_dev.argtypes = lib.ccg_kma_ltd.argtypes
        lib.ccg_selftest_row_sum.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_double),
                                             C.POINTER(C.c_int)]
        _engine = lib
    return _engine


def host_lib():
    global _host
    if _host is None:
        if not os.path.exists(HOST_PATH):
            raise CcgError(f"{HOST_PATH} missing: run __graft_entry__.build()")
        lib = C.CDLL(HOST_PATH)
        lib.ccq_new.restype = C.c_void_p
        lib.ccq_new.argtypes = [C.c_uint32]
        lib.ccq_open.restype = C.c_void_p
        lib.ccq_open.argtypes = [C.c_char_p]
        lib.ccq_peek.restype = C.c_int
        lib.ccq_peek.argtypes = [C.c_void_p]
        lib.ccq_close.argtypes = [C.c_void_p]
        lib.ccq_ltd_new.restype = C.c_void_p
        lib.ccq_ltd_new.argtypes = [C.c_int, C.c_int, C.c_double]
        lib.ccq_ltd_free.argtypes = [C.c_void_p]
        lib.ccq_names_new.restype = C.c_void_p
        lib.ccq_names_new.argtypes = [C.c_int, C.c_uint32]
        lib.ccq_names_free.argtypes = [C.c_void_p]
        lib.ccq_load_phy.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_char, C.c_char, C.POINTER(C.c_int)]
        lib.ccq_replay_newick.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_int, C.c_int]
        lib.ccq_newick_pair.argtypes = [C.c_void_p, C.c_double, C.c_int]
        lib.ccq_code_table.argtypes = [C.c_uint, C.c_void_p]
        lib.ccq_pack.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        lib.ccq_init_inc.argtypes = [C.c_void_p, C.c_int]
        lib.ccq_inc_update.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_uint, C.c_int]
        lib.ccq_npos.argtypes = [C.c_void_p, C.c_int]
        lib.ccq_load_msa.restype = C.c_void_p
        lib.ccq_load_msa.argtypes = [C.c_void_p, C.c_uint, C.c_uint, C.c_double, C.c_uint, C.c_void_p]
        lib.ccq_load_msa_par.restype = C.c_void_p
        lib.ccq_load_msa_par.argtypes = [C.c_void_p, C.c_uint, C.c_uint, C.c_double, C.c_uint, C.c_int, C.c_void_p]
        lib.ccq_msa_free.argtypes = [C.c_void_p]
        lib.ccq_load_kma.restype = C.c_void_p
        lib.ccq_load_kma.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.c_uint, C.c_uint, C.c_double, C.c_int,
                                     C.c_void_p]
        lib.ccq_kma_free.argtypes = [C.c_void_p]
        _host = lib
    return _host


# ---------------------------------------------------------------- host structs
class _Str(C.Structure):
    _fields_ = [("size", C.c_uint32), ("len", C.c_uint32), ("seq", C.c_char_p)]


class _Ltd(C.Structure):
    _fields_ = [("n", C.c_int), ("size", C.c_int), ("et", C.c_int), ("bs", C.c_double), ("mat", C.c_void_p)]


class _Names(C.Structure):
    _fields_ = [("cap", C.c_int), ("names", C.POINTER(C.POINTER(_Str))), ("header", C.POINTER(_Str))]


class _Msa(C.Structure):
    _fields_ = [("n", C.c_int), ("len", C.c_int), ("W", C.c_int), ("pair", C.c_int),
                ("headers", C.POINTER(C.c_char_p)), ("seqs", C.POINTER(C.c_uint64)),
                ("incs", C.POINTER(C.c_uint32)), ("minLength", C.c_uint)]


class _Kma(C.Structure):
    _fields_ = [("nfiles", C.c_int), ("n", C.c_int), ("status", C.c_int), ("include", C.POINTER(C.c_uint8)),
                ("file_of", C.POINTER(C.c_int)), ("stride1", C.c_int64), ("stride2", C.c_int64),
                ("rec1", C.POINTER(C.c_uint16)), ("rec2", C.POINTER(C.c_uint16)),
                ("len1", C.POINTER(C.c_int32)), ("len2", C.POINTER(C.c_int32))]


# ---------------------------------------------------------------- engine API
class Device:
    """An open gfx950 device + engine stream (ccg_init)."""

    def __init__(self, device: int = 0):
        self.lib = engine_lib()
        h = C.c_void_p()
        rc = self.lib.ccg_init(int(device), C.byref(h))
        if rc != 0:
            raise CcgError(f"ccg_init({device}) failed: {self.lib.ccg_strerror(rc).decode()}")
        self.h = h

    @staticmethod
    def count() -> int:
        """Visible GPUs (ccg_device_count)."""
        c = C.c_int(0)
        rc = engine_lib().ccg_device_count(C.byref(c))
        return c.value if rc == 0 else 0

    def close(self):
        if self.h:
            self.lib.ccg_destroy(self.h)
            self.h = None

    def configure(self, cu_mask=None, nosync=False):
        """ccg_ctx_configure: cu_mask (a sequence of CU indices, or None: all)
        limits the engine stream to those compute units; nosync: the entry
        points do not wait for the whole device first (two contexts side by
        side: the caller orders their inputs)."""
        words = None
        nw = 0
        if cu_mask is not None:
            cus = sorted(set(int(x) for x in cu_mask))
            nw = max(cus) // 32 + 1 if cus else 0
            words = (C.c_uint32 * max(nw, 1))()
            for cu in cus:
                words[cu // 32] |= 1 << (cu % 32)
        self._check(self.lib.ccg_ctx_configure(self.h, words, nw, CCG_CTX_NOSYNC if nosync else 0),
                    "ccg_ctx_configure")
        if nw:
            _register_shutdown(self.lib)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self) -> str:
        buf = C.create_string_buffer(256)
        self.lib.ccg_device_info(self.h, buf, 256)
        return buf.value.decode()

    def _check(self, rc, what):
        if rc != 0:
            raise CcgError(f"{what}: {self.lib.ccg_strerror(rc).decode()}")

    def snp_ltd(self, seqs, incs, n, length, pair=False, norm=0, min_length=1, etype=8, byte_scale=1.0,
                proxi=0, want_n=False, row_range=(0, 0)):
        """All-pairs SNP distances (ccg_snp_ltd).  seqs: uint64[n, stride]
        (qseq2nibble layout); incs: uint32[stride] or uint32[n, stride].
        Returns (D, N, inc) with D/N packed LT arrays of the element type."""
        seqs = np.ascontiguousarray(seqs, dtype=np.uint64)
        incs = np.ascontiguousarray(incs, dtype=np.uint32)
        stride = seqs.shape[1]
        m = n * (n - 1) // 2
        D = np.zeros(max(m, 1), dtype=ETYPES[etype])
        N = np.zeros(max(m, 1), dtype=ETYPES[etype]) if (want_n and pair) else None
        a = SnpArgs(n, length, stride, seqs.ctypes.data, incs.ctypes.data, int(pair), norm, min_length, proxi,
                    etype, byte_scale, row_range[0], row_range[1])
        inc = C.c_int(0)
        rc = self.lib.ccg_snp_ltd(self.h, C.byref(a), D.ctypes.data, N.ctypes.data if N is not None else None,
                                  C.byref(inc))
        self._check(rc, "ccg_snp_ltd")
        return D[:m], (N[:m] if N is not None else None), inc.value

    def tree(self, D, n, etype=8, byte_scale=1.0, method=CCG_TREE_DNJ, flags=0, exact=True, profile=False,
             max_joins=0):
        """NJ/DNJ on a packed host LT (ccg_tree).  Returns (joins, final_n, final_d, stats)."""
        D = np.ascontiguousarray(D, dtype=ETYPES[etype])
        assert D.size == n * (n - 1) // 2
        return self._tree(self.lib.ccg_tree, D.ctypes.data, n, etype, byte_scale, method, flags, exact, profile,
                          max_joins)

    def tree_dev(self, dptr, n, etype=8, byte_scale=1.0, method=CCG_TREE_DNJ, flags=0, exact=True, profile=False,
                 max_joins=0):
        """Same on a device LT (ccg_tree_dev); the buffer is consumed."""
        return self._tree(self.lib.ccg_tree_dev, dptr, n, etype, byte_scale, method, flags, exact, profile,
                          max_joins)

    def tree_dev_state(self, dptr, n, etype=8, byte_scale=1.0, flags=0, exact=True, profile=False, max_joins=0,
                       state=None, want_state=True):
        """DNJ on a device LT with a checkpoint (ccg_tree_dev_state): `state`
        (a dict n, cand, sD, Q, N, P, e.g. a previous call's) resumes the loop
        instead of initialising it; with want_state the state after the last
        join comes back.  Returns (joins, final_n, final_d, stats, state)."""
        sin = None
        if state is not None:
            arrs = [np.ascontiguousarray(state[k], dtype=t) for k, t in
                    (("sD", np.float64), ("Q", np.float64), ("N", np.int32), ("P", np.int32))]
            assert int(state["n"]) == n and all(len(x) >= n for x in arrs)
            sin = DnjState(n, int(state["cand"]), *[x.ctypes.data for x in arrs])
        out, sout = None, None
        if want_state:
            out = {"sD": np.zeros(n), "Q": np.zeros(n), "N": np.zeros(n, dtype=np.int32),
                   "P": np.zeros(n, dtype=np.int32)}
            sout = DnjState(0, 0, out["sD"].ctypes.data, out["Q"].ctypes.data, out["N"].ctypes.data,
                            out["P"].ctypes.data)
        joins = np.zeros(max(n, 1), dtype=JOIN_DTYPE)
        nj, fn, fd = C.c_int(0), C.c_int(0), C.c_double(0)
        st = (C.c_int64 * (12 + 2 * NKSTAT))()
        a = TreeArgs(n, etype, byte_scale, CCG_TREE_DNJ, flags, int(exact), int(profile), int(max_joins))
        rc = self.lib.ccg_tree_dev_state(self.h, C.byref(a), C.c_void_p(dptr), C.byref(sin) if sin else None,
                                         C.byref(sout) if sout else None, joins.ctypes.data, C.byref(nj),
                                         C.byref(fn), C.byref(fd), st)
        self._check(rc, "ccg_tree_dev_state")
        if out is not None:
            m = sout.n
            out = {k: v[:m] for k, v in out.items()}
            out["n"], out["cand"] = m, sout.cand
        return joins[:nj.value], fn.value, fd.value, list(st), out

    def _tree(self, fn_, dptr, n, etype, byte_scale, method, flags, exact, profile, max_joins=0):
        joins = np.zeros(max(n, 1), dtype=JOIN_DTYPE)
        nj = C.c_int(0)
        fn = C.c_int(0)
        fd = C.c_double(0)
        st = (C.c_int64 * (12 + 2 * NKSTAT))()
        a = TreeArgs(n, etype, byte_scale, method, flags, int(exact), int(profile), int(max_joins))
        rc = fn_(self.h, C.byref(a), C.c_void_p(dptr), joins.ctypes.data, C.byref(nj), C.byref(fn), C.byref(fd), st)
        self._check(rc, "ccg_tree")
        return joins[:nj.value], fn.value, fd.value, list(st)

    def tree_shard(self, D, n, coll=None, etype=8, byte_scale=1.0, method=CCG_TREE_NJ, flags=0, exact=True,
                   profile=False, max_joins=0):
        """Sharded NJ / DNJ from the full host LT (ccg_tree_shard): this rank
        uploads its own row bands only.  `coll`: a HostColl / RcclColl (None =
        world 1)."""
        D = np.ascontiguousarray(D, dtype=ETYPES[etype])
        assert D.size == n * (n - 1) // 2
        return self._tree_shard(self.lib.ccg_tree_shard, D.ctypes.data, n, coll, etype, byte_scale, method, flags,
                                exact, profile, max_joins)

    def tree_shard_dev(self, dptr, n, coll=None, etype=8, byte_scale=1.0, method=CCG_TREE_NJ, flags=0, exact=True,
                       profile=False, max_joins=0):
        """Sharded NJ / DNJ on this rank's device row bands (ccg_tree_shard_dev; consumed)."""
        return self._tree_shard(self.lib.ccg_tree_shard_dev, dptr, n, coll, etype, byte_scale, method, flags,
                                exact, profile, max_joins)

    def _tree_shard(self, fn_, ptr, n, coll, etype, byte_scale, method, flags, exact, profile, max_joins):
        joins = np.zeros(max(n, 1), dtype=JOIN_DTYPE)
        nj = C.c_int(0)
        fn = C.c_int(0)
        fd = C.c_double(0)
        st = (C.c_int64 * (12 + 2 * NKSTAT))()
        a = TreeArgs(n, etype, byte_scale, method, flags, int(exact), int(profile), int(max_joins))
        cp = C.byref(coll.c) if coll is not None else None
        rc = fn_(self.h, C.byref(a), cp, C.c_void_p(ptr), joins.ctypes.data, C.byref(nj), C.byref(fn), C.byref(fd),
                 st)
        self._check(rc, "ccg_tree_shard")
        return joins[:nj.value], fn.value, fd.value, list(st)

    def kma_ltd(self, K, metric="cos", norm=0, min_depth=15, min_length=1, min_cov=0.5, etype=8, byte_scale=1.0,
                want_n=False):
        """Count-matrix distances (ccg_kma_ltd) of the samples of a
        load_kma() result.  Returns (D, N, fatal) with fatal the flat index of
        the first pair where the reference would exit(1), or -1."""
        mid, ln = kma_metric(metric)
        n = K["n"]
        m = n * (n - 1) // 2
        D = np.zeros(max(m, 1), dtype=ETYPES[etype])
        N = np.zeros(max(m, 1), dtype=ETYPES[etype]) if want_n else None
        a = KmaArgs(n, mid, ln, norm, min_depth, min_length, min_cov, etype, byte_scale,
                    K["stride1"], K["rec1"].ctypes.data, K["len1"].ctypes.data,
                    K["stride2"], K["rec2"].ctypes.data, K["len2"].ctypes.data)
        fatal = C.c_int64(-1)
        rc = self.lib.ccg_kma_ltd(self.h, C.byref(a), D.ctypes.data, N.ctypes.data if N is not None else None,
                                  C.byref(fatal))
        self._check(rc, "ccg_kma_ltd")
        return D[:m], (N[:m] if N is not None else None), fatal.value

    def kma_ltd_dev(self, n, rec1_ptr, len1_ptr, stride1, rec2_ptr, len2_ptr, stride2, D_ptr, N_ptr=None,
                    metric="cos", norm=0, min_depth=15, min_length=1, min_cov=0.5, etype=8, byte_scale=1.0):
        """ccg_kma_ltd_dev on device views; returns the fatal flat index or -1."""
        mid, ln = kma_metric(metric)
        a = KmaArgs(n, mid, ln, norm, min_depth, min_length, min_cov, etype, byte_scale,
                    stride1, rec1_ptr, len1_ptr, stride2, rec2_ptr, len2_ptr)
        fatal = C.c_int64(-1)
        self._check(self.lib.ccg_kma_ltd_dev(self.h, C.byref(a), C.c_void_p(D_ptr),
                                             C.c_void_p(N_ptr) if N_ptr else None, C.byref(fatal)),
                    "ccg_kma_ltd_dev")
        return fatal.value

    def last_dist_ms(self):
        """HIP-event duration of the last dist call's pair kernels (ccg_last_dist_ms)."""
        ms = C.c_double(0)
        self._check(self.lib.ccg_last_dist_ms(self.h, C.byref(ms)), "ccg_last_dist_ms")
        return ms.value

    def selftest_row_sum(self, c):
        """The engine's exact-mode row sum of c (ccg_selftest_row_sum): returns
        (serial sum, True when the parallel binade-segmented form produced it)."""
        c = np.ascontiguousarray(c, dtype=np.float64)
        out = C.c_double(0)
        par = C.c_int(0)
        self._check(self.lib.ccg_selftest_row_sum(self.h, c.ctypes.data, len(c), C.byref(out), C.byref(par)),
                    "ccg_selftest_row_sum")
        return out.value, bool(par.value)

    # ---- device memory (ccg_malloc & co.) for HBM-resident inputs
    def malloc(self, nbytes):
        p = C.c_void_p()
        self._check(self.lib.ccg_malloc(self.h, C.byref(p), nbytes), "ccg_malloc")
        return p.value

    def free(self, p):
        self._check(self.lib.ccg_free(self.h, C.c_void_p(p)), "ccg_free")

    def h2d(self, dst, arr):
        arr = np.ascontiguousarray(arr)
        self._check(self.lib.ccg_memcpy_h2d(self.h, C.c_void_p(dst), arr.ctypes.data, arr.nbytes), "h2d")

    def d2h(self, arr, src):
        self._check(self.lib.ccg_memcpy_d2h(self.h, arr.ctypes.data, C.c_void_p(src), arr.nbytes), "d2h")

    def sync(self):
        self._check(self.lib.ccg_synchronize(self.h), "ccg_synchronize")

    def snp_ltd_dev(self, seqs_ptr, incs_ptr, n, length, stride, D_ptr, N_ptr=None, pair=False, norm=0,
                    min_length=1, etype=8, byte_scale=1.0, row_range=(0, 0)):
        """ccg_snp_ltd_dev on device pointers.  Returns getNpos(mask) (non-pair)."""
        a = SnpArgs(n, length, stride, seqs_ptr, incs_ptr, int(pair), norm, min_length, 0, etype, byte_scale,
                    row_range[0], row_range[1])
        inc = C.c_int(0)
        self._check(self.lib.ccg_snp_ltd_dev(self.h, C.byref(a), C.c_void_p(D_ptr),
                                             C.c_void_p(N_ptr) if N_ptr else None, C.byref(inc)), "ccg_snp_ltd_dev")
        return inc.value


    def snp_ltd_shard_dev(self, seqs_ptr, incs_ptr, n, length, stride, Dloc_ptr, rank, world, norm=0, etype=8,
                          byte_scale=1.0, pair=False, min_length=1, proxi=0):
        """ccg_snp_ltd_shard_dev: the rank's rows of the band layout, straight
        into its shard buffer (device pointers).  Returns getNpos(mask) (0 in
        pair mode, where incs holds one mask per taxon)."""
        a = SnpArgs(n, length, stride, seqs_ptr, incs_ptr, int(pair), norm, min_length, proxi if pair else 0, etype,
                    byte_scale, 0, 0)
        inc = C.c_int(0)
        self._check(self.lib.ccg_snp_ltd_shard_dev(self.h, C.byref(a), rank, world, C.c_void_p(Dloc_ptr),
                                                   C.byref(inc)), "ccg_snp_ltd_shard_dev")
        return inc.value

    def snp_ltd_shard(self, seqs, incs, n, length, Dloc_ptr, rank, world, norm=0, etype=8, byte_scale=1.0,
                      pair=False, min_length=1, proxi=0):
        """ccg_snp_ltd_shard: as snp_ltd_shard_dev with the packed MSA in host
        memory (numpy uint64[n, stride] / uint32 masks), streamed into the bit
        planes; Dloc_ptr is the rank's device shard."""
        seqs = np.ascontiguousarray(seqs, dtype=np.uint64)
        incs = np.ascontiguousarray(incs, dtype=np.uint32)
        a = SnpArgs(n, length, seqs.shape[1], seqs.ctypes.data, incs.ctypes.data, int(pair), norm, min_length,
                    proxi if pair else 0, etype, byte_scale, 0, 0)
        inc = C.c_int(0)
        self._check(self.lib.ccg_snp_ltd_shard(self.h, C.byref(a), rank, world, C.c_void_p(Dloc_ptr), C.byref(inc)),
                    "ccg_snp_ltd_shard")
        return inc.value


# ---------------------------------------------------------------- sharding
def tree_shard_bytes(n, etype=4, method=CCG_TREE_DNJ, world=8):
    """(device bytes ccg_tree_shard_dev allocates beside the shard, bound on
    the init's hard-column gather buffer) -- ccg_tree_shard_bytes (no GPU)."""
    d, g = C.c_int64(0), C.c_int64(0)
    rc = engine_lib().ccg_tree_shard_bytes(int(n), etype, method, world, C.byref(d), C.byref(g))
    if rc:
        raise CcgError(f"ccg_tree_shard_bytes: {rc}")
    return d.value, g.value


def shard_owner(row, world):
    """Rank owning LT row `row`: bands of SHARD_BAND rows dealt round-robin."""
    return (row // SHARD_BAND) % world


def shard_row_offset(row, rank, world):
    """Element offset of owned row `row` in its rank's buffer (ccg_shard_row_offset)."""
    return engine_lib().ccg_shard_row_offset(int(row), int(rank), int(world))


def shard_elems(n, rank, world):
    """Elements of a rank's rows below n (ccg_shard_elems)."""
    return engine_lib().ccg_shard_elems(int(n), int(rank), int(world))


def shard_extract(D, n, rank, world):
    """This rank's rows of a full packed LT, back to back (the layout of
    ccg_tree_shard_dev's buffer)."""
    D = np.asarray(D)
    out = np.empty(shard_elems(n, rank, world), dtype=D.dtype)
    for g in range(rank, (n + SHARD_BAND - 1) // SHARD_BAND, world):
        r0, r1 = g * SHARD_BAND, min(g * SHARD_BAND + SHARD_BAND, n)
        o = shard_row_offset(r0, rank, world)
        out[o:o + (r1 * (r1 - 1) - r0 * (r0 - 1)) // 2] = D[r0 * (r0 - 1) // 2:r1 * (r1 - 1) // 2]
    return out


class HostColl:
    """Host-staged ccg_coll over torch.distributed (gloo): the engine copies
    each exchange to host memory and calls back here.  For tests and for
    transports without GPU-direct collectives."""

    def __init__(self, dist, group=None, allgather_native=True):
        """allgather_native=False leaves ccg_coll.allgather NULL, so the engine
        emulates it with the allreduce (tests both paths)."""
        import torch
        self._torch = torch
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.calls = 0
        self.bytes = 0
        self.errors = []

        def _arr(buf, nbytes):
            return torch.from_numpy(np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(buf)))

        def allreduce(user, buf, nbytes, stream):
            try:
                self.calls += 1
                self.bytes += nbytes
                if nbytes:
                    t = _arr(buf, nbytes)
                    # gloo sums uint8 elementwise; only one rank is non-zero per byte
                    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
                return 0
            except Exception as e:  # never unwind through C
                self.errors.append(repr(e))
                return 1

        def broadcast(user, send, recv, nbytes, root, stream):
            try:
                self.calls += 1
                self.bytes += nbytes
                if nbytes:
                    t = _arr(recv, nbytes)
                    if self.rank == root and send != recv:
                        C.memmove(recv, send, nbytes)
                    dist.broadcast(t, src=dist.get_global_rank(group, root) if group is not None else root,
                                   group=group)
                return 0
            except Exception as e:
                self.errors.append(repr(e))
                return 1

        def allgather(user, send, recv, nbytes, stream):
            try:
                self.calls += 1
                self.bytes += nbytes * self.world
                if nbytes:
                    mine = _arr(send, nbytes).clone()   # send may alias this rank's slot of recv
                    out = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(self.world)]
                    dist.all_gather(out, mine, group=group)
                    allb = torch.cat(out).numpy()   # keep it alive across the copy
                    C.memmove(recv, allb.ctypes.data, nbytes * self.world)
                return 0
            except Exception as e:
                self.errors.append(repr(e))
                return 1

        self._ar = ALLREDUCE_FN(allreduce)   # keep the thunks alive
        self._bc = BROADCAST_FN(broadcast)
        self._ag = ALLGATHER_FN(allgather)
        self.c = Coll(None, self.rank, self.world, 1, self._ar, self._bc,
                      self._ag if allgather_native else ALLGATHER_FN())


class RcclColl:
    """ccg_coll over RCCL (ccg_rccl_open): device buffers, enqueued on the
    engine stream.  Rank 0 makes the id; it travels over `dist` (any backend)."""

    def __init__(self, dev, dist, group=None):
        import torch
        lib = engine_lib()
        self.lib = lib
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        ident = (C.c_uint8 * RCCL_ID_BYTES)()
        if rank == 0:
            rc = lib.ccg_rccl_unique_id(ident)
            if rc != 0:
                raise CcgError(f"ccg_rccl_unique_id: {lib.ccg_strerror(rc).decode()}")
        obj = [bytes(ident)]
        dist.broadcast_object_list(obj, src=0, group=group)
        C.memmove(ident, obj[0], RCCL_ID_BYTES)
        self.c = Coll()
        rc = lib.ccg_rccl_open(dev.h, ident, rank, world, C.byref(self.c))
        if rc != 0:
            raise CcgError(f"ccg_rccl_open: {lib.ccg_strerror(rc).decode()}")
        self.rank, self.world = rank, world

    def close(self):
        if self.c.user:
            self.lib.ccg_rccl_close(C.byref(self.c))


_SHUTDOWN = []


def _register_shutdown(lib):
    """At interpreter exit (after the last GPU work), release the CU-masked
    streams the engine keeps (ccg_shutdown)."""
    if not _SHUTDOWN:
        import atexit
        _SHUTDOWN.append(lib)
        atexit.register(lambda: lib.ccg_shutdown())


# ---------------------------------------------------------------- host API
def load_phylip(path, etype=8, byte_scale=1.0, sep="\t", quotes=""):
    """All matrices of a Phylip file (ccq_load_phy).  Returns a list of
    (names, D) with D the packed LT array."""
    lib = host_lib()
    r = lib.ccq_open(path.encode())
    if not r:
        raise FileNotFoundError(path)
    D = lib.ccq_ltd_new(32, etype, byte_scale)
    T = lib.ccq_names_new(32, 4)
    out = []
    err = C.c_int(0)
    try:
        while True:
            n = lib.ccq_load_phy(r, D, T, sep.encode()[:1] or b"\t", quotes.encode()[:1] or b"\0", C.byref(err))
            if n <= 0:
                break
            ltd = _Ltd.from_address(D)
            names = _Names.from_address(T)
            nm = [names.names[k].contents.seq[:names.names[k].contents.len].decode() for k in range(n)]
            m = n * (n - 1) // 2
            buf = (C.c_char * (m * etype)).from_address(ltd.mat) if m else b""
            arr = np.frombuffer(bytes(buf), dtype=ETYPES[etype]).copy() if m else np.zeros(0, ETYPES[etype])
            out.append((nm, arr))
    finally:
        lib.ccq_close(r)
        lib.ccq_ltd_free(D)
        lib.ccq_names_free(T)
    return out


def newick_from_phylip(path, joins_fn, etype=8, byte_scale=1.0, flags=0, precision=9):
    """Runs `joins_fn(D, n) -> (joins, final_n, final_d)` on every matrix of a
    Phylip file and rebuilds the Newick strings exactly as `ccphylo tree`
    prints them (one per matrix, with the trailing ';').  The name table is
    shared across matrices like the reference's (tree.c:61-66)."""
    lib = host_lib()
    r = lib.ccq_open(path.encode())
    if not r:
        raise FileNotFoundError(path)
    D = lib.ccq_ltd_new(32, etype, byte_scale)
    T = lib.ccq_names_new(32, 4)
    err = C.c_int(0)
    trees = []
    try:
        while True:
            n = lib.ccq_load_phy(r, D, T, b"\t", b"\0", C.byref(err))
            if n <= 0:
                break
            ltd = _Ltd.from_address(D)
            m = n * (n - 1) // 2
            if n > 2:
                arr = np.frombuffer((C.c_char * (m * etype)).from_address(ltd.mat), dtype=ETYPES[etype]).copy()
                joins, fn, fd = joins_fn(arr, n)
                joins = np.ascontiguousarray(joins, dtype=JOIN_DTYPE)
                lib.ccq_replay_newick(T, n, joins.ctypes.data, len(joins), fn, fd, flags, precision)
            elif n == 2:
                lib.ccq_newick_pair(T, float(np.frombuffer((C.c_char * etype).from_address(ltd.mat),
                                                           dtype=ETYPES[etype])[0]) / (byte_scale if etype <= 2 else 1.0),
                                    precision)
            names = _Names.from_address(T)
            s = names.names[0].contents.seq.decode()
            hdr = names.header.contents
            trees.append((">" + hdr.seq.decode() if hdr.len else "") + s + ";")
    finally:
        lib.ccq_close(r)
        lib.ccq_ltd_free(D)
        lib.ccq_names_free(T)
    return trees


def load_msa(path, flag=1, min_length=1, min_cov=0.5, proxi=0, threads=0, log_path=None):
    """FASTA MSA -> (headers, seqs uint64[n, W], incs, minLength) per ltdMsaMatrix_get.
    threads > 0: the parallel loader (ccq_load_msa_par); log_path: where the
    Included / Excluded lines go (default /dev/null)."""
    lib = host_lib()
    r = lib.ccq_open(path.encode())
    if not r:
        raise FileNotFoundError(path)
    libc = C.CDLL(None)
    libc.fopen.restype = C.c_void_p
    libc.fopen.argtypes = [C.c_char_p, C.c_char_p]
    libc.fclose.argtypes = [C.c_void_p]
    log = libc.fopen((log_path or "/dev/null").encode(), b"w")
    try:
        lib.ccq_peek(r)
        if threads > 0:
            Mp = lib.ccq_load_msa_par(r, flag, min_length, min_cov, proxi, threads, log)
        else:
            Mp = lib.ccq_load_msa(r, flag, min_length, min_cov, proxi, log)
    finally:
        lib.ccq_close(r)
        libc.fclose(log)
    M = _Msa.from_address(Mp)
    n, W = M.n, M.W
    heads = [M.headers[k].decode() for k in range(n)]
    seqs = np.ctypeslib.as_array(M.seqs, shape=(max(n, 1) * W,))[: n * W].reshape(n, W).copy() if n else np.zeros((0, W), np.uint64)
    ninc = n if M.pair else 1
    incs = np.ctypeslib.as_array(M.incs, shape=(max(ninc, 1) * W,))[: ninc * W].copy() if (n and W) else np.zeros(W, np.uint32)
    if M.pair:
        incs = incs.reshape(n, W)
    res = (heads, seqs, incs, M.len, M.minLength)
    lib.ccq_msa_free(Mp)
    return res


def load_kma(files, tmpl, min_depth=15, min_length=1, min_cov=0.5, threads=16):
    """KMA count matrices -> the engine's sample views (ccq_load_kma): a dict
    with n, include (per file), file_of, rec1 (n, stride1, 8), len1, rec2,
    len2 as numpy arrays."""
    lib = host_lib()
    libc = C.CDLL(None)
    libc.fopen.restype = C.c_void_p
    libc.fopen.argtypes = [C.c_char_p, C.c_char_p]
    libc.fclose.argtypes = [C.c_void_p]
    log = libc.fopen(b"/dev/null", b"w")
    arr = (C.c_char_p * max(len(files), 1))(*[f.encode() for f in files])
    try:
        p = lib.ccq_load_kma(arr, len(files), tmpl.encode(), min_depth, min_length, min_cov, threads, log)
    finally:
        libc.fclose(log)
    K = _Kma.from_address(p)
    try:
        if K.status:
            raise CcgError(f"ccq_load_kma: cannot read the inputs ({K.status})")
        n, s1, s2 = K.n, K.stride1, K.stride2

        def take(ptr, count, dtype):
            return np.ctypeslib.as_array(ptr, shape=(max(count, 1),))[:count].copy().astype(dtype)
        out = {"n": n, "stride1": s1, "stride2": s2,
               "include": take(K.include, len(files), np.uint8),
               "file_of": take(K.file_of, n, np.int32),
               "rec1": take(K.rec1, n * s1 * 8, np.uint16).reshape(n, s1, 8),
               "rec2": take(K.rec2, n * s2 * 8, np.uint16).reshape(n, s2, 8),
               "len1": take(K.len1, n, np.int32), "len2": take(K.len2, n, np.int32)}
    finally:
        lib.ccq_kma_free(p)
    return out


def write_phylip(path, D, n, names, flag=1, precision=9, etype=8, byte_scale=1.0):
    """Writes a packed LT with the host writer (ccq_print_phy, ref phy.c:59)."""
    lib = host_lib()
    libc = C.CDLL(None)
    libc.fopen.restype = C.c_void_p
    libc.fopen.argtypes = [C.c_char_p, C.c_char_p]
    libc.fclose.argtypes = [C.c_void_p]
    lib.ccq_print_phy.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_char_p), C.c_void_p, C.c_char_p,
                                  C.c_uint, C.c_int]
    D = np.ascontiguousarray(D, dtype=ETYPES[etype])
    ltd = _Ltd(n, n, etype, byte_scale, D.ctypes.data if D.size else None)
    arr = (C.c_char_p * max(n, 1))(*[s.encode() for s in names])
    fp = libc.fopen(path.encode(), b"wb")
    if not fp:
        raise OSError(path)
    lib.ccq_print_phy(fp, C.byref(ltd), arr, None, None, flag, precision)
    libc.fclose(fp)
