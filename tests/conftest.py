"""Shared fixtures.  `-m gpu` tests need an MI355X (gfx950); everything else
runs on CPU (oracle vs golden vectors, host layer, C-ABI symbol checks)."""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


def ensure_built():
    need = [os.path.join(ROOT, "ccphylo_amd", "lib", "libccphylo_host.so"),
            os.path.join(ROOT, "ccphylo_amd", "lib", "libccphylo_amd.so"),
            os.path.join(ROOT, "ccphylo_amd", "bin", "ccphylo"),
            os.path.join(ROOT, "oracle", "_build", "liboracle.so")]
    if not all(os.path.exists(p) for p in need):
        import __graft_entry__
        __graft_entry__.build()


@pytest.fixture(scope="session", autouse=True)
def _built():
    ensure_built()


@pytest.fixture(scope="session", autouse=True)
def _heartbeat(request):
    """GPU sessions: a line every 30 s in gpurun_out/pytest_heartbeat.log
    naming the running test, so that a long test (the configs[3] world-8
    rehearsal runs minutes with its output captured) is not taken for a hung
    run by a watchdog that watches the run's output files."""
    import threading
    import time
    if "gpu" not in (request.config.getoption("-m") or "") or "not gpu" in (request.config.getoption("-m") or ""):
        yield
        return
    path = os.path.join(ROOT, "gpurun_out", "pytest_heartbeat.log")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    stop = threading.Event()
    t0 = time.time()

    def beat():
        while not stop.wait(30.0):
            with open(path, "a") as f:
                f.write(f"{time.time() - t0:.0f} s {os.environ.get('PYTEST_CURRENT_TEST', '')}\n")
    th = threading.Thread(target=beat, daemon=True)
    th.start()
    yield
    stop.set()


def golden_cases(kind=None):
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        cases = json.load(f)["cases"]
    return [c for c in cases if kind is None or c["kind"] == kind]


def golden_bytes(case):
    with open(os.path.join(GOLDEN, case["out"]), "rb") as f:
        return f.read()


def parse_tree_args(args):
    """tree CLI args of a golden case -> (input, method, etype, bs, flags, precision)."""
    inp, method, et, bs, flags, prec = None, 1, 8, 1.0, 0, 9
    k = 1
    while k < len(args):
        a = args[k]
        if a == "-i":
            inp = args[k + 1]; k += 1
        elif a == "-m":
            method = {"nj": 0, "dnj": 1, "hnj": 2}[args[k + 1]]; k += 1
        elif a == "-p":
            et = 4
        elif a in ("-s", "-b"):
            et = 2 if a == "-s" else 1
            if k + 1 < len(args) and not args[k + 1].startswith("-"):
                bs = float(args[k + 1]); k += 1
        elif a == "-f":
            flags = int(args[k + 1]); k += 1
        elif a == "-x":
            prec = int(args[k + 1]); k += 1
        k += 1
    return os.path.join(GOLDEN, inp), method, et, bs, flags, prec


def print_phylip(D, n, names, flag, precision, etype=8, bs=1.0, include=None, comment=None):
    """Formats a packed LT with the product host writer (ccq_print_phy).
    `include` (one flag per name) selects the printed names; `comment` is
    the '#' line of format flag 4 (the template name)."""
    import tempfile
    from ccphylo_amd import native
    lib = native.host_lib()
    libc = C.CDLL(None)
    libc.fopen.restype = C.c_void_p
    libc.fopen.argtypes = [C.c_char_p, C.c_char_p]
    libc.fclose.argtypes = [C.c_void_p]
    lib.ccq_print_phy.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_char_p), C.c_void_p, C.c_char_p,
                                  C.c_uint, C.c_int]
    ltd = native._Ltd(n, n, etype, bs, D.ctypes.data if D.size else None)
    arr = (C.c_char_p * max(len(names), 1))(*[s.encode() for s in names])
    inc = None
    if include is not None:
        inc = np.ascontiguousarray(include, dtype=np.uint8)
    with tempfile.NamedTemporaryFile(delete=False) as t:
        path = t.name
    fp = libc.fopen(path.encode(), b"wb")
    lib.ccq_print_phy(fp, C.byref(ltd), arr, inc.ctypes.data if inc is not None else None,
                      comment.encode() if comment is not None else None, flag, precision)
    libc.fclose(fp)
    with open(path, "rb") as f:
        data = f.read()
    os.unlink(path)
    return data


def parse_dist_args(args):
    """dist CLI args of a golden case -> dict."""
    o = dict(inp=None, flag=1, norm=0, minLength=1, minCov=0.5, proxi=0, et=8, bs=1.0, prec=9, nout=False)
    k = 1
    while k < len(args):
        a = args[k]
        nxt = args[k + 1] if k + 1 < len(args) else None
        if a == "-i": o["inp"] = os.path.join(GOLDEN, nxt); k += 1
        elif a == "-f": o["flag"] = int(nxt); k += 1
        elif a == "-W": o["norm"] = int(nxt); k += 1
        elif a == "-L": o["minLength"] = int(nxt); k += 1
        elif a == "-C": o["minCov"] = float(nxt) / 100; k += 1
        elif a == "-P": o["proxi"] = int(nxt); k += 1
        elif a == "-x": o["prec"] = int(nxt); k += 1
        elif a == "-n": o["nout"] = True; k += 1
        elif a == "-p": o["et"] = 4
        elif a in ("-s", "-b"):
            o["et"] = 2 if a == "-s" else 1
            if nxt is not None and not nxt.startswith("-"):
                o["bs"] = float(nxt); k += 1
        k += 1
    return o


def parse_kma_args(args):
    """dist CLI args of a KMA (*.mat) golden case -> dict (dist.c:508-690 option meanings)."""
    o = dict(files=[], tmpl=None, metric="cos", flag=1, norm=0, minDepth=15, minLength=1, minCov=0.5, et=8, bs=1.0,
             prec=9, nout=False)
    k = 1
    while k < len(args):
        a = args[k]
        nxt = args[k + 1] if k + 1 < len(args) else None
        if a == "-i":
            while k + 1 < len(args) and not args[k + 1].startswith("-"):
                o["files"].append(os.path.join(GOLDEN, args[k + 1]))
                k += 1
        elif a == "-r": o["tmpl"] = nxt; k += 1
        elif a == "-d": o["metric"] = nxt; k += 1
        elif a == "-f": o["flag"] = int(nxt); k += 1
        elif a == "-W": o["norm"] = int(nxt); k += 1
        elif a == "-E": o["minDepth"] = int(float(nxt)); k += 1
        elif a == "-L": o["minLength"] = int(nxt); k += 1
        elif a == "-C": o["minCov"] = float(nxt) / 100; k += 1
        elif a == "-x": o["prec"] = int(nxt); k += 1
        elif a == "-n": o["nout"] = True; k += 1
        elif a == "-p": o["et"] = 4
        elif a in ("-s", "-b"):
            o["et"] = 2 if a == "-s" else 1
            if nxt is not None and not nxt.startswith("-"):
                o["bs"] = float(nxt); k += 1
        k += 1
    return o
