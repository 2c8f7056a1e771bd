"""CPU: the C-ABI libraries load and export every symbol their headers
declare; the engine fails loudly (no CPU fallback) without a gfx950 GPU."""
import os
import re
import subprocess

import pytest

from conftest import GOLDEN, ROOT

NO_GPU = not os.path.exists("/dev/kfd")


def header_functions(name):
    with open(os.path.join(ROOT, "include", name)) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*[A-Za-z_][\w\s\*]*?\b(cc[gq]_\w+)\s*\(", src, flags=re.M)))


def exported(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if ln.strip()}


def test_engine_exports_every_header_symbol():
    from ccphylo_amd import native
    decl = header_functions("ccphylo_amd.h")
    assert decl, "no declarations parsed"
    assert sorted(decl) == sorted(native.ENGINE_SYMBOLS)
    missing = set(decl) - exported(native.ENGINE_PATH)
    assert not missing, missing


def test_host_exports_every_header_symbol():
    from ccphylo_amd import native
    decl = header_functions("ccphylo_host.h")
    assert decl
    assert sorted(decl) == sorted(native.HOST_SYMBOLS)
    missing = set(decl) - exported(native.HOST_PATH)
    assert not missing, missing


def test_engine_lib_loads_and_strerror():
    from ccphylo_amd import native
    lib = native.engine_lib()
    for code, text in ((0, b"success"), (-1, b"invalid argument"), (-2, b"no gfx950"), (-5, b"not supported")):
        assert text in lib.ccg_strerror(code)


def test_stats_layout_matches_header():
    from ccphylo_amd import native
    with open(os.path.join(ROOT, "include", "ccphylo_amd.h")) as f:
        h = f.read()
    assert int(re.search(r"#define CCG_NKSTAT\s+(\d+)", h).group(1)) == native.NKSTAT == len(native.KSTAT_NAMES)


@pytest.mark.skipif(not NO_GPU, reason="checks the no-GPU behaviour")
def test_no_cpu_fallback_engine():
    import ctypes as C
    from ccphylo_amd import native
    lib = native.engine_lib()
    ctx = C.c_void_p()
    assert lib.ccg_init(0, C.byref(ctx)) == -2   # CCG_ENODEV
    with pytest.raises(native.CcgError):
        native.Device(0)


@pytest.mark.skipif(not NO_GPU, reason="checks the no-GPU behaviour")
def test_no_cpu_fallback_cli():
    from ccphylo_amd import native
    p = subprocess.run([native.CLI_PATH, "tree", "-i", "test.phy.gz"], cwd=GOLDEN, capture_output=True, timeout=60)
    assert p.returncode != 0
    assert b"gfx950" in p.stderr or b"GPU" in p.stderr
    assert p.stdout == b""


def test_cli_refuses_out_of_scope_options():
    from ccphylo_amd import native
    for args in (["tree", "-i", "test.phy.gz", "-m", "upgma"], ["dist", "-i", "msa64.fsa", "-V", "x"]):
        p = subprocess.run([native.CLI_PATH] + args, cwd=GOLDEN, capture_output=True, timeout=60)
        assert p.returncode != 0, args
        assert b"not implemented" in p.stderr or b"not supported" in p.stderr, (args, p.stderr)
