"""CPU: rows A1-A3 of SURVEY 8(a) in isolation -- the product host layer's code
table (fsacmp.c:32 get2BitTable), 2-bit packing (qseqs.c:60 qseq2nibble) and
include masks (fsacmp.c:164 initIncPos / :181 getIncPos) against known-answer
vectors written out by hand from the reference's rules, and against the
oracle's restatement on random sequences (SURVEY 8(c) golden item (v))."""
import ctypes as C

import numpy as np
import pytest


@pytest.fixture(scope="module")
def libs():
    import ccphylo_amd as cg
    from oracle import pyoracle
    h = cg.host_lib()
    h.ccq_code_table.argtypes = [C.c_uint, C.c_void_p]
    h.ccq_pack.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    h.ccq_pack.restype = C.c_int
    h.ccq_init_inc.argtypes = [C.c_void_p, C.c_int]
    h.ccq_inc_update.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_uint, C.c_int]
    h.ccq_npos.argtypes = [C.c_void_p, C.c_int]
    h.ccq_npos.restype = C.c_int
    o = pyoracle.lib()
    return h, o


def _table(lib, fn, flag):
    t = np.zeros(256, np.uint8)
    getattr(lib, fn)(flag, t.ctypes.data)
    return t


@pytest.mark.parametrize("flag", [1, 9, 33, 3])
def test_code_table_known_answers(libs, flag):
    h, o = libs
    t = _table(h, "ccq_code_table", flag)
    for ch, v in zip("ACGTU", (0, 1, 2, 3, 3)):
        assert t[ord(ch)] == v
    for ch in "N-RYKMSWBDHV":
        assert t[ord(ch)] == 4
    low = [t[ord(c)] for c in "acgtu"]
    assert low == ([0, 1, 2, 3, 3] if flag & 8 else [4] * 5)   # lowercase only with flag 8
    for ch in "\r\t 0*>":
        assert t[ord(ch)] == 32                                # dropped by FileBuffgetFsa
    assert (t == _table(o, "orc_code_table", flag)).all()


def test_pack_known_answers(libs):
    h, _ = libs
    # ACGT -> 00 01 10 11 in the top byte, MSB first; code 4 packs as 00
    codes = np.array([0, 1, 2, 3], np.uint8)
    out = np.zeros(2, np.uint64)
    assert h.ccq_pack(codes.ctypes.data, 4, out.ctypes.data) == 0
    assert int(out[0]) == 0x1B << 56
    codes = np.array([4, 3, 4, 1] + [2] * 30, np.uint8)    # 34 positions: a second, left-aligned word
    out = np.zeros(3, np.uint64)
    assert h.ccq_pack(codes.ctypes.data, 34, out.ctypes.data) == 2
    w0 = 0
    for p, c in enumerate(codes[:32]):
        w0 |= (int(c) & 3) << (62 - 2 * p)
    assert int(out[0]) == w0
    assert int(out[1]) == (2 << 62) | (2 << 60)


@pytest.mark.parametrize("L", [1, 31, 32, 33, 1000, 4097])
def test_pack_and_masks_vs_oracle(libs, L):
    h, o = libs
    rng = np.random.default_rng(L)
    W = L // 32 + 1
    ref = rng.choice(np.array([0, 1, 2, 3, 4], np.uint8), size=L, p=[0.24, 0.24, 0.24, 0.24, 0.04])
    for proxi in (0, 1, 5, 40):
        for variant in (0, 8, 32):
            mh = np.zeros(W + 2, np.uint32)
            mo = np.zeros(W + 2, np.uint32)
            h.ccq_init_inc(mh[1:].ctypes.data, L)
            o.orc_init_inc(mo[1:].ctypes.data, L)
            assert (mh == mo).all()
            for t in range(4):
                seq = ref.copy()
                flip = rng.random(L) < 0.05
                seq[flip] = rng.choice(np.array([0, 1, 2, 3, 4, 16 | 1], np.uint8), size=int(flip.sum()))
                ph, po = np.zeros(W, np.uint64), np.zeros(W, np.uint64)
                s4 = (seq & 0x0F).astype(np.uint8)
                s4[s4 > 4] = 4
                assert h.ccq_pack(s4.ctypes.data, L, ph.ctypes.data) == o.orc_pack(s4.ctypes.data, L, po.ctypes.data)
                assert (ph == po).all()
                # mask word -1 is the reference's include[-1] (a first SNP with lastSNP = -1)
                # both strip the insignificance bit (16) from seq and ref in place
                sh, rh, so, ro = seq.copy(), ref.copy(), seq.copy(), ref.copy()
                h.ccq_inc_update(mh[1:].ctypes.data, sh.ctypes.data, rh.ctypes.data, L, proxi, variant)
                o.orc_inc_update(mo[1:].ctypes.data, so.ctypes.data, ro.ctypes.data, L, proxi, variant)
                assert (mh == mo).all() and (sh == so).all() and (rh == ro).all(), (proxi, variant, t)
            assert h.ccq_npos(mh[1:].ctypes.data, L) == o.orc_npos(mo[1:].ctypes.data, L)
            # tail bits past L stay zero (fsacmp.c:164)
            if L % 32:
                assert int(mh[1 + L // 32]) & ((1 << (32 - L % 32)) - 1) == 0
