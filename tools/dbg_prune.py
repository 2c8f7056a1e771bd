"""Development aid: which DNJ scan configurations reproduce the serial
reference on one matrix (first differing join), for narrowing a parity
failure to a kernel form.  python tools/dbg_prune.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import ccphylo_amd as cg  # noqa: E402
from oracle import pyoracle  # noqa: E402
from test_gpu import _clade_ltd, _euclid  # noqa: E402

dev = cg.Device(0)
base = {"CCG_PREFOLD_N": "0", "CCG_SEG_MUL": "1", "CCG_S_SPLIT_N": "100", "CCG_S_BANDS": "64"}
for kind, n, et in (("clade", 2600, 4), ("clade", 2600, 8), ("euc", 2200, 4)):
    D = _clade_ltd(n, n + 4) if kind == "clade" else _euclid(n, n + 3)
    if et == 4:
        D = D.astype(np.float32)
    ref = pyoracle.tree(D, n, etype=et, method=1)
    for mode in ("20", "21", "9", "4"):
        for prune in ("1", "0"):
            for fold in ("1", "0"):
                os.environ.update(base)
                os.environ.update({"CCG_SCAN_WAVE": mode, "CCG_SCAN_PRUNE": prune, "CCG_SCAN_FOLD": fold})
                got = dev.tree(D, n, etype=et, method=1, exact=True, profile=True)
                j = got[0]
                bad = np.nonzero((j["i"] != ref[0]["i"][:len(j)]) | (j["j"] != ref[0]["j"][:len(j)]))[0] \
                    if len(j) == len(ref[0]) else [-1]
                print(kind, n, et, "mode", mode, "prune", prune, "fold", fold,
                      "OK" if len(bad) == 0 and got[1:3] == ref[1:3] else f"FIRST BAD {bad[0] if len(bad) else 'final'}",
                      "cells", got[3][1], flush=True)
