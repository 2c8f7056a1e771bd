"""Parity at sizes beyond the test suite (one-off evidence, not a test): DNJ
and HNJ on an N-taxon Euclidean matrix (configs[1]'s data, default N=30000)
on the GPU, exact and fast row sums, against the oracle's serial restatement
(oracle/ccoracle.c, test infrastructure) on the host.  Reports whether the
join lists (topology and order) are identical and the largest relative
branch-length difference.

    python tools/parity_large.py [N]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def splits(joins, n, final_n):
    """Unrooted splits of the tree a join list builds (rows j/i merged into row
    j, the last row moved to i, as dnj.c:1014-1024), as rooting-invariant
    hashes: a clade is the sum of its leaves' random 64-bit keys, normalised
    to min(h, total - h)."""
    rng = np.random.default_rng(12345)
    keys = rng.integers(1, 2 ** 62, size=n, dtype=np.uint64)
    total = int(keys.astype(object).sum()) % (1 << 64)
    rows = [int(k) for k in keys]
    m = n
    out = set()
    for J in joins:
        i, j = int(J["i"]), int(J["j"])
        h = (rows[j] + rows[i]) % (1 << 64)
        rows[j] = h
        m -= 1
        rows[i] = rows[m]
        out.add(min(h, (total - h) % (1 << 64)))
    return out


def main():
    import ccphylo_amd as cg
    from oracle import pyoracle
    from tools.synth import euclid
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 30000
    D = euclid(n, 1)
    dev = cg.Device(0)
    out = {"n": n, "data": "Euclidean U[0,1)^8 (seed 1), %.9f-quantized", "methods": {}}
    for method, name in ((cg.CCG_TREE_DNJ, "dnj"), (cg.CCG_TREE_HNJ, "hnj")):
        t0 = time.perf_counter()
        ref, rfn, rfd = pyoracle.tree(D, n, method=method)
        tref = time.perf_counter() - t0
        res = {"oracle_s": round(tref, 2)}
        for exact in (True, False):
            t0 = time.perf_counter()
            got, fn, fd, _ = dev.tree(D, n, method=method, exact=exact)
            tg = time.perf_counter() - t0
            same = len(got) == len(ref) and bool((got["i"] == ref["i"]).all() and (got["j"] == ref["j"]).all())
            rel = 0.0
            if same:
                for f in ("Li", "Lj"):
                    nz = np.abs(ref[f]) > 0
                    if nz.any():
                        rel = max(rel, float((np.abs(got[f] - ref[f])[nz] / np.abs(ref[f])[nz]).max()))
            sp_ref, sp_got = splits(ref, n, rfn), splits(got, n, fn)
            res["exact" if exact else "fast"] = {
                "joins_identical": same, "topology_identical": sp_ref == sp_got,
                "splits_differing": len(sp_ref ^ sp_got) // 2, "bit_identical": same and bool((got == ref).all()) and (fn, fd) == (rfn, rfd),
                "max_rel_length_diff": rel, "gpu_wall_s": round(tg, 3)}
        out["methods"][name] = res
        print(json.dumps({name: res}), flush=True)
    dev.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
