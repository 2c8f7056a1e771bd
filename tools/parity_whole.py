"""Whole-tree DNJ parity at configs[2]'s size (n = 50k, the large-n engine:
band rows of S, k_dnj_fold chunk summaries, k_dnj_join_pf, the 16-byte
nontemporal wave scan), split over two machines: the GPU box builds the tree,
this container runs the oracle (oracle/ccoracle.c, the reference's serial
minQpair / exact row sums; test infrastructure only) on the same matrix.

The matrix is generated deterministically by numpy on both sides (Euclidean
distances of U[0,1)^8 points, seed 11, `--kind int`: times 5000 and rounded
to integers, SNP-count-like with many ties; `--kind euc`: 9 decimals), and
its sha256 is compared.

    python tools/parity_whole.py --gpu gpurun_out/pw.npz [--n 50000] [--kind int]   (GPU box)
    python tools/parity_whole.py --oracle gpurun_out/pw.npz                       (here)
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def matrix(n, kind, seed=11, threads=16):
    from concurrent.futures import ThreadPoolExecutor
    rng = np.random.default_rng(seed)
    pts = rng.random((n, 8))
    D = np.empty(n * (n - 1) // 2)

    def rows(r0, r1):   # row by row, the same arithmetic in any thread
        for i in range(max(r0, 1), r1):
            o = i * (i - 1) // 2
            d = np.sqrt(((pts[:i] - pts[i]) ** 2).sum(1))
            D[o:o + i] = np.rint(d * 5000.0) if kind == "int" else np.round(d * 1e9) / 1e9
    step = 512
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda r: rows(r, min(n, r + step)), range(0, n, step)))
    return D


def sha(D):
    return hashlib.sha256(D.view(np.uint8)).hexdigest()[:16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpu")
    ap.add_argument("--oracle")
    ap.add_argument("--n", type=int, default=50_000)
    ap.add_argument("--kind", default="int", choices=["int", "euc"])
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    import ccphylo_amd as cg
    if a.gpu:
        D = matrix(a.n, a.kind)
        dev = cg.Device(0)
        t0 = time.perf_counter()
        j, fn, fd, st = dev.tree(D, a.n, method=cg.CCG_TREE_DNJ, exact=True, profile=True)
        dt = time.perf_counter() - t0
        K = cg.native.NKSTAT
        np.savez(a.gpu, joins=j, fn=fn, fd=fd, n=a.n, kind=a.kind, sha=sha(D), seconds=dt,
                 ref_rows=st[10 + 2 * K], ref_cells=st[11 + 2 * K], rows=st[0], cells=st[1])
        print(json.dumps({"n": a.n, "kind": a.kind, "joins": len(j), "seconds": round(dt, 2), "sha": sha(D)}))
        return
    z = np.load(a.oracle)
    n, kind = int(z["n"]), str(z["kind"])
    D = matrix(n, kind)
    assert sha(D) == str(z["sha"]), "the two sides generated different matrices"
    from oracle import pyoracle
    t0 = time.perf_counter()
    rj, rfn, rfd, rst = pyoracle.tree(D, n, method=cg.CCG_TREE_DNJ, stats=True, threads=a.threads, copy=False)
    dt = time.perf_counter() - t0
    gj = z["joins"]
    same_ij = len(gj) == len(rj) and bool(((gj["i"] == rj["i"]) & (gj["j"] == rj["j"])).all())
    same_len = same_ij and bool(((gj["Li"] == rj["Li"]) & (gj["Lj"] == rj["Lj"])).all())
    out = {"n": n, "kind": kind, "matrix_sha256": str(z["sha"]), "joins": len(gj), "oracle_joins": len(rj),
           "joins_identical": same_ij, "branch_lengths_identical": same_len,
           "final_identical": (int(z["fn"]), float(z["fd"])) == (rfn, rfd),
           "engine_reference_rule_rows_cells": [int(z["ref_rows"]), int(z["ref_cells"])],
           "oracle_rows_cells": [int(rst[0]), int(rst[1])],
           "counters_equal": (int(z["ref_rows"]), int(z["ref_cells"])) == (int(rst[0]), int(rst[1])),
           "engine_rows_cells": [int(z["rows"]), int(z["cells"])],
           "gpu_tree_s": round(float(z["seconds"]), 2), "oracle_s": round(dt, 1)}
    if not same_ij:
        bad = np.nonzero((gj["i"][:len(rj)] != rj["i"][:len(gj)]) | (gj["j"][:len(rj)] != rj["j"][:len(gj)]))[0]
        out["first_differing_join"] = int(bad[0]) if bad.size else None
    print(json.dumps(out))


if __name__ == "__main__":
    main()
