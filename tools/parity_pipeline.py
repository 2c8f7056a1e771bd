"""Whole-pipeline parity at configs[2]'s taxon count: `ccphylo dist` -> `tree`
on a clade-structured alignment (the headline's kind of data: integer SNP
counts with many exact Q ties), split over two machines.

The GPU box runs the product path, HBM-resident end to end: the packed
alignment -> ccg_snp_ltd_dev (non-pair, double LT) -> ccg_tree_dev (exact
DNJ, the whole tree).  This container runs the oracle (oracle/ccoracle.c,
test infrastructure only: fsacmp.c:552 per cell, then the serial
DNJ of dnj.c:985 with its minQpair decisions) on the same input.  Both sides
generate the alignment with numpy (tools/synth.clade_packed, fixed seed); the
packed input's and the LT's sha256 are compared, then every join, branch
length, the final pair and the reference-rule rescan counters.

    python tools/parity_pipeline.py --gpu gpurun_out/pp.npz [--n 50000] [--L 20000]   (GPU box)
    python tools/parity_pipeline.py --oracle gpurun_out/pp.npz [--threads 8]          (here)
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint8)).hexdigest()[:16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpu")
    ap.add_argument("--oracle")
    ap.add_argument("--n", type=int, default=50_000)
    ap.add_argument("--L", type=int, default=20_000)
    ap.add_argument("--clades", type=int, default=512)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    import ccphylo_amd as cg
    from tools.synth import clade_packed
    if a.gpu:
        import torch
        n, L = a.n, a.L
        seqs, incs = clade_packed(n, L, a.clades, a.seed)
        W = seqs.shape[1]
        dev = cg.Device(0)
        S = torch.from_numpy(seqs.view(np.int64)).cuda()
        I = torch.from_numpy(incs.view(np.int32)).cuda()
        D = torch.empty(n * (n - 1) // 2, dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        inc = dev.snp_ltd_dev(S.data_ptr(), I.data_ptr(), n, L, W, D.data_ptr())
        torch.cuda.synchronize()
        tdist = time.perf_counter() - t0
        del S, I
        dsha = sha(D.cpu().numpy())
        t0 = time.perf_counter()
        j, fn, fd, st = dev.tree_dev(D.data_ptr(), n, method=cg.CCG_TREE_DNJ, exact=True, profile=True)
        ttree = time.perf_counter() - t0
        K = cg.native.NKSTAT
        np.savez(a.gpu, joins=j, fn=fn, fd=fd, n=n, L=L, clades=a.clades, seed=a.seed, inc=inc,
                 input_sha=sha(seqs) + sha(incs), ltd_sha=dsha, dist_s=tdist, tree_s=ttree,
                 ref_rows=st[10 + 2 * K], ref_cells=st[11 + 2 * K], rows=st[0], cells=st[1])
        print(json.dumps({"n": n, "L": L, "joins": len(j), "dist_s": round(tdist, 2), "tree_s": round(ttree, 2),
                          "ltd_sha": dsha}), flush=True)
        return
    from oracle import pyoracle
    z = np.load(a.oracle)
    n, L = int(z["n"]), int(z["L"])
    seqs, incs = clade_packed(n, L, int(z["clades"]), int(z["seed"]))
    assert sha(seqs) + sha(incs) == str(z["input_sha"]), "the two sides generated different alignments"
    t0 = time.perf_counter()
    D, _, inc = pyoracle.snp_ltd(seqs, incs, n, L, threads=a.threads)
    t_dist = time.perf_counter() - t0
    del seqs
    dsha = sha(D)
    out = {"n": n, "L": L, "clades": int(z["clades"]), "included_positions": [int(z["inc"]), int(inc)],
           "ltd_sha256": [str(z["ltd_sha"]), dsha], "ltd_identical": dsha == str(z["ltd_sha"])}
    t0 = time.perf_counter()
    rj, rfn, rfd, rst = pyoracle.tree(D, n, method=cg.CCG_TREE_DNJ, stats=True, threads=a.threads, copy=False)
    t_tree = time.perf_counter() - t0
    gj = z["joins"]
    same_ij = len(gj) == len(rj) and bool(((gj["i"] == rj["i"]) & (gj["j"] == rj["j"])).all())
    same_len = same_ij and bool(((gj["Li"] == rj["Li"]) & (gj["Lj"] == rj["Lj"])).all())
    out.update({"joins": len(gj), "oracle_joins": len(rj), "joins_identical": same_ij,
                "branch_lengths_identical": same_len,
                "final_identical": (int(z["fn"]), float(z["fd"])) == (rfn, rfd),
                "engine_reference_rule_rows_cells": [int(z["ref_rows"]), int(z["ref_cells"])],
                "oracle_rows_cells": [int(rst[0]), int(rst[1])],
                "counters_equal": (int(z["ref_rows"]), int(z["ref_cells"])) == (int(rst[0]), int(rst[1])),
                "engine_rows_cells": [int(z["rows"]), int(z["cells"])],
                "gpu_dist_s": round(float(z["dist_s"]), 2), "gpu_tree_s": round(float(z["tree_s"]), 2),
                "oracle_dist_s": round(t_dist, 1), "oracle_tree_s": round(t_tree, 1), "oracle_threads": a.threads})
    if not same_ij:
        bad = np.nonzero((gj["i"][:len(rj)] != rj["i"][:len(gj)]) | (gj["j"][:len(rj)] != rj["j"][:len(gj)]))[0]
        out["first_differing_join"] = int(bad[0]) if bad.size else None
    print(json.dumps(out))


if __name__ == "__main__":
    main()
