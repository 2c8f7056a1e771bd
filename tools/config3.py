"""BASELINE configs[2]: N=50k taxa x L=5M bp synthetic alignment, dist + tree
on one MI355X, end to end in HBM (no text): packed sequences -> ccg_snp_ltd_dev
-> LT (double) -> ccg_tree_dev (DNJ).

Tree-like data: `clades` random root sequences; taxon t is the
root of clade t % clades with ~0.8% of its 2-bit codes flipped (bits set with
p = 1/256 each), so distances cluster.  The global include mask drops every
10th word (the "N columns" of config 3).

    python tools/config3.py [--n 50000] [--L 5000000] [--check]
--check compares a few LT cells with the oracle's fsacmp (host copies).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def make_packed(torch, n, W, clades=512, seed=3, chunk=1024):
    g = torch.Generator(device="cuda").manual_seed(seed)
    roots = torch.randint(-2**62, 2**62, (clades, W), dtype=torch.int64, device="cuda", generator=g)
    seqs = torch.empty((n, W), dtype=torch.int64, device="cuda")
    for t0 in range(0, n, chunk):
        t1 = min(n, t0 + chunk)
        m = torch.randint(-2**62, 2**62, (t1 - t0, W), dtype=torch.int64, device="cuda", generator=g)
        for _ in range(7):
            m &= torch.randint(-2**62, 2**62, (t1 - t0, W), dtype=torch.int64, device="cuda", generator=g)
        idx = torch.arange(t0, t1, device="cuda") % clades
        seqs[t0:t1] = roots[idx] ^ m
        del m
    del roots
    return seqs


def run(dev, torch, n=50_000, L=5_000_000, check=False, sums="fast"):
    import ccphylo_amd as cg
    W = L // 32 + 1
    t0 = time.perf_counter()
    seqs = make_packed(torch, n, W)
    incs = torch.full((W,), -1, dtype=torch.int32, device="cuda")
    incs[::10] = 0
    incs[(L + 31) // 32:] = 0
    if L % 32:
        incs[(L + 31) // 32 - 1] &= ((0xFFFFFFFF << (32 - L % 32)) & 0xFFFFFFFF) - (1 << 32)
    torch.cuda.synchronize()
    tgen = time.perf_counter() - t0
    m = n * (n - 1) // 2
    D = torch.empty(m, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    inc = dev.snp_ltd_dev(seqs.data_ptr(), incs.data_ptr(), n, L, W, D.data_ptr())
    torch.cuda.synchronize()
    tdist = time.perf_counter() - t0
    res = {"n": n, "L": L, "gen_s": round(tgen, 2), "dist_s": round(tdist, 3),
           "taxa_pairs_per_s": round(m / tdist, 1), "included_positions": inc}
    if check:
        from oracle import pyoracle
        import numpy as np
        lib = pyoracle.lib()
        hinc = incs.cpu().numpy().view(np.uint32).copy()
        bad = 0
        for (i, j) in ((1, 0), (n - 1, 0), (n - 1, n - 2), (n // 2, n // 3), (12345 % n, 77 % n)):
            if i <= j:
                continue
            a = seqs[i].cpu().numpy().view(np.uint64).copy()
            b = seqs[j].cpu().numpy().view(np.uint64).copy()
            ref = lib.orc_fsacmp(a.ctypes.data, b.ctypes.data, hinc.ctypes.data, L)
            got = float(D[i * (i - 1) // 2 + j].item())
            bad += got != ref
        res["check_mismatches"] = bad
    del seqs, incs
    torch.cuda.empty_cache()
    t0 = time.perf_counter()
    joins, fn, fd, st = dev.tree_dev(D.data_ptr(), n, method=cg.CCG_TREE_DNJ, exact=sums == "exact")
    torch.cuda.synchronize()
    ttree = time.perf_counter() - t0
    res.update({"tree_s": round(ttree, 3), "joins": len(joins), "joins_per_s": round(len(joins) / ttree, 1),
                "rows_rescanned": int(st[0]), "cells_rescanned": int(st[1]), "row_sums": sums,
                "total_s": round(tdist + ttree, 3)})
    del D
    torch.cuda.empty_cache()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50_000)
    ap.add_argument("--L", type=int, default=5_000_000)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--sums", choices=["fast", "exact"], default="fast")
    a = ap.parse_args()
    import torch
    import ccphylo_amd as cg
    dev = cg.Device(0)
    print(json.dumps(run(dev, torch, a.n, a.L, a.check, a.sums)), flush=True)


if __name__ == "__main__":
    main()
