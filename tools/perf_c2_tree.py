"""The headline's DNJ tree (configs[2]: the 50k x 5 Mbp tree-like alignment
through the GPU dist) timed under several engine settings, one matrix:

    python tools/perf_c2_tree.py [--n 50000] [--joins 0] "CCG_SCAN_PRUNE=0" "" "CCG_S_BANDS=112" ...

Each argument is a space-separated list of environment settings (empty: the
defaults).  The LT is computed once, kept on the host and copied back for
every run; the joins' sha256 must agree across settings."""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50_000)
    ap.add_argument("--L", type=int, default=5_000_000)
    ap.add_argument("--joins", type=int, default=0)
    ap.add_argument("--joins-list", default="", help="comma-separated join prefixes, each timed under every setting")
    ap.add_argument("--exact", type=int, default=1)
    ap.add_argument("settings", nargs="*")
    a = ap.parse_args()
    import torch
    import ccphylo_amd as cg
    from bench import make_headline_alignment
    K = cg.native.NKSTAT
    n, L = a.n, a.L
    dev = cg.Device(0)
    seqs, incs, W = make_headline_alignment(torch, n, L)
    Dd = torch.empty(n * (n - 1) // 2, dtype=torch.float64, device="cuda")
    dev.snp_ltd_dev(seqs.data_ptr(), incs.data_ptr(), n, L, W, Dd.data_ptr())
    torch.cuda.synchronize()
    del seqs, incs
    torch.cuda.empty_cache()
    host = Dd.cpu()
    runs = [(s_, int(jl)) for jl in (a.joins_list.split(",") if a.joins_list else [a.joins])
            for s_ in (a.settings or [""])]
    for st_, max_joins in runs:
        env = dict(kv.split("=", 1) for kv in st_.split())
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        Dd.copy_(host)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        j, fn, fd, st = dev.tree_dev(Dd.data_ptr(), n, method=cg.CCG_TREE_DNJ, exact=bool(a.exact),
                                     max_joins=max_joins, profile=True)
        dt = time.perf_counter() - t0
        kern = {name: round(st[5 + 2 * c] / 1e3 / max(len(j), 1), 2)
                for c, name in enumerate(["init", "top", "scan", "argmin", "update", "requeue", "pop", "plan",
                                          "coll", "xsum"]) if st[4 + 2 * c]}
        print(json.dumps({"settings": st_ or "defaults", "joins": len(j), "tree_s": round(dt, 3),
                          "joins_per_s": round(len(j) / dt, 1),
                          "joins_sha": hashlib.sha256(j.tobytes()).hexdigest()[:16],
                          "rows": st[0], "cells": st[1], "ref_rows": st[10 + 2 * K], "ref_cells": st[11 + 2 * K],
                          "engine_over_reference_cells": round(st[1] / max(st[11 + 2 * K], 1), 3),
                          "us_per_join_by_class": kern}), flush=True)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


if __name__ == "__main__":
    main()
