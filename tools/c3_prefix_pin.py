"""configs[3]'s 200k float matrix from either generator: the engine's first K
exact DNJ joins against the oracle's serial-decision DNJ (dnj.c:985-1052,
threaded rescans) on the same LT, with the reference-rule counters of both
(test infrastructure: the oracle is the checker).  One JSON line.

    python tools/c3_prefix_pin.py [n] [K] [elementwise|cdist] [threads]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    import ccphylo_amd as cg
    from oracle import pyoracle
    from tools.synth import euclid_shard_dev
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    gen = sys.argv[3] if len(sys.argv) > 3 else "cdist"
    threads = int(sys.argv[4]) if len(sys.argv) > 4 else 16
    loc = euclid_shard_dev(torch, n, 0, 1, dtype=torch.float32, cdist=gen == "cdist")
    host = loc.cpu().numpy()
    dev = cg.Device(0)
    t0 = time.perf_counter()
    j, fn, fd, st = dev.tree_dev(loc.data_ptr(), n, etype=4, method=cg.CCG_TREE_DNJ, exact=True, max_joins=k,
                                 profile=True)
    tg = time.perf_counter() - t0
    del loc
    torch.cuda.empty_cache()
    K = cg.native.NKSTAT
    print(json.dumps({"stage": "engine done", "seconds": round(tg, 2)}), flush=True)
    t0 = time.perf_counter()
    rj, rfn, rfd, rst = pyoracle.tree(host, n, etype=4, method=cg.CCG_TREE_DNJ, max_joins=k, threads=threads,
                                      copy=False, stats=True)
    to = time.perf_counter() - t0
    first_diff = None
    m = min(len(j), len(rj))
    for name in ("i", "j", "Li", "Lj"):
        bad = np.nonzero(j[name][:m] != rj[name][:m])[0]
        if len(bad) and (first_diff is None or bad[0] < first_diff):
            first_diff = int(bad[0])
    print(json.dumps({"n": n, "generator": gen, "joins": m, "joins_identical": first_diff is None and len(j) == len(rj),
                      "first_differing_join": first_diff,
                      "engine_reference_rule_rows_cells": [int(st[10 + 2 * K]), int(st[11 + 2 * K])],
                      "oracle_rows_cells": [int(rst[0]), int(rst[1])],
                      "engine_s": round(tg, 2), "oracle_s": round(to, 1), "oracle_threads": threads}), flush=True)


if __name__ == "__main__":
    main()
