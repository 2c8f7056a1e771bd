"""configs[3] on one GPU (development aid): DNJ on one N=200k Euclidean float
matrix with the single-GPU engine, join prefixes of growing length, so the
cost per join along the tree shows where time goes.

    python tools/perf_c3.py [N] [prefix ...] [--fast] [--shard]

Prints one JSON line per prefix: seconds, rows / cells rescanned, the
exact-sum counters (stats[6+2N] serial-order sums, [7+2N] by the chain),
and per kernel class the HIP-event time (a profiled run)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import ccphylo_amd as cg  # noqa: E402
from ccphylo_amd import native as nt  # noqa: E402
from tools.synth import euclid_shard_dev  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
n = int(args[0]) if args else 200_000
prefixes = [int(x) for x in args[1:]] or [20_000, 60_000, 120_000]
exact = "--fast" not in sys.argv
if "--shard" in sys.argv:
    os.environ["CCG_SHARD_FORCE"] = "1"
dev = cg.Device(0)
N = nt.NKSTAT
for k in prefixes:
    loc = euclid_shard_dev(torch, n, 0, 1, dtype=torch.float32)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    j, fn, fd, st = dev.tree_shard_dev(loc.data_ptr(), n, None, etype=4, method=cg.CCG_TREE_DNJ, exact=exact,
                                       max_joins=k, profile=True)
    dt = time.perf_counter() - t0
    del loc
    torch.cuda.empty_cache()
    cls = {nt.KSTAT_NAMES[c]: round(st[5 + 2 * c] / 1e9, 3) for c in range(N) if st[4 + 2 * c]}
    import hashlib
    h = hashlib.sha256(j.tobytes()).hexdigest()[:12]
    print(json.dumps({"n": n, "joins": len(j), "seconds": round(dt, 2), "exact": exact, "sha": h,
                      "rows": int(st[0]), "cells": int(st[1]), "serial_sums": int(st[6 + 2 * N]),
                      "chain_sums": int(st[7 + 2 * N]), "class_s": cls}), flush=True)
