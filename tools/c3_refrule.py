"""configs[3] (N=200k float Euclidean, the bench's matrix) DNJ rescans along
the tree: the engine's speculative rows / cells against the rows / cells the
reference's own minQpair rule rescans (dnj.c:78), counted by the engine from
its replay decisions (stats[10/11 + 2 NKSTAT]).  One JSON line per prefix.

usage: python tools/c3_refrule.py [n] [prefix,prefix,...] [float|double] [cdist]
(prefix 0: the whole tree; CCG_PROGRESS=1 prints a line per 16384 joins)
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import ccphylo_amd as cg  # noqa: E402
from ccphylo_amd import native as nt  # noqa: E402
from tools.synth import euclid_shard_dev  # noqa: E402


def heartbeat(every=40.0):
    import threading

    def beat():
        t0 = time.perf_counter()
        while True:
            time.sleep(every)
            print(f"... {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()


def main():
    heartbeat()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    prefixes = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [10_000, 30_000]
    dt_ = torch.float32 if (len(sys.argv) < 4 or sys.argv[3] == "float") else torch.float64
    legacy = len(sys.argv) > 4 and sys.argv[4] == "cdist"   # the round-4 generator (torch.cdist)
    et = 4 if dt_ == torch.float32 else 8
    dev = cg.Device(0)
    K = nt.NKSTAT
    for p in prefixes:
        loc = euclid_shard_dev(torch, n, 0, 1, dtype=dt_, cdist=legacy)
        torch.cuda.synchronize()
        t = time.perf_counter()
        j, fn, fd, st = dev.tree_dev(loc.data_ptr(), n, etype=et, method=cg.CCG_TREE_DNJ, exact=True, profile=True,
                                     max_joins=p)
        dt = time.perf_counter() - t
        del loc
        torch.cuda.empty_cache()
        per = {name: round(st[5 + 2 * c] / 1e9, 3) for c, name in enumerate(nt.KSTAT_NAMES) if st[4 + 2 * c]}
        print(json.dumps({"n": n, "etype": et, "generator": "torch.cdist (round 4)" if legacy else "elementwise",
                          "joins": len(j), "seconds": round(dt, 2),
                          "engine_rows": int(st[0]), "engine_cells": int(st[1]),
                          "reference_rule_rows": int(st[10 + 2 * K]), "reference_rule_cells": int(st[11 + 2 * K]),
                          "engine_over_reference_cells": round(st[1] / max(1, st[11 + 2 * K]), 3),
                          "kernel_s": per}), flush=True)


if __name__ == "__main__":
    main()
