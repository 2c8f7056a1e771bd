"""The row-sharded DNJ's per-join device cost by kernel class (the input of
DESIGN.md §6's configs[4] projection): configs[3]'s 200k float Euclidean
matrix (tools/synth, seed 4) through ccg_tree_shard_dev's sharded kernels at
world 1 (CCG_SHARD_FORCE=1: the band layout is the packed LT, the
collectives are the self transport's copies), profiled (HIP events between
the kernel classes on the engine stream), over join prefixes.  One JSON line
per prefix: us per join by class, engine cells per join.

    python tools/shard_cost.py [n] [prefix,prefix,...]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    prefixes = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "2000,20000").split(",")]
    os.environ["CCG_SHARD_FORCE"] = "1"
    import torch
    import ccphylo_amd as cg
    from ccphylo_amd import native as nt
    from tools.synth import euclid_shard_dev
    names = ["init", "dnj_select", "dnj_scan", "nj_argmin", "update", "dnj_requeue", "nj_pop", "dnj_find", "coll",
             "exact_sum"]
    K = nt.NKSTAT
    dev = cg.Device(0)
    loc = euclid_shard_dev(torch, n, 0, 1, dtype=torch.float32)
    work = torch.empty_like(loc)
    for k in prefixes:
        work.copy_(loc)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        j, fn, fd, st = dev.tree_shard_dev(work.data_ptr(), n, None, etype=4, method=cg.CCG_TREE_DNJ, exact=True,
                                           max_joins=k, profile=True)
        dt = time.perf_counter() - t0
        per = {nm: round(st[5 + 2 * c] / 1e3 / len(j), 2) for c, nm in enumerate(names)
               if st[4 + 2 * c] and nm != "init"}
        print(json.dumps({"n": n, "world": 1, "kernels": "sharded (CCG_SHARD_FORCE=1)", "joins": len(j),
                          "wall_s": round(dt, 3), "device_s": round(st[3] / 1e6, 3),
                          "device_us_per_join": per, "device_us_per_join_total": round(sum(per.values()), 2),
                          "engine_cells_per_join": round(st[1] / len(j), 1),
                          "reference_rule_cells_per_join": round(st[11 + 2 * K] / len(j), 1)}), flush=True)
    dev.close()


if __name__ == "__main__":
    main()
