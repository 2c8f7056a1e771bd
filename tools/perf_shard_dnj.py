"""Sharded DNJ (ccg_tree_shard_dev, CCG_TREE_DNJ) against the single-GPU DNJ
engine on one GPU (development aid):
  python tools/perf_shard_dnj.py [n ...] [--joins K] [--float]
Every n: the Euclidean matrix of tools/synth.euclid_shard_dev at world 1 (the
shard layout of world 1 IS the reference LT layout), both engines on copies,
joins compared, device time and per-class kernel time printed."""
import sys
import os
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import ccphylo_amd as cg  # noqa: E402
from ccphylo_amd import native as nt  # noqa: E402
from tools.synth import euclid_shard_dev  # noqa: E402


def report(tag, n, nj, st, wall):
    us = st[3]
    print(f"{tag:10s} n={n} joins {nj} device {us / 1e6:.3f} s wall {wall:.3f} s -> {nj / (us / 1e6):.0f} joins/s; "
          f"rows {st[0]} cells {st[1]}", flush=True)
    for c, name in enumerate(nt.KSTAT_NAMES):
        cnt, ns = st[4 + 2 * c], st[5 + 2 * c]
        if cnt:
            print(f"   {name:12s} {cnt:8d} x {ns / cnt / 1e3:8.2f} us = {ns / 1e9:.3f} s", flush=True)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("-")]
    joins = [0]
    if "--joins" in sys.argv:
        js = sys.argv[sys.argv.index("--joins") + 1]
        joins = [int(x) for x in js.split(",")]
        args = [a for a in args if a != js]
    prof = "--prof" in sys.argv
    fl = "--float" in sys.argv
    et = 4 if fl else 8
    sizes = [int(a) for a in args] or [10000]
    dev = cg.Device(0)
    for n in sizes:
        t = time.perf_counter()
        loc = euclid_shard_dev(torch, n, 0, 1, dtype=torch.float32 if fl else torch.float64)
        torch.cuda.synchronize()
        print(f"n={n}: matrix {loc.numel() * loc.element_size() / 1e9:.1f} GB generated in {time.perf_counter() - t:.1f} s",
              flush=True)
        work = torch.empty_like(loc)
        for k in joins:
            run_one(dev, n, loc, work, et, k, prof)
        del loc, work
        torch.cuda.empty_cache()


def run_one(dev, n, loc, work, et, joins, prof):
        res = {}
        for tag in (("single",) if "--single" in sys.argv else ("single", "shard-w1")):
            work.copy_(loc)
            torch.cuda.synchronize()
            t = time.perf_counter()
            if tag == "single":
                j, fn, fd, st = dev.tree_dev(work.data_ptr(), n, etype=et, method=cg.CCG_TREE_DNJ, exact=False,
                                             profile=prof, max_joins=joins)
            else:
                j, fn, fd, st = dev.tree_shard_dev(work.data_ptr(), n, None, etype=et, method=cg.CCG_TREE_DNJ,
                                                   exact=False, profile=prof, max_joins=joins)
            report(tag, n, len(j), st, time.perf_counter() - t)
            res[tag] = j
        if "shard-w1" in res:
            a, b = res["single"], res["shard-w1"]
            print("   identical joins:", bool(len(a) == len(b) and (a == b).all()), flush=True)


if __name__ == "__main__":
    main()
