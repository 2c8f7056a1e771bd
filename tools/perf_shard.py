"""Single-GPU NJ vs the sharded NJ engine at world 1 (no transport) and
over RCCL world 1: joins/s and per-class kernel time."""
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import ccphylo_amd as cg  # noqa: E402
from ccphylo_amd import native as nt  # noqa: E402
from tools.synth import euclid  # noqa: E402


def report(tag, n, st, wall):
    us = st[3]
    print(f"{tag:12s} n={n} device {us / 1e6:.3f} s  wall {wall:.3f} s  {(n - 2) / (us / 1e6):.0f} joins/s", flush=True)
    for c, name in enumerate(nt.KSTAT_NAMES):
        cnt, ns = st[4 + 2 * c], st[5 + 2 * c]
        if cnt:
            print(f"   {name:12s} {cnt:8d} x {ns / cnt / 1e3:8.2f} us = {ns / 1e9:.3f} s")


def main():
    import faulthandler
    faulthandler.enable()
    prof = "--noprof" not in sys.argv
    sizes = [int(a) for a in sys.argv[1:] if not a.startswith("-")] or [4000, 10000]
    dev = cg.Device(0)
    for n in sizes:
        D = euclid(n, 1)
        for tag, fn in (("single", lambda: dev.tree(D, n, method=0, exact=False, profile=prof)),
                        ("shard-w1", lambda: dev.tree_shard(D, n, None, method=0, exact=False, profile=prof))):
            t = time.perf_counter()
            j, fnn, fd, st = fn()
            report(tag, n, st, time.perf_counter() - t)
            if tag == "single":
                ref = j
            else:
                print("   identical joins:", bool(len(j) == len(ref) and (j == ref).all()))


if __name__ == "__main__":
    main()
