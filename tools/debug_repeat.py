"""Repeat GPU trees vs the oracle to catch nondeterminism (development aid)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import ccphylo_amd as cg
from oracle import pyoracle
mats = cg.load_phylip(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "test.phy.gz"))
names, D = mats[0]
n = len(names)
dev = cg.Device(0)
for flags in (0, 2):
    for method in (1, 0):
        rj, rfn, rfd = pyoracle.tree(D, n, method=method, flags=flags)
        bad = 0
        for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):
            for exact in (True, False):
                j, fn, fd, st = dev.tree(D, n, method=method, flags=flags, exact=exact)
                same_ij = len(j) == len(rj) and (j["i"] == rj["i"]).all() and (j["j"] == rj["j"]).all()
                same_L = same_ij and (j["Li"] == rj["Li"]).all() and (j["Lj"] == rj["Lj"]).all()
                if not (same_ij and (same_L or not exact)):
                    bad += 1
                    if bad <= 3:
                        k = next((t for t in range(min(len(j), len(rj))) if tuple(j[t]) != tuple(rj[t])), None)
                        print(f"flags={flags} method={method} exact={exact} rep={rep}: first diff at join {k}: gpu {j[k] if k is not None else None} ref {rj[k] if k is not None else None} n={len(j)}/{len(rj)}")
        print(f"flags={flags} method={method}: {bad} bad runs")
