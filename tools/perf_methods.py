"""Joins/s of the three tree methods (hnj, nj, dnj) at N (default 10k), fast and exact row sums (development aid)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import ccphylo_amd as cg
from tools.synth import euclid
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
D = euclid(n)
dev = cg.Device(0)
for method, name in ((2, "hnj"), (0, "nj"), (1, "dnj")):
    for exact in (False, True):
        j, fn, fd, st = dev.tree(D, n, method=method, exact=exact)
        _, _, _, sp = dev.tree(D, n, method=method, exact=exact, profile=True)
        parts = []
        for c, nm in enumerate(cg.native.KSTAT_NAMES):
            if sp[4 + 2 * c]:
                parts.append(f"{nm} {sp[5 + 2 * c] / sp[4 + 2 * c] / 1e3:.2f}us x{sp[4 + 2 * c]}")
        print(f"{name} exact={exact}: device {st[3]/1e6:.3f}s joins {len(j)} -> {len(j)/(st[3]/1e6):.0f} joins/s; " + ", ".join(parts), flush=True)
