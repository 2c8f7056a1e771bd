"""One DNJ (or NJ) run at n taxa on the euclid test matrix, for profilers
(development aid):  python tools/perf_dnj.py 10000 [dnj|nj] [exact]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ccphylo_amd as cg  # noqa: E402
from tools.synth import euclid  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
method = cg.CCG_TREE_NJ if (len(sys.argv) > 2 and sys.argv[2] == "nj") else cg.CCG_TREE_DNJ
exact = len(sys.argv) > 3 and sys.argv[3] == "exact"
D = euclid(n)
dev = cg.Device(0)
joins, fn, fd, st = dev.tree(D, n, method=method, exact=exact)
print(f"{len(joins)} joins, device {st[3] / 1e3:.1f} ms -> {len(joins) / (st[3] / 1e6):.0f} joins/s", flush=True)
