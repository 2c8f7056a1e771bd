"""Exact-mode row sums on the GPU (development aid): the parallel
binade-segmented sum alone (ccg_selftest_row_sum, CCG_SELFTEST_REPS timing)
and inside DNJ / NJ / HNJ at N (default 10k): joins/s, requeue/pop time,
how many sums needed the serial order and how many the chain computed."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import ccphylo_amd as cg  # noqa: E402
from tools.synth import euclid  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
dev = cg.Device(0)
rng = np.random.default_rng(1)
os.environ["CCG_SELFTEST_REPS"] = "200"
for m in (1000, 10000, 50000):
    dev.selftest_row_sum(np.round(rng.random(m) * 1e9) / 1e9)
del os.environ["CCG_SELFTEST_REPS"]
D = euclid(n)
K = cg.native.NKSTAT
for method, name in ((1, "dnj"), (0, "nj"), (2, "hnj")):
    j, fn, fd, st = dev.tree(D, n, method=method, exact=True)
    _, _, _, sp = dev.tree(D, n, method=method, exact=True, profile=True)
    parts = [f"{nm} {sp[5 + 2 * c] / sp[4 + 2 * c] / 1e3:.2f}us" for c, nm in enumerate(cg.native.KSTAT_NAMES)
             if sp[4 + 2 * c]]
    print(f"{name} exact: {len(j) / (st[3] / 1e6):.0f} joins/s; serial-order sums {sp[6 + 2 * K]}, by the chain "
          f"{sp[7 + 2 * K]}; " + ", ".join(parts), flush=True)
