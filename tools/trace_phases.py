"""Phase stamps of the DNJ/NJ join kernels (diagnostic engine build).

    make -C ccphylo_amd trace
    CCPHYLO_AMD_ENGINE=ccphylo_amd/lib/libccphylo_amd_trace.so CCG_TRACE_N=5000 \
        python tools/trace_phases.py 10000 [dnj|nj]
The engine prints the averaged stamps to stderr (us from each kernel's first
block entry; gap = previous kernel's last block exit -> this kernel's first entry).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ccphylo_amd as cg
from tools.synth import euclid  # noqa: E402
import numpy as np  # noqa: E402




n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
method = cg.CCG_TREE_NJ if (len(sys.argv) > 2 and sys.argv[2] == "nj") else cg.CCG_TREE_DNJ
D = euclid(n)
dev = cg.Device(0)
for exact in (False, True):
    joins, fn, fd, st = dev.tree(D, n, method=method, exact=exact)
    print(f"exact={exact}: {len(joins)} joins, device {st[3] / 1e3:.1f} ms", flush=True)
