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
dev = cg.Device(0)
if "--c2" in sys.argv:   # the bench headline's alignment (configs[2] data at this n, 5 Mbp)
    import torch
    from bench import make_headline_alignment
    seqs, incs, W = make_headline_alignment(torch, n, 5_000_000)
    Dd = torch.empty(n * (n - 1) // 2, dtype=torch.float64, device="cuda")
    dev.snp_ltd_dev(seqs.data_ptr(), incs.data_ptr(), n, 5_000_000, W, Dd.data_ptr())
    D = Dd.cpu().numpy()
    del seqs, Dd
    torch.cuda.empty_cache()
elif "--clade" in sys.argv:   # config-3-like clade data (tools/config3.py) through the GPU dist
    import torch
    from tools.config3 import make_packed
    L = 1_000_000
    W = L // 32 + 1
    seqs = make_packed(torch, n, W)
    incs = torch.full((W,), -1, dtype=torch.int32, device="cuda")
    incs[(L + 31) // 32:] = 0
    Dd = torch.empty(n * (n - 1) // 2, dtype=torch.float64, device="cuda")
    dev.snp_ltd_dev(seqs.data_ptr(), incs.data_ptr(), n, L, W, Dd.data_ptr())
    D = Dd.cpu().numpy()
    del seqs, Dd
elif "--c3" in sys.argv:   # configs[3]'s float Euclidean matrix on the device, a join prefix (--joins J)
    import torch
    from tools.synth import euclid_shard_dev
    J = int(sys.argv[sys.argv.index("--joins") + 1]) if "--joins" in sys.argv else 26000
    loc = euclid_shard_dev(torch, n, 0, 1, dtype=torch.float32)
    torch.cuda.synchronize()
    joins, fn, fd, st = dev.tree_dev(loc.data_ptr(), n, etype=4, method=method, exact=True, max_joins=J)
    print(f"c3 prefix: {len(joins)} joins, device {st[3] / 1e3:.1f} ms", flush=True)
    sys.exit(0)
else:
    D = euclid(n)
for exact in ((True,) if "--exact" in sys.argv else (False, True)):
    joins, fn, fd, st = dev.tree(D, n, method=method, exact=exact)
    print(f"exact={exact}: {len(joins)} joins, device {st[3] / 1e3:.1f} ms", flush=True)
