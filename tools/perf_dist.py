"""dist throughput on device-resident random MSAs (development aid):
    python tools/perf_dist.py [N] [L] [pair]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import ccphylo_amd as cg  # noqa: E402
from bench import dist_extra  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
L = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
torch.cuda.set_device(0)
dev = cg.Device(0)
print(dist_extra(dev, torch, n=n, L=L, pair=len(sys.argv) > 3 and sys.argv[3] == "pair"), flush=True)
