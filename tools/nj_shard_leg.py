"""The bench nj_sharded leg alone (development aid)."""
import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
import ccphylo_amd as cg
from bench import nj_shard_extra
torch.cuda.set_device(0)
dev = cg.Device(0)
for _ in range(2):
    r = nj_shard_extra(dev, torch, n=100000, joins=64)
    print({k: r[k] for k in ("joins_per_s", "ms_per_join", "hbm_GBps_aggregate", "argmin_kernel_GBps_per_gpu", "coll_us_per_join")}, flush=True)
