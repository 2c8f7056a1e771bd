"""dist into the band shards (ccg_snp_ltd_shard_dev) against the full-LT
kernel on the same device-resident random MSA (development aid):
    python tools/perf_dist_shard.py [N] [L] [world] [pair]
Times every rank of `world` one after another on this GPU (each rank's rows
only), so sum-over-ranks vs the full kernel shows the band form's overhead
and max-over-ranks shows the balance an N-GPU node would see."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import ccphylo_amd as cg  # noqa: E402
from ccphylo_amd import native as nt  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
L = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
world = int(sys.argv[3]) if len(sys.argv) > 3 else 8
pair = len(sys.argv) > 4 and sys.argv[4] == "pair"
torch.cuda.set_device(0)
dev = cg.Device(0)
W = L // 32 + 1
g = torch.Generator(device="cuda").manual_seed(3)
seqs = torch.randint(-2**62, 2**62, (n, W), dtype=torch.int64, device="cuda", generator=g)
incs = torch.full((n, W) if pair else (W,), -1, dtype=torch.int32, device="cuda")
incs[..., (L + 31) // 32:] = 0
if L % 32:
    incs[..., (L + 31) // 32 - 1] = ((0xFFFFFFFF << (32 - L % 32)) & 0xFFFFFFFF) - (1 << 32)
if pair:
    incs &= torch.randint(-2**31, 2**31, incs.shape, dtype=torch.int32, device="cuda", generator=g) | 0x7FFF7FFF
m = n * (n - 1) // 2


def timed(fn, reps=3):
    fn()
    best = 1e30
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


Dd = torch.empty(m, dtype=torch.float64, device="cuda")
t_full = timed(lambda: dev.snp_ltd_dev(seqs.data_ptr(), incs.data_ptr(), n, L, W, Dd.data_ptr(), pair=pair))
full = Dd.cpu().numpy()
del Dd
ranks = []
ok = True
for r in range(world):
    e = nt.shard_elems(n, r, world)
    Dl = torch.empty(max(e, 1), dtype=torch.float64, device="cuda")
    t = timed(lambda: dev.snp_ltd_shard_dev(seqs.data_ptr(), incs.data_ptr(), n, L, W, Dl.data_ptr(), r, world,
                                             pair=pair))
    ok = ok and bool((Dl[:e].cpu().numpy() == nt.shard_extract(full, n, r, world)).all())
    ranks.append({"rank": r, "cells": e, "seconds": round(t, 4)})
    del Dl
tmax = max(x["seconds"] for x in ranks)
tsum = sum(x["seconds"] for x in ranks)
print(json.dumps({"n": n, "L": L, "world": world, "mode": "pair (-f 3)" if pair else "non-pair",
                  "full_seconds": round(t_full, 4), "full_taxa_pairs_per_s": round(m / t_full, 1),
                  "band_sum_seconds": round(tsum, 4), "band_max_seconds": tmax,
                  "band_overhead_sum_vs_full": round(tsum / t_full, 3),
                  "node_taxa_pairs_per_s_at_max": round(m / tmax, 1), "identical_to_band_extract": ok,
                  "ranks": ranks}), flush=True)
