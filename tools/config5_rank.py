"""One rank of BASELINE configs[4] on one GPU: n = 1e6 taxa x L = 100 kbp,
world 8, the rank's dist straight into its float band shard (250 GB), with
the packed MSA in host memory streamed into the bit planes
(ccg_snp_ltd_shard), so the rank's HBM holds the planes (25 GB) and the shard
only -- the per-rank memory plan of DESIGN.md 6 ("configs[4] memory budget").

    python tools/config5_rank.py [--n 1000000] [--L 100000] [--world 8] [--rank 0] [--check]

Reports the dist time of the rank, HBM free before / after the shard
allocation (hipMemGetInfo through torch), and (--check) sampled shard cells
against the oracle's fsacmp (fsacmp.c:552, test infrastructure only).
The alignment is tools/config3.make_packed's tree-like data, generated on the
GPU in row chunks and moved to host memory (the same bytes on every rank)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def make_packed_host(torch, n, W, clades=512, seed=3, chunk=8192):
    """make_packed's construction (random clade roots, ~0.8% of the 2-bit codes
    flipped per taxon) chunk by chunk into a host array."""
    import numpy as np
    g = torch.Generator(device="cuda").manual_seed(seed)
    roots = torch.randint(-2**62, 2**62, (clades, W), dtype=torch.int64, device="cuda", generator=g)
    host = np.empty((n, W), dtype=np.uint64)
    ht = torch.from_numpy(host.view(np.int64))
    for t0 in range(0, n, chunk):
        t1 = min(n, t0 + chunk)
        m = torch.randint(-2**62, 2**62, (t1 - t0, W), dtype=torch.int64, device="cuda", generator=g)
        for _ in range(7):
            m &= torch.randint(-2**62, 2**62, (t1 - t0, W), dtype=torch.int64, device="cuda", generator=g)
        idx = torch.arange(t0, t1, device="cuda") % clades
        ht[t0:t1].copy_(roots[idx] ^ m)
        del m
    del roots
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return host


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--L", type=int, default=100_000)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    import numpy as np
    import torch
    import ccphylo_amd as cg
    from ccphylo_amd import native as nt
    n, L, world, rank = a.n, a.L, a.world, a.rank
    W = L // 32 + 1
    torch.cuda.set_device(0)
    dev = cg.Device(0)
    t0 = time.perf_counter()
    seqs = make_packed_host(torch, n, W)
    incs = np.full(W, 0xFFFFFFFF, dtype=np.uint32)
    incs[::10] = 0
    incs[(L + 31) // 32:] = 0
    if L % 32:
        incs[(L + 31) // 32 - 1] &= (0xFFFFFFFF << (32 - L % 32)) & 0xFFFFFFFF
    tgen = time.perf_counter() - t0
    print(json.dumps({"stage": "generated", "gen_s": round(tgen, 1), "host_GB": round(seqs.nbytes / 1e9, 2)}),
          flush=True)
    free0, total = torch.cuda.mem_get_info()
    elems = nt.shard_elems(n, rank, world)
    Dloc = dev.malloc(elems * 4)
    free1, _ = torch.cuda.mem_get_info()
    W32 = (L + 31) // 32
    Wp = -(-W32 // 16) * 16   # plane words per taxon (KC = 16), rows padded to 128
    planes = -(-n // 128) * 128 * Wp * 8
    t0 = time.perf_counter()
    inc = dev.snp_ltd_shard(seqs, incs, n, L, Dloc, rank, world, etype=4)
    tdist = time.perf_counter() - t0
    res = {"n": n, "L": L, "world": world, "rank": rank, "dist_s": round(tdist, 3), "included_positions": inc,
           "rank_cells": elems, "rank_taxa_pairs_per_s": round(elems / tdist, 1),
           "position_pairs_per_s": elems * float(L) / tdist,
           "hbm_total_GB": round(total / 1e9, 2), "hbm_free_before_GB": round(free0 / 1e9, 2),
           "shard_GB": round(elems * 4 / 1e9, 2), "hbm_free_after_shard_GB": round(free1 / 1e9, 2),
           "planes_GB": round(planes / 1e9, 2), "staging_GB": 0.27,
           "peak_GB_planned": round((elems * 4 + planes + (256 << 20)) / 1e9, 2),
           "packed_msa_host_GB": round(seqs.nbytes / 1e9, 2),
           "config": "configs[4] one rank: tree-like packed alignment in host memory -> ccg_snp_ltd_shard (planes "
                     "streamed into HBM) -> the rank's float band shard"}
    if a.check:
        from oracle import pyoracle
        lib = pyoracle.lib()
        rng = np.random.default_rng(1)
        host = np.empty(1, dtype=np.float32)
        bad = checked = 0
        rows = [r for r in (n - 1, n // 2 + 3, 8 * world * 3 + rank * 8 + 5, 8 * rank + 1) if nt.shard_owner(r, world) == rank]
        rows += [int(b) * 8 + int(rng.integers(0, 8)) for b in rng.integers(0, n // 8, 64) if b % world == rank][:8]
        for i in rows:
            if i >= n or i < 1:
                continue
            for j in sorted({0, i // 2, i - 1, int(rng.integers(0, i))}):
                ref = lib.orc_fsacmp(seqs[i].ctypes.data, seqs[j].ctypes.data, incs.ctypes.data, L)
                dev.d2h(host, Dloc + 4 * (nt.shard_row_offset(i, rank, world) + j))
                bad += float(host[0]) != float(ref)
                checked += 1
        res["check_cells"] = checked
        res["check_mismatches"] = bad
    dev.free(Dloc)
    print(json.dumps(res), flush=True)
    dev.close()


if __name__ == "__main__":
    main()
