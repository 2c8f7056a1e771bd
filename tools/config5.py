"""BASELINE configs[4] pipeline: dist writes each rank's LT shard in HBM and the
sharded DNJ consumes it in place ("dist writes the
shards that DNJ consumes in place").  One process per GPU (torchrun env), or
world 1 as a rehearsal on one GPU at reduced n.

Per rank: the same tree-like packed alignment (tools/config3.make_packed,
identical seed on every rank) -> ccg_snp_ltd_shard_dev (float LT rows of the
rank's bands: SNP counts are exact in float below 2^24) ->
ccg_tree_shard_dev (DNJ, fast row sums, RCCL between ranks) for the first
`--joins` joins.  Timings are the max over ranks.

    python tools/config5.py [--n 200000] [--L 100000] [--joins 2000]
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/config5.py --n 1000000
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200_000)
    ap.add_argument("--L", type=int, default=100_000)
    ap.add_argument("--joins", type=int, default=2000)
    ap.add_argument("--check", action="store_true", help="compare a few shard cells with the oracle's fsacmp")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
    torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    import ccphylo_amd as cg
    from ccphylo_amd import native as nt
    from tools.config3 import make_packed

    def tmax(x):
        if world == 1:
            return x
        t = torch.tensor([x])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0])

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    n, L = args.n, args.L
    W = L // 32 + 1
    dev = cg.Device(torch.cuda.current_device())
    t0 = time.perf_counter()
    seqs = make_packed(torch, n, W)
    incs = torch.full((W,), -1, dtype=torch.int32, device="cuda")
    incs[::10] = 0
    incs[(L + 31) // 32:] = 0
    if L % 32:
        incs[(L + 31) // 32 - 1] &= ((0xFFFFFFFF << (32 - L % 32)) & 0xFFFFFFFF) - (1 << 32)
    barrier()
    tgen = time.perf_counter() - t0
    m = nt.shard_elems(n, rank, world)
    Dloc = torch.empty(max(m, 1), dtype=torch.float32, device="cuda")
    barrier()
    t0 = time.perf_counter()
    inc = dev.snp_ltd_shard_dev(seqs.data_ptr(), incs.data_ptr(), n, L, W, Dloc.data_ptr(), rank, world, etype=4)
    torch.cuda.synchronize()
    tdist = tmax(time.perf_counter() - t0)
    res = {"n": n, "L": L, "world": world, "gen_s": round(tgen, 2), "dist_s": round(tdist, 3),
           "taxa_pairs_per_s": round(n * (n - 1) / 2 / tdist, 1), "included_positions": inc,
           "lt_GB_per_rank": round(4 * m / 1e9, 2)}
    if args.check:
        import numpy as np
        from oracle import pyoracle
        lib = pyoracle.lib()
        hinc = incs.cpu().numpy().view(np.uint32).copy()
        bad = 0
        for i in (n - 1, n // 2 + 3, 8 * world * 3 + rank * 8 + 5):
            if i >= n or not nt.shard_owner(i, world) == rank:
                continue
            for j in (0, i // 2, i - 1):
                a = seqs[i].cpu().numpy().view(np.uint64).copy()
                b = seqs[j].cpu().numpy().view(np.uint64).copy()
                ref = lib.orc_fsacmp(a.ctypes.data, b.ctypes.data, hinc.ctypes.data, L)
                bad += float(Dloc[nt.shard_row_offset(i, rank, world) + j].item()) != float(ref)
        res["check_mismatches"] = bad
    del seqs, incs
    torch.cuda.empty_cache()
    coll = nt.RcclColl(dev, dist) if world > 1 else None
    try:
        barrier()
        t0 = time.perf_counter()
        j, fn, fd, st = dev.tree_shard_dev(Dloc.data_ptr(), n, coll, etype=4, method=cg.CCG_TREE_DNJ, exact=False,
                                           max_joins=args.joins)
        torch.cuda.synchronize()
        ttree = tmax(time.perf_counter() - t0)
    finally:
        if coll is not None:
            coll.close()
    res.update({"joins": len(j), "tree_s_incl_init": round(ttree, 3), "joins_per_s_incl_init": round(len(j) / ttree, 1),
                "config": "configs[4] pipeline: tree-like packed alignment in HBM -> ccg_snp_ltd_shard_dev (float LT "
                          "band shards) -> ccg_tree_shard_dev DNJ in place (first joins, init included)"})
    if rank == 0:
        print(json.dumps(res), flush=True)
    dev.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
