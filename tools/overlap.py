"""Two engine contexts of one MI355X side by side (ccg_ctx_configure): one
matrix's dist on one set of compute units while the previous matrix's tree
runs on the rest (development aid for the pipelined headline):

    python tools/overlap.py [--n 50000] [--L 5000000] [--tree-cus 32] [--layout stride|low] [--steps 3]

Prints JSON lines: each leg alone on the whole chip, each alone on its CU set,
then the pipelined steps (dist of matrix k+1 beside the tree of matrix k, two
host threads); the joins' sha256 must not change."""
import argparse
import hashlib
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50_000)
    ap.add_argument("--L", type=int, default=5_000_000)
    ap.add_argument("--tree-cus", type=int, default=32)
    ap.add_argument("--layout", choices=["stride", "low", "xcd"], default="low",
                    help="stride: every (cus / k)-th CU; low: CUs 0 .. k-1; xcd: k / 8 CUs at the start of each "
                         "32-CU group (one per XCD if the mask's CU numbering is XCD-major)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--profile", action="store_true", help="per-join kernel times of the tree, masked and whole chip")
    a = ap.parse_args()
    import torch
    import ccphylo_amd as cg
    from bench import make_headline_alignment
    n, L = a.n, a.L
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    if a.layout == "stride":
        step = ncu // a.tree_cus
        tcus = [c for c in range(ncu) if c % step == 0][:a.tree_cus]
    elif a.layout == "xcd":
        per = max(1, a.tree_cus // 8)
        tcus = [g * (ncu // 8) + i for g in range(8) for i in range(per)]
    else:
        tcus = list(range(a.tree_cus))
    dcus = [c for c in range(ncu) if c not in set(tcus)]
    seqs, incs, W = make_headline_alignment(torch, n, L)
    m = n * (n - 1) // 2
    Ds = [torch.empty(m, dtype=torch.float64, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()
    dev = cg.Device(0)

    def dist(d, k):
        t0 = time.perf_counter()
        d.snp_ltd_dev(seqs.data_ptr(), incs.data_ptr(), n, L, W, Ds[k % 2].data_ptr())
        return time.perf_counter() - t0

    def tree(d, k, prof=None):
        t0 = time.perf_counter()
        j, fn, fd, st = d.tree_dev(Ds[k % 2].data_ptr(), n, method=cg.CCG_TREE_DNJ, exact=True, profile=prof is not None)
        sha = hashlib.sha256(np.ascontiguousarray(j).tobytes() + np.array([fn, fd]).tobytes()).hexdigest()[:16]
        if prof is not None:   # per-join microseconds by kernel class (HIP events)
            from ccphylo_amd import native as nt
            prof.update({name: round(st[5 + 2 * c] / 1e3 / max(len(j), 1), 2)
                         for c, name in enumerate(nt.KSTAT_NAMES) if st[4 + 2 * c]})
        return time.perf_counter() - t0, sha

    out = {"n": n, "L": L, "cus": ncu, "tree_cus": tcus, "layout": a.layout}
    out["dist_all_s"] = round(dist(dev, 0), 3)
    ts, sha0 = tree(dev, 0)
    out["tree_all_s"] = round(ts, 3)
    print(json.dumps(out), flush=True)
    dd, dt = cg.Device(0), cg.Device(0)
    dd.configure(cu_mask=dcus, nosync=True)
    dt.configure(cu_mask=tcus, nosync=True)
    r = {"dist_masked_s": round(dist(dd, 0), 3)}
    ts, sha = tree(dt, 0)
    r["tree_masked_s"] = round(ts, 3)
    if a.profile:
        prof = {}
        dist(dd, 0)
        tree(dt, 0, prof)
        full = {}
        dist(dev, 0)
        tree(dev, 0, full)
        r["us_per_join_masked"], r["us_per_join_all"] = prof, full
    r["sha_same"] = sha == sha0
    print(json.dumps(r), flush=True)
    dist(dd, 0)   # matrix 0 ready for the first pipelined tree
    t_all = time.perf_counter()
    for k in range(a.steps):
        res = {}

        def run_d():
            res["dist"] = dist(dd, k + 1)

        def run_t():
            res["tree"] = tree(dt, k)
        t0 = time.perf_counter()
        th = [threading.Thread(target=run_d), threading.Thread(target=run_t)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        print(json.dumps({"step": k, "wall_s": round(time.perf_counter() - t0, 3), "dist_s": round(res["dist"], 3),
                          "tree_s": round(res["tree"][0], 3), "sha_same": res["tree"][1] == sha0}), flush=True)
    print(json.dumps({"pipelined_s_per_matrix": round((time.perf_counter() - t_all) / a.steps, 3),
                      "sequential_s_per_matrix": round(out["dist_all_s"] + out["tree_all_s"], 3)}), flush=True)


if __name__ == "__main__":
    main()
    # (the CU-masked streams live to the process's end, ccg_ctx_configure; the
    # runtime's exit-time teardown of them is skipped, as in bench.py)
    sys.stdout.flush()
    os._exit(0)
