"""configs[3]'s late tree against the oracle (joins past 12k
pinned by nothing).  In the default suite at 40k taxa (test_late_tree_resume_40k,
well under a minute); at configs[3]'s 200k OPT-IN (CCG_LATE=1, about 10 minutes on one MI355X;
run it with `pytest -s` so the engine's progress lines keep the call alive):
the whole 200k float tree does not fit the default GPU suite's time, and the
oracle's serial rule rescans ~4e9 cells per join there.

The single engine (default float path: row-group rescans, k_dnj_fold,
k_dnj_join_pf) builds the bench's configs[3] tree (Euclidean U[0,1)^8,
seed 4, float LT) in legs with ccg_tree_dev_state.  At each cut k (default
60k, 120k, 180k joins) the engine's checkpoint (the LT of n - k rows, sD, Q,
N, P and minPos's candidate, dnj.c:985-1052) is copied to the host and the
oracle (oracle/ccoracle.c, threaded rescans with the serial loop's decisions)
continues m joins from it (default 200) while the engine continues m joins
from the same checkpoint: both must make the same joins, bit for bit, with
the same reference-rule rescan counts.  Results go to $CCG_LATE_OUT (JSON
lines) when set.  Reference: dnj.c:43-128 (minQpair), nj.c:911 (the serial
row sum), dnj.c:607-975 (updateDNJ, DNJ_popArrange)."""
import json
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_late_tree_resume_40k():
    """The same check at a size the default GPU suite affords:
    a 40k float Euclidean matrix (seed 4), cut at 15k joins (matrix 25k: the
    float row groups over the compacted enumeration with pruning, k_dnj_fold
    and the long-listing k_dnj_join_pf path run from the checkpoint on) and at
    30k joins (matrix 10k: the small-n plan and scans); at each cut the oracle
    continues 200 joins from the engine's state, joins and reference-rule
    counters identical."""
    _late_legs(40_000, [15_000, 30_000], 200, os.environ.get("CCG_LATE_OUT"))


@pytest.mark.skipif(not os.environ.get("CCG_LATE"), reason="opt-in: CCG_LATE=1 (about 10 minutes)")
def test_config3_late_tree_resume():
    n = int(os.environ.get("CCG_LATE_N", 200_000))
    cuts = [int(x) for x in os.environ.get("CCG_LATE_CUTS", "60000,120000,180000").split(",")]
    m = int(os.environ.get("CCG_LATE_M", 200))
    os.environ.setdefault("CCG_PROGRESS", "1")
    # CCG_LATE_GEN=cdist: round 4's torch.cdist matrix (its reference rule
    # rescans ~1.7e9 cells per join: give it fewer joins per cut)
    _late_legs(n, cuts, m, os.environ.get("CCG_LATE_OUT"), cdist=os.environ.get("CCG_LATE_GEN") == "cdist")


def _late_legs(n, cuts, m, out, cdist=False):
    import torch
    import ccphylo_amd as cg
    from ccphylo_amd import native
    from oracle import pyoracle
    from tools.synth import euclid_shard_dev
    K = native.NKSTAT
    threads = min(16, os.cpu_count() or 4)
    dev = cg.Device(0)
    D = euclid_shard_dev(torch, n, 0, 1, dtype=torch.float32, cdist=cdist)   # world 1: the packed LT
    torch.cuda.synchronize()
    state, done, t_gpu = None, 0, 0.0
    for k in cuts:
        cur = n - done
        t0 = time.perf_counter()
        _, _, _, _, st = dev.tree_dev_state(D.data_ptr(), cur, etype=4, max_joins=k - done, state=state)
        t_gpu += time.perf_counter() - t0
        done, cur = k, n - k
        assert st["n"] == cur
        cells = D[:cur * (cur - 1) // 2].cpu().numpy()
        ost = pyoracle.DnjState(cells, cur, st["sD"].copy(), st["Q"].copy(), st["N"].copy(), st["P"].copy(),
                                st["cand"], etype=4)
        t0 = time.perf_counter()
        gj, _, _, gs, state = dev.tree_dev_state(D.data_ptr(), cur, etype=4, max_joins=m, state=st, profile=True)
        tg = time.perf_counter() - t0
        t_gpu += tg
        done += m
        t0 = time.perf_counter()
        rj, _, _, rs = pyoracle.dnj_resume(ost, max_joins=m, threads=threads, stats=True)
        to = time.perf_counter() - t0
        del cells, ost
        same = len(gj) == len(rj) == m and bool((gj == rj).all())
        rec = {"n": n, "generator": "torch.cdist (round 4)" if cdist else "elementwise (round 5)", "cut": k,
               "matrix_size": cur, "joins_compared": m, "joins_identical": same,
               "engine_reference_rule_rows_cells": [int(gs[10 + 2 * K]), int(gs[11 + 2 * K])],
               "oracle_rows_cells": [int(rs[0]), int(rs[1])],
               "engine_rows_cells": [int(gs[0]), int(gs[1])],
               "gpu_leg_s": round(tg, 3), "oracle_leg_s": round(to, 1), "oracle_threads": threads,
               "gpu_tree_s_so_far": round(t_gpu, 1)}
        print(json.dumps(rec), flush=True)
        if out:
            with open(out, "a") as f:
                f.write(json.dumps(rec) + "\n")
        assert same, ("late joins differ", k, int(np.nonzero(gj != rj)[0][0]) if len(gj) == len(rj) else None)
        assert (int(gs[10 + 2 * K]), int(gs[11 + 2 * K])) == (int(rs[0]), int(rs[1]))
    dev.close()
