"""Whole-tree parity on the headline's OWN matrix: the
bench's configs[2] alignment (50k taxa x 5 Mbp, tools/config3.make_packed
seed 3, generated on the GPU), its GPU dist (double LT, 10 GB), the engine's
whole exact DNJ tree, and the oracle's serial-decision DNJ (oracle/ccoracle.c,
dnj.c:43-128 / :985-1052; test infrastructure, the checker) on the same LT,
on the GPU box's host cores.

The oracle dist is infeasible at 5 Mbp (2.9e15 position pairs), so 64 LT
cells are checked against the oracle's fsacmp (fsacmp.c:552) instead.

The oracle's whole 50k tree takes longer than one GPU call may run, so it
runs in segments [C0, C1) that chain exactly:
  - segment 0 starts from dnj_init on the GPU LT (initSummaD + initHNJ on the
    host, from the raw matrix);
  - a later segment starts from the ENGINE's checkpoint at C0
    (ccg_tree_dev_state), and
  - every segment ends by comparing the oracle's whole loop state at C1 (the
    LT of the n - C1 remaining rows, sD, Q, N, P and minPos's candidate) with
    the engine's checkpoint at C1, bit for bit.
So the oracle's joins [0, C1) equal the engine's and the two states at C1 are
identical; the next segment, started from the engine's state at C1, is
therefore the oracle's own continuation.  Joins are compared against the
engine's uninterrupted whole tree (one ccg_tree_dev call, the bench's form),
whose joins sha is printed beside the bench's.

    python tools/parity_headline.py --start 0 --budget 900 --out gpurun_out/r06_parity_headline.jsonl
    python tools/parity_headline.py --start C1 --budget 900 --out ...   (the next call)
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint8)).hexdigest()[:16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50_000)
    ap.add_argument("--L", type=int, default=5_000_000)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--start", type=int, default=0, help="first join of this segment (0 or a previous C1)")
    ap.add_argument("--budget", type=float, default=900.0, help="seconds of oracle time in this call")
    ap.add_argument("--chunk", type=int, default=250, help="oracle joins between progress lines")
    ap.add_argument("--cells", type=int, default=64, help="LT cells checked against orc_fsacmp (segment 0)")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--out")
    a = ap.parse_args()
    import torch
    import ccphylo_amd as cg
    from bench import make_headline_alignment
    from oracle import pyoracle
    n, L = a.n, a.L
    K = cg.native.NKSTAT
    T0 = time.perf_counter()
    rec = {"n": n, "L": L, "seed": a.seed, "segment_start": a.start}

    def emit(msg):
        print(msg, flush=True)

    dev = cg.Device(0)
    seqs, incs, W = make_headline_alignment(torch, n, L, seed=a.seed)
    D = torch.empty(n * (n - 1) // 2, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    rec["included_positions"] = int(dev.snp_ltd_dev(seqs.data_ptr(), incs.data_ptr(), n, L, W, D.data_ptr()))
    torch.cuda.synchronize()
    if a.start == 0 and a.cells:
        lib = pyoracle.lib()
        hinc = incs.cpu().numpy().view(np.uint32).copy()
        rng = np.random.default_rng(6)
        pairs = [(1, 0), (n - 1, 0), (n - 1, n - 2), (n // 2, n // 3)]
        while len(pairs) < a.cells:
            i, j = sorted(rng.choice(n, 2, replace=False).tolist(), reverse=True)
            pairs.append((i, j))
        bad = []
        for i, j in pairs:
            x = seqs[i].cpu().numpy().view(np.uint64).copy()
            y = seqs[j].cpu().numpy().view(np.uint64).copy()
            want = float(lib.orc_fsacmp(x.ctypes.data, y.ctypes.data, hinc.ctypes.data, L))
            if float(D[i * (i - 1) // 2 + j].item()) != want:
                bad.append((i, j))
        rec["cells_checked_vs_orc_fsacmp"] = len(pairs)
        rec["cells_identical"] = not bad
        emit(f"{len(pairs)} LT cells vs orc_fsacmp: {'identical' if not bad else bad[:4]}")
    del seqs, incs
    torch.cuda.empty_cache()
    rec["ltd_sha256"] = sha(D.cpu().numpy()) if a.start == 0 else None
    # the engine's uninterrupted whole tree (the bench's form), on a copy
    Dw = D.clone()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gj, gfn, gfd, _ = dev.tree_dev(Dw.data_ptr(), n, method=cg.CCG_TREE_DNJ, exact=True)
    rec["gpu_tree_s"] = round(time.perf_counter() - t0, 3)
    rec["engine_joins_sha256"] = hashlib.sha256(np.ascontiguousarray(gj).tobytes() +
                                                np.array([gfn, gfd]).tobytes()).hexdigest()[:16]
    del Dw
    torch.cuda.empty_cache()
    emit(f"engine whole tree: {len(gj)} joins in {rec['gpu_tree_s']} s, sha {rec['engine_joins_sha256']}")
    # the oracle's starting state
    t0 = time.perf_counter()
    st_start, cur0 = None, n - a.start
    if a.start == 0:
        host = D.cpu().numpy()
        ost = pyoracle.dnj_init(host, n, threads=a.threads)
        rec["start_from"] = "oracle dnj_init on the GPU LT"
    else:
        # D becomes the engine's LT at `start` (in place); st_start its vectors
        _, _, _, _, st_start = dev.tree_dev_state(D.data_ptr(), n, max_joins=a.start)
        assert st_start["n"] == cur0
        host = D[:cur0 * (cur0 - 1) // 2].cpu().numpy()
        ost = pyoracle.DnjState(host, cur0, st_start["sD"].copy(), st_start["Q"].copy(), st_start["N"].copy(),
                                st_start["P"].copy(), st_start["cand"])
        rec["start_from"] = f"engine checkpoint at join {a.start}"
    emit(f"oracle start state ({rec['start_from']}) in {time.perf_counter() - t0:.1f} s")
    # oracle joins until the budget
    done, t0, same = a.start, time.perf_counter(), True
    rrows = rcells = 0
    while ost.n > 2 and time.perf_counter() - t0 < a.budget:
        rj, _, _, rs = pyoracle.dnj_resume(ost, max_joins=a.chunk, threads=a.threads, stats=True)
        rrows += int(rs[0])
        rcells += int(rs[1])
        ok = bool((gj[done:done + len(rj)] == rj).all()) and done + len(rj) <= len(gj)
        if not ok and same:
            bad = np.nonzero(gj[done:done + len(rj)] != rj)[0]
            rec["first_differing_join"] = done + int(bad[0]) if bad.size else done
        same = same and ok
        done += len(rj)
        emit(f"oracle joins [{a.start}, {done}) identical {same}; {time.perf_counter() - t0:.0f} s, "
             f"matrix {ost.n}")
        if not same:
            break
    rec["segment_end"] = done
    rec["joins_compared"] = done - a.start
    rec["joins_identical"] = same
    rec["oracle_s"] = round(time.perf_counter() - t0, 1)
    rec["oracle_threads"] = a.threads
    rec["oracle_reference_rule_rows_cells"] = [rrows, rcells]
    if ost.n <= 2:   # the whole tree: the final pair too
        rec["final_identical"] = (int(ost.n), float(ost.D[0]) if ost.n == 2 else -1.0) == (int(gfn), float(gfd))
    elif same:
        # the engine's checkpoint at `done`, continued from its state at
        # `start` (D holds that state's LT: the oracle works on a host copy)
        _, _, _, _, st1 = dev.tree_dev_state(D.data_ptr(), cur0, max_joins=done - a.start, state=st_start)
        cur = n - done
        eng = D[:cur * (cur - 1) // 2].cpu().numpy()
        cmp = {"ltd": bool(np.array_equal(eng.view(np.uint64), ost.D[:cur * (cur - 1) // 2].view(np.uint64))),
               "sD": bool(np.array_equal(st1["sD"][:cur].view(np.uint64), ost.sD[:cur].view(np.uint64))),
               "Q": bool(np.array_equal(st1["Q"][:cur].view(np.uint64), ost.Q[:cur].view(np.uint64))),
               "N": bool(np.array_equal(st1["N"][:cur], ost.N[:cur])),
               "P": bool(np.array_equal(st1["P"][:cur], ost.P[:cur])),
               "cand": int(st1["cand"]) == int(ost.cand)}
        rec["state_at_end_identical"] = cmp
        rec["state_matrix_size"] = cur
        if not all(cmp.values()):
            for k in ("sD", "Q", "N", "P"):
                if not cmp[k]:
                    x, y = st1[k][:cur], getattr(ost, k)[:cur]
                    rec.setdefault("state_first_diff", {})[k] = int(np.nonzero(x != y)[0][0])
    rec["wall_s"] = round(time.perf_counter() - T0, 1)
    emit(json.dumps(rec))
    if a.out:
        with open(a.out, "a") as f:
            f.write(json.dumps(rec) + "\n")
    dev.close()



if __name__ == "__main__":
    main()
