"""The headline's exact DNJ tree alone on a CU-masked context of k CUs
(bits 0 .. k-1, the pipeline's tree layout), nothing beside it, with optional
engine knobs per run: where does the tree's cliff below 64 CUs
(profiles/r06_cu_split.txt) come from?  One JSON line per run: the tree
context's device seconds, and a profiled run's per-kernel-class device us per
join.

    python tools/tree_cus.py [n] [L] 'k[:VAR=val,VAR=val]' ...
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import ccphylo_amd as cg
    from bench import KNAMES, make_headline_alignment
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 5_000_000
    runs = sys.argv[3:] or ["64", "56", "48"]
    seqs, incs, W = make_headline_alignment(torch, n, L)
    D0 = torch.empty(n * (n - 1) // 2, dtype=torch.float64, device="cuda")
    ddev = cg.Device(0)
    ddev.snp_ltd_dev(seqs.data_ptr(), incs.data_ptr(), n, L, W, D0.data_ptr())
    del seqs, incs
    D = torch.empty_like(D0)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    devs = {}
    for spec in runs:
        k, _, kv = spec.partition(":")
        k = int(k)
        env = dict(x.split("=", 1) for x in kv.split(",") if x)
        old = {v: os.environ.get(v) for v in env}
        os.environ.update(env)
        if k not in devs:
            devs[k] = cg.Device(0)
            if k < ncu:
                devs[k].configure(cu_mask=list(range(k)), nosync=True)
        tdev = devs[k]
        out = {"n": n, "tree_cus": k, "env": env}
        for prof in (False, True):
            D.copy_(D0)
            torch.cuda.synchronize()
            _, _, _, st = tdev.tree_dev(D.data_ptr(), n, method=cg.CCG_TREE_DNJ, exact=True, profile=prof)
            if prof:
                out["us_per_join"] = {name: round(st[5 + 2 * c] / 1e3 / max(n - 3, 1), 2)
                                      for c, name in enumerate(KNAMES) if st[4 + 2 * c]}
                out["launches_per_join"] = {name: round(st[4 + 2 * c] / max(n - 3, 1), 2)
                                            for c, name in enumerate(KNAMES) if st[4 + 2 * c]}
            else:
                out["tree_device_s"] = round(st[3] / 1e6, 3)
        print(json.dumps(out), flush=True)
        for v, x in old.items():
            if x is None:
                os.environ.pop(v, None)
            else:
                os.environ[v] = x


if __name__ == "__main__":
    main()
