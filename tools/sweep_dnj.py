"""DNJ joins/s at N (default 10k) over engine knobs (development aid).

    python tools/sweep_dnj.py N "CCG_SEG_MUL=1 CCG_SCAN_MAX=2048" "CCG_SEG_MUL=2 CCG_SCAN_MAX=1024" ...

Every configuration runs in this one process (the engine reads its
environment knobs at each tree run): fast and exact row sums, best of 2,
and the per-kernel HIP-event averages of a profiled run."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ccphylo_amd as cg  # noqa: E402
from tools.synth import euclid  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
cfgs = sys.argv[2:] or [""]
method = cg.CCG_TREE_NJ if os.environ.get("SWEEP_METHOD") == "nj" else cg.CCG_TREE_DNJ
dev = cg.Device(0)
if os.environ.get("SWEEP_DATA") == "c2":   # the bench headline's alignment at this n (configs[2] data)
    import torch
    from bench import make_headline_alignment
    seqs, incs, W = make_headline_alignment(torch, n, 5_000_000)
    Dd = torch.empty(n * (n - 1) // 2, dtype=torch.float64, device="cuda")
    dev.snp_ltd_dev(seqs.data_ptr(), incs.data_ptr(), n, 5_000_000, W, Dd.data_ptr())
    D = Dd.cpu().numpy()
    del seqs, incs, Dd
    torch.cuda.empty_cache()
else:
    D = euclid(n)
modes = (True,) if os.environ.get("SWEEP_EXACT_ONLY") else (False, True)
reps = int(os.environ.get("SWEEP_REPS", "2"))
ref = None
for cfg in cfgs:
    env = dict(kv.split("=") for kv in cfg.split())
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    out = []
    for exact in modes:
        best = 0.0
        for _ in range(reps):
            j, fn, fd, st = dev.tree(D, n, method=method, exact=exact)
            best = max(best, len(j) / (st[3] / 1e6))
        if exact:
            key = (j["i"].tobytes(), j["j"].tobytes(), j["Li"].tobytes(), j["Lj"].tobytes())
            same = "ref" if ref is None else ("same" if key == ref else "DIFFERENT")
            ref = ref or key
        _, _, _, sp = dev.tree(D, n, method=method, exact=exact, profile=True)
        parts = [f"{nm} {sp[5 + 2 * c] / sp[4 + 2 * c] / 1e3:.1f}" for c, nm in enumerate(cg.native.KSTAT_NAMES)
                 if sp[4 + 2 * c] and nm != "init"]
        nk = cg.native.NKSTAT
        out.append(f"{'exact' if exact else 'fast'} {best:8.0f} j/s [{', '.join(parts)}] serial {sp[6 + 2 * nk]} "
                   f"chain {sp[7 + 2 * nk]}")
    print(f"{cfg or 'default':40s} " + " | ".join(out) + f" joins {same}; rows {st[0]} cells {st[1]}", flush=True)
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
