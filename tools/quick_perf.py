"""Quick GPU timing of the engine (development aid, not the bench)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import ccphylo_amd as cg
from tools.synth import euclid


n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
what = sys.argv[2] if len(sys.argv) > 2 else "all"
t = time.time(); D = euclid(n); print(f"gen {time.time()-t:.1f}s", flush=True)
dev = cg.Device(0)
print(dev.info())
for method, exact in [(1, True), (1, False), (0, True)]:
    if what != "all" and what != ("dnj" if method else "nj"):
        continue
    t = time.time()
    joins, fn, fd, st = dev.tree(D, n, method=method, exact=exact)
    w = time.time() - t
    _, _, _, sp = dev.tree(D, n, method=method, exact=exact, profile=True)
    parts = []
    for c, name in enumerate(cg.native.KSTAT_NAMES):
        if sp[4 + 2 * c]:
            parts.append(f"{name} {sp[5 + 2 * c] / sp[4 + 2 * c] / 1e3:.2f}us x{sp[4 + 2 * c]}")
    print("   per-kernel avg: " + ", ".join(parts), flush=True)
    print(f"{'dnj' if method else 'nj'} exact={exact}: wall {w:.3f}s device {st[3]/1e6:.3f}s joins {len(joins)} "
          f"-> {len(joins)/(st[3]/1e6):.0f} joins/s; rows {st[0]} cells {st[1]} launches {st[2]}", flush=True)
# dist
for (N, L, pair) in [(2048, 100000, False), (1024, 100000, True)]:
    W = L // 32 + 1
    rng = np.random.default_rng(1)
    seqs = rng.integers(0, 2**63, size=(N, W), dtype=np.uint64)
    incs = np.full((N, W) if pair else W, 0xFFFFFFFF, np.uint32)
    t = time.time()
    Dd, _, _ = dev.snp_ltd(seqs, incs, N, L, pair=pair)
    w = time.time() - t
    pairs = N * (N - 1) / 2
    print(f"dist N={N} L={L} pair={pair}: wall {w:.3f}s -> {pairs/w:.3e} pairs/s, {pairs*L/w:.3e} nt-cmp/s (incl. H2D/D2H)", flush=True)
