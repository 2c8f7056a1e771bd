"""Per-kernel DNJ profile on config-3-like (clade-structured) data, plus the
serial reference's rescan counts (oracle) for the same matrix."""
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import torch  # noqa: E402
import ccphylo_amd as cg  # noqa: E402
from ccphylo_amd import native as nt  # noqa: E402
from tools.config3 import make_packed  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8000
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    oracle = "--oracle" in sys.argv
    dev = cg.Device(0)
    W = L // 32 + 1
    seqs = make_packed(torch, n, W)
    incs = torch.full((W,), -1, dtype=torch.int32, device="cuda")
    incs[(L + 31) // 32:] = 0
    m = n * (n - 1) // 2
    D = torch.empty(m, dtype=torch.float64, device="cuda")
    dev.snp_ltd_dev(seqs.data_ptr(), incs.data_ptr(), n, L, W, D.data_ptr())
    Dh = D.cpu().numpy().copy()
    import hashlib
    print("D md5", hashlib.md5(Dh.tobytes()).hexdigest(), "seqs md5",
          hashlib.md5(seqs.cpu().numpy().tobytes()).hexdigest(), flush=True)
    for exact in (False, True):
        D.copy_(torch.from_numpy(Dh).cuda())
        t = time.perf_counter()
        j, fn, fd, st = dev.tree_dev(D.data_ptr(), n, method=1, exact=exact, profile=True)
        dt = time.perf_counter() - t
        print(f"exact={exact}: {len(j)} joins {dt:.3f} s ({len(j) / dt:.0f}/s) rows {st[0]} cells {st[1]} "
              f"launches {st[2]}", flush=True)
        for c, name in enumerate(nt.KSTAT_NAMES):
            cnt, ns = st[4 + 2 * c], st[5 + 2 * c]
            if cnt:
                print(f"   {name:12s} {cnt:8d} x {ns / cnt / 1e3:9.2f} us = {ns / 1e9:.3f} s")
        print(f"   cells top/rest: {st[4 + 2 * nt.NKSTAT]} / {st[5 + 2 * nt.NKSTAT]}")
    if oracle:
        from oracle import pyoracle
        t = time.perf_counter()
        rj, rfn, rfd, rst = pyoracle.tree(Dh, n, method=1, stats=True)
        dt = time.perf_counter() - t
        print(f"oracle: {dt:.2f} s rows {rst[0]} cells {rst[1]}; joins equal to exact GPU: "
              f"{bool((rj['i'] == j['i']).all() and (rj['j'] == j['j']).all())}", flush=True)


if __name__ == "__main__":
    main()
