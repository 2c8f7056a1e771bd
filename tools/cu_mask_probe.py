"""Does a CU-masked engine context leave the process's GPU runtime usable
for torch after it is destroyed?  (development aid: round 5's bench crashed
in torch elementwise ops after the pipelined leg)

    python tools/cu_mask_probe.py [close|keep|nomask]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "close"
    import numpy as np
    import torch
    import ccphylo_amd as cg
    from tools.synth import euclid, euclid_shard_dev
    n = 3000
    D = euclid(n)
    dev = cg.Device(0)
    t = cg.Device(0)
    if mode != "nomask":
        t.configure(cu_mask=list(range(64)), nosync=True)
    j, fn, fd, _ = t.tree(D, n, method=cg.CCG_TREE_DNJ, exact=True)
    if mode != "keep":
        t.close()
    print(f"{mode}: tree on the masked context, {len(j)} joins", flush=True)
    t0 = time.perf_counter()
    loc = euclid_shard_dev(torch, 200_000, 0, 1, dtype=torch.float32)
    torch.cuda.synchronize()
    print(f"{mode}: torch after it: {loc.numel()} cells in {time.perf_counter() - t0:.1f} s", flush=True)
    del loc
    j2 = dev.tree(D, n, method=cg.CCG_TREE_DNJ, exact=True)[0]
    print(f"{mode}: whole-chip context after it: same joins {bool((j2 == j).all())}", flush=True)


if __name__ == "__main__":
    main()
