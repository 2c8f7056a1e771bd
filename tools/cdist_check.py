"""The two configs[3] generators against numpy at small n: the same points
(CPU generator, seed 4), distances in float64 by numpy, both GPU forms
stored as float32.  Prints max |difference|, the count of cells that differ
and of zero cells, per generator (development aid: which LT the `cdist`
runs of a round actually built).

    python tools/cdist_check.py [n]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    from tools.synth import euclid_shard_dev
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    g = torch.Generator().manual_seed(4)
    pts = torch.rand((n, 8), generator=g, dtype=torch.float64).numpy()
    i, j = np.tril_indices(n, -1)
    ref = np.sqrt(((pts[i] - pts[j]) ** 2).sum(1)).astype(np.float32)
    for cd in (False, True):
        got = euclid_shard_dev(torch, n, 0, 1, dtype=torch.float32, cdist=cd).cpu().numpy()
        diff = np.abs(got.astype(np.float64) - ref.astype(np.float64))
        print(json.dumps({"n": n, "generator": "cdist" if cd else "elementwise", "max_abs_diff": float(diff.max()),
                          "cells_differing": int((got != ref).sum()), "zero_cells": int((got == 0).sum()),
                          "cells": int(got.size), "first": got[:4].tolist(), "ref_first": ref[:4].tolist()}),
              flush=True)


if __name__ == "__main__":
    main()
