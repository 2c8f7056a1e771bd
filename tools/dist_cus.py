"""The headline dist alone on a CU-masked context of k CUs (bits 256 - k ..
255 of the mask, as pipelined_leg gives the dist), nothing beside it: does
the dist in the pipeline lose time to the tree beside it (power, HBM) or to
its 192 CUs?  Prints one JSON line per k: k_snp_mfma3's device ms (HIP
events on the context's stream).

    python tools/dist_cus.py [n] [L] [k ...]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import ccphylo_amd as cg
    from bench import make_headline_alignment
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 5_000_000
    ks = [int(x) for x in sys.argv[3:]] or [256, 192, 128]
    seqs, incs, W = make_headline_alignment(torch, n, L)
    D = torch.empty(n * (n - 1) // 2, dtype=torch.float64, device="cuda")
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    for k in ks:
        dev = cg.Device(0)
        if k < ncu:
            dev.configure(cu_mask=list(range(ncu - k, ncu)), nosync=True)
        dev.snp_ltd_dev(seqs.data_ptr(), incs.data_ptr(), n, L, W, D.data_ptr())
        ms = dev.last_dist_ms()
        print(json.dumps({"n": n, "L": L, "dist_cus": k, "dist_ms": round(ms, 1)}), flush=True)
        dev.close()


if __name__ == "__main__":
    main()
