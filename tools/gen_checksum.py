"""Is a configs[3] generator deterministic?  Builds the 200k float LT twice
per generator (elementwise, torch.cdist) in one process and prints exact
order-independent checksums of its bit patterns (int64 sums of the int32
words and of word x (index mod 2^16)), so two runs, or two boxes, can be
compared without moving 80 GB.

    python tools/gen_checksum.py [n] [reps]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def checksum(torch, t):
    w = t.view(torch.int32)
    s1, s2 = 0, 0
    step = 1 << 28
    for a in range(0, w.numel(), step):
        x = w[a:a + step].to(torch.int64)
        idx = torch.arange(a, a + x.numel(), device=x.device, dtype=torch.int64) & 0xFFFF
        s1 += int(x.sum().item())
        s2 += int((x * idx).sum().item())
    return s1, s2


def main():
    import torch
    from tools.synth import euclid_shard_dev
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    for cd in (False, True):
        for r in range(reps):
            loc = euclid_shard_dev(torch, n, 0, 1, dtype=torch.float32, cdist=cd)
            torch.cuda.synchronize()
            print(json.dumps({"n": n, "generator": "cdist" if cd else "elementwise", "rep": r,
                              "checksum": checksum(torch, loc)}), flush=True)
            del loc
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
