"""World-8 rehearsal of the sharded pipeline at n ~ 20k on one GPU (VERDICT
r01 item 6): `ccphylo dist ... --tree --gpus 8 --transport host` (8 rank
threads sharing the device, host-memory collectives) against `--gpus 1`,
Newick compared byte for byte, for DNJ and NJ.

    python tools/rehearse_world8.py [n] [L]

Writes a clade-structured random FASTA under $TMPDIR (n taxa, L bp)."""
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "ccphylo_amd", "bin", "ccphylo")


def write_fasta(path, n, L, seed=7):
    rng = np.random.default_rng(seed)
    lut = np.frombuffer(b"ACGT", dtype=np.uint8)
    base = rng.integers(0, 4, L)
    clades = [base.copy() for _ in range(32)]
    for c in clades:
        idx = rng.integers(0, L, L // 20)
        c[idx] = rng.integers(0, 4, len(idx))
    with open(path, "wb") as f:
        for k in range(n):
            s = clades[k % 32].copy()
            idx = rng.integers(0, L, L // 100)
            s[idx] = rng.integers(0, 4, len(idx))
            f.write(b">t%d\n" % k + lut[s].tobytes() + b"\n")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
    with tempfile.TemporaryDirectory() as td:
        fa = os.path.join(td, "m.fsa")
        t = time.perf_counter()
        write_fasta(fa, n, L)
        print(f"FASTA {n} x {L} written in {time.perf_counter() - t:.1f} s", flush=True)
        ok = True
        for method in ("dnj", "nj"):
            outs = {}
            for g in (1, 8):
                out = os.path.join(td, f"{method}{g}.nwck")
                t = time.perf_counter()
                p = subprocess.run([CLI, "dist", "-i", fa, "--tree", out, "--tree_method", method, "--gpus", str(g),
                                    "--transport", "host"], capture_output=True, timeout=900)
                dt = time.perf_counter() - t
                if p.returncode:
                    print(f"{method} --gpus {g}: rc {p.returncode}: {p.stderr.decode()[-800:]}", flush=True)
                    sys.exit(1)
                outs[g] = open(out, "rb").read()
                print(f"{method} --gpus {g}: {dt:.1f} s, Newick {len(outs[g])} bytes", flush=True)
            same = outs[1] == outs[8]
            ok = ok and same
            print(f"{method}: world 8 Newick identical to world 1: {same}", flush=True)
    sys.exit(0 if ok else 2)


if __name__ == "__main__":
    main()
