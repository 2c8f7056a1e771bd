"""End-to-end `ccphylo tree` on an N-taxon Phylip file: this CLI (GPU) vs the
reference binary (oracle/_ref, when present).  Prints the stderr timing lines."""
import os
import subprocess
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ccphylo_amd as cg  # noqa: E402
from tools.synth import euclid  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
D = euclid(n, seed=1)
with tempfile.TemporaryDirectory(dir="/tmp") as td:
    path = os.path.join(td, "m.phy")
    t = time.perf_counter()
    cg.native.write_phylip(path, D, n, [f"t{k}" for k in range(n)])
    print(f"write {time.perf_counter() - t:.2f} s, {os.path.getsize(path) / 1e6:.0f} MB", flush=True)
    runs = [("gpu", [cg.CLI_PATH, "tree", "-i", path]), ("gpu-fast", [cg.CLI_PATH, "tree", "-i", path, "--fast_sums"])]
    ref = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref", "ccphylo")
    if os.path.exists(ref) and "--noref" not in sys.argv:
        runs.append(("reference", [ref, "tree", "-i", path]))
    outs = {}
    for tag, cmd in runs:
        t = time.perf_counter()
        p = subprocess.run(cmd, capture_output=True)
        dt = time.perf_counter() - t
        outs[tag] = p.stdout
        print(f"{tag:10s} wall {dt:.2f} s rc {p.returncode} | " + " | ".join(p.stderr.decode().strip().splitlines()[-2:]),
              flush=True)
    if "reference" in outs:
        print("gpu == reference bytes:", outs["gpu"] == outs["reference"])
