"""MSA loader speed: the serial ccq_load_msa against the parallel
ccq_load_msa_par on a random n x L FASTA (development aid; DESIGN.md
"Host I/O fast paths").

    python tools/bench_loader.py [n] [L] [threads...]

Writes the FASTA under $TMPDIR (60-column lines), loads it once to warm the
page cache, then times each loader and checks that the results agree."""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import ccphylo_amd as cg  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
L = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
threads = [int(t) for t in sys.argv[3:]] or [16]
rng = np.random.default_rng(1)
lut = np.frombuffer(b"ACGT", dtype=np.uint8)
with tempfile.TemporaryDirectory() as td:
    path = os.path.join(td, "bench.fsa")
    t0 = time.perf_counter()
    base = lut[rng.integers(0, 4, L)]
    with open(path, "wb") as f:
        for k in range(n):
            s = base.copy()
            idx = rng.integers(0, L, L // 100)
            s[idx] = lut[rng.integers(0, 4, len(idx))]
            s[rng.integers(0, L, 20)] = ord("N")
            body = s.tobytes()
            f.write(b">t%d\n" % k + b"\n".join(body[i:i + 60] for i in range(0, L, 60)) + b"\n")
    size = os.path.getsize(path)
    print(f"wrote {n} x {L} FASTA, {size / 1e9:.2f} GB in {time.perf_counter() - t0:.1f} s", flush=True)
    with open(path, "rb") as f:
        while f.read(1 << 26):
            pass
    t0 = time.perf_counter()
    ref = cg.load_msa(path, 1, 1, 0.5, 0)
    ts = time.perf_counter() - t0
    print(f"serial ccq_load_msa: {ts:.2f} s ({size / ts / 1e9:.2f} GB/s)", flush=True)
    for t in threads:
        t0 = time.perf_counter()
        got = cg.load_msa(path, 1, 1, 0.5, 0, threads=t)
        tp = time.perf_counter() - t0
        same = ref[0] == got[0] and (ref[1] == got[1]).all() and (ref[2] == got[2]).all() and ref[3:] == got[3:]
        print(f"ccq_load_msa_par, {t} threads: {tp:.2f} s ({size / tp / 1e9:.2f} GB/s), {ts / tp:.1f}x the serial; "
              f"identical {same}", flush=True)
