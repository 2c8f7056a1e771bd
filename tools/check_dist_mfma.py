"""The MFMA forms of the non-pair SNP distance (k_snp_mfma2, CCG_DIST_MFMA=2,
the default; k_snp_mfma, 1) against the VALU tile kernel (k_snp_tile, 0) on the same device-resident random
MSA (development aid; the engine reads CCG_DIST_MFMA once per process, so
each mode runs in its own child process):
    python tools/check_dist_mfma.py [N] [L] [seed]
Prints both rates and whether the LT matrices are bit-identical."""
import os
import subprocess
import sys

CHILD = r"""
import sys, time, hashlib
sys.path.insert(0, {root!r})
import torch
import ccphylo_amd as cg
n, L, seed = {n}, {L}, {seed}
torch.cuda.set_device(0)
dev = cg.Device(0)
W = L // 32 + 1
g = torch.Generator(device="cuda").manual_seed(seed)
seqs = torch.randint(-2**62, 2**62, (n, W), dtype=torch.int64, device="cuda", generator=g)
# a third of the positions identical over all taxa, so distances spread
seqs[:, : W // 3] = seqs[0, : W // 3]
incs = torch.full((W,), -1, dtype=torch.int32, device="cuda")
incs[(L + 31) // 32:] = 0
if L % 32:
    incs[(L + 31) // 32 - 1] = ((0xFFFFFFFF << (32 - L % 32)) & 0xFFFFFFFF) - (1 << 32)
incs[W // 2] = 0x0F0F0F0F   # some excluded positions
m = n * (n - 1) // 2
D = torch.empty(m, dtype=torch.float64, device="cuda")
dev.snp_ltd_dev(seqs.data_ptr(), incs.data_ptr(), n, L, W, D.data_ptr())
best = 1e9
for _ in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dev.snp_ltd_dev(seqs.data_ptr(), incs.data_ptr(), n, L, W, D.data_ptr())
    torch.cuda.synchronize()
    best = min(best, time.perf_counter() - t0)
h = hashlib.sha256(D.cpu().numpy().tobytes()).hexdigest()
print(f"RESULT {{best:.5f}} {{m / best:.4e}} {{h}} {{float(D.min())}} {{float(D.max())}}", flush=True)
"""


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {}
    for mode in ("0", "1", "2"):
        env = dict(os.environ, CCG_DIST_MFMA=mode)
        p = subprocess.run([sys.executable, "-c", CHILD.format(root=root, n=n, L=L, seed=seed)], env=env,
                           capture_output=True, text=True, timeout=600)
        line = [x for x in p.stdout.splitlines() if x.startswith("RESULT")]
        if p.returncode or not line:
            print(f"mode {mode} failed (rc {p.returncode}):\n{p.stderr[-2000:]}", flush=True)
            sys.exit(1)
        _, t, rate, h, dmin, dmax = line[0].split()
        out[mode] = h
        print(f"{ {'0': 'VALU', '1': 'MFMA 128', '2': 'MFMA 256'}[mode]}: N={n} L={L}: {float(t):.4f} s, {float(rate):.3e} taxa-pairs/s, "
              f"{float(rate) * L:.3e} nt-comparisons/s, D in [{dmin}, {dmax}]", flush=True)
    same = out["0"] == out["1"] == out["2"]
    print("identical:", same, flush=True)
    sys.exit(0 if same else 2)


if __name__ == "__main__":
    main()
