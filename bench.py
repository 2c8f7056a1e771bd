#!/usr/bin/env python3
"""bench.py -- headline benchmark of ccphylo_amd (driver contract).

Metric (BASELINE.json): "taxa-pairs/sec (dist) + NJ iterations/sec at N taxa".
The headline workload is configs[2], the largest single-GPU configuration
with both halves of the metric: a 50k-taxon x 5 Mbp synthetic tree-like
alignment, packed in HBM, -> `ccphylo dist` (all-pairs SNP counts, the full
LT) -> `ccphylo tree -m dnj` with exact row sums (bit-identical to the
reference), in place.  A step is the whole pipeline on the resident packed
alignment (the tree consumes the LT, so every step recomputes it); `value`
is taxa pairs per second of that pipeline, n(n-1)/2 / step time, and the
line carries its split (dist taxa-pairs/s, NJ iterations/s).

Multi-GPU (torchrun, one process per GPU, N > 1): the SAME matrix sharded:
dist writes each rank's LT row bands (ccg_snp_ltd_shard_dev) and the sharded
DNJ (ccg_tree_shard_dev, exact) consumes them over RCCL -- strong scaling of
one pipeline, `scaling: "strong"`.  `joins_sha256` is the hash of the join
list, identical for every N when the sharded tree equals the single-GPU one.

Roofline: the dominant kernel by device time of the step (the MFMA dist
kernel at N = 1; its duration from HIP events on the engine stream,
ccg_last_dist_ms), with every tree kernel class beside it (HIP events of a
profiled step); `traffic` from the committed rocprofv3 PMC summary.
cpu_baseline: the reference binary (oracle/_ref, built from the reference's
sources) running the same pipeline (`dist -t <nproc>` then `tree`) on the
first taxa of the same alignment, whose distances and Newick are compared
with the GPU's.

SURVEY 8(d) prices the DNJ rescans by the cells the REFERENCE's minQpair
rule rescans: the engine counts them from its replay decisions (stats[10/11
+ 2 NKSTAT]); `split.reference_rule_cells` is the whole headline tree's, and
the scan kernels report `frac_reference_rule` beside the engine-cell `frac`.

extras: configs[1] (N = 10k Phylip matrix: DNJ exact and fast, NJ, HNJ, with
the reference's DNJ and NJ on the host), the oracle's serial count of the
reference-rule cells at configs[1] and on a configs[2] prefix (checks the
engine's counters), dist alone at 8192 x 1 Mbp (non-pair and pair mode), KMA
`cos`, configs[3] (one 200k float matrix, exact DNJ, a 20k-join prefix by
default -- the whole tree is profiles/r03_config3_whole_tree.json: the
single-GPU engine at N = 1, sharded over RCCL at N > 1) and the sharded NJ.
"""
import argparse
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
# VALU dist kernel (k_snp_tile, CCG_DIST_MFMA=0; the MFMA kernels below are
# the default): 32-bit integer VALU issue.  A 32-position word pair costs 3
# instructions (v_xor, v_bitop3, v_bcnt with accumulate).  Nominal peak
# (MI355X_MICROARCH.md): 256 CUs x 4 SIMD-32 x 32 lanes/clk x 2.4 GHz =
# 7.86e13 instruction-lanes/s (`peak`, `frac`).  Measured on gfx950
# (profiles/r02_valu_mix.txt, profiles/r02_pmc_dist.json): these wave64
# integer instructions issue once per ~4 cycles per SIMD (16 lanes/clk), each
# alone as in the mix, so their ceiling is half the nominal: 256 x 4 x 16 x
# 2.4e9 = 3.93e13 (`int32_wave64_ceiling`, `frac_of_int32_ceiling`).
VALU_NOMINAL_LANE_OPS = 256 * 4 * 32 * 2.4e9
# Non-pair dist runs on the matrix cores (k_snp_mfma, the default): a code is
# the tetrahedron vector (+-1)^3 in MX-fp4, 3 MACs = 6 flops per position pair
# (dist = (3 L - dot) / 4, exact).  Peak: the MX-fp4 dense rate, ~10 PF
# (MI355X_MICROARCH.md).  Measured ceiling: tools/micro/mfma_valu
# (profiles/r06_mfma_valu.txt) issues register-fed fp4 MFMAs, 16 accumulators
# per wave, at 3.60e15 MAC/s = 7.2 PF sustained (one MFMA per 32.8 cycles at
# the ~1.76 GHz the chip holds under that load; round 2's tools/micro/mfma_fp4,
# 4 accumulators: 7.1 PF).
MFMA_FP4_DENSE_TFLOPS = 10000.0
MFMA_FP4_MEASURED_TFLOPS = 7202.0
FLOPS_PER_POSITION_PAIR = 6.0
VALU_INT32_CEILING = 256 * 4 * 16 * 2.4e9
OPS_PER_WORD_PAIR = 3.0
OPS_PER_WORD_PAIR_PAIRMODE = 6.0   # v_and (masks), v_xor, v_bitop3, v_and, 2x v_bcnt (dist and n)
KNAMES = ["init", "dnj_select", "dnj_scan", "nj_argmin", "update", "dnj_requeue", "nj_pop", "dnj_find", "coll",
          "exact_sum"]
def _latest(*names):
    """The newest committed profile of a kind (this round's, else the last)."""
    for nm in names:
        p = os.path.join(ROOT, "profiles", nm)
        if os.path.exists(p):
            return p
    return os.path.join(ROOT, "profiles", names[-1])


PMC_SUMMARY = _latest("r06_pmc.json", "r05_pmc.json", "r04_pmc.json", "r03_pmc.json", "r02_pmc.json")
PMC_HEADLINE = _latest("r06_pmc_headline.json", "r05_pmc_headline.json", "r04_pmc_headline.json", "r03_pmc_headline.json")
SHARD_LEG_TIMEOUT_S = 600
HEADLINE_TIMEOUT_S = 1200


_LEG = ["start"]
_T0 = time.perf_counter()


def log(msg):
    """Progress on stderr (the JSON line is the only stdout)."""
    _LEG[0] = msg
    print(f"[bench {time.perf_counter() - _T0:7.1f} s] {msg}", file=sys.stderr, flush=True)


def start_heartbeat(every=45.0):
    """A line every `every` seconds while a long leg runs (a single call such
    as the oracle's prefix or a whole tree may take minutes)."""
    import threading

    def beat():
        while True:
            time.sleep(every)
            print(f"[bench {time.perf_counter() - _T0:7.1f} s] ... {_LEG[0]}", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()


def host_cpus():
    """CPUs this process may run on, and the cgroup CPU quota (cpu.max) when
    one limits it (the GPU box reports every host CPU but grants a share)."""
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            if q != "max":
                quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return ncpu, quota


def effective_cores():
    """The CPUs a CPU baseline can actually use: the affinity set, capped by
    the cgroup quota (the GPU box lists every host CPU but grants 16)."""
    import math
    ncpu, quota = host_cpus()
    return max(1, min(ncpu, math.ceil(quota))) if quota else ncpu


from tools.synth import euclid as euclid_ltd  # noqa: E402


def algorithmic_bytes_total(kernel, n, s, cells_select, cells_scan, cells_help=0):
    """Compulsory HBM bytes of all launches of one class over a whole tree
    (joins at matrix sizes n .. 3); DESIGN.md, 'Roofline accounting'.
    s = bytes per D element; the n-vectors are f64 (sD, Q) and i32 (N, P).
    cells_help: the S cells k_dnj_plan's helper blocks rescanned (pruning,
    single engine, stats[8 + 2 NKSTAT]): the plan's bytes, not the scan's."""
    sizes = range(3, n + 1)
    sn = float(sum(sizes))
    if kernel == "dnj_select":      # (sharded engine) rescanned D cells of S + the sD vector once
        return s * cells_select + 8.0 * sn
    if kernel == "dnj_scan":        # one GPU: every rescanned D cell (S and the rows below it) + the sD vector once
        return s * (cells_select + cells_scan - cells_help) + 8.0 * sn
    if kernel == "dnj_scan_ref":    # the cells the reference's minQpair rule rescans (cells_scan)
        return s * cells_scan + 8.0 * sn
    if kernel == "dnj_find":        # k_dnj_plan: Q of every row; P, the partner cell, sD of row and partner
        # for the top rows; the helpers' S rescans (row cells + the sD gathers per cell)
        return 8.0 * sn + (20.0 + s) * float(sum(min(k - 1, 960) for k in sizes)) + (s + 8.0) * cells_help
    if kernel == "nj_argmin":       # every LT cell + sD
        return sum(s * k * (k - 1) / 2 + 8.0 * k for k in sizes)
    if kernel == "update":          # D_ik, D_kj read, D_kj written; sD, N read+written
        return (3.0 * s + 24.0) * sn
    if kernel == "dnj_requeue":     # row/col j, row n-1 read; row/col i written; Q, P, sD, N
        return (4.0 * s + 36.0) * sn
    if kernel == "nj_pop":          # row n-1 read, row/col i written
        return 2.0 * s * sn
    if kernel == "init":            # two passes over the LT
        return 2.0 * s * n * (n - 1) / 2
    if kernel == "exact_sum":       # the new row's contributions, read once (+ the update partials)
        return 8.0 * sn + 32.0 * sum((k + 255) // 256 for k in sizes)
    return 0.0


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (FETCH_SIZE and WRITE_SIZE passes, corrected as MI355X_MICROARCH.md says)."""
    try:
        with open(PMC_SUMMARY) as f:
            d = json.load(f)
        k = d["kernels"].get(kernel)
        return (k["hbm_bytes_per_launch"], d["source"]) if k else (None, None)
    except (OSError, KeyError, ValueError):
        return None, None


KERNEL_STATS = _latest("r06_kernel_stats.csv", "r05_kernel_stats.csv", "r04_kernel_stats.csv", "r03_kernel_stats.csv", "r02_kernel_stats.csv")
KSYM = {"dnj_select": "k_dnj_select", "dnj_scan": "k_dnj_scan", "dnj_find": "k_dnj_plan", "update": "k_dnj_join",
        "dnj_requeue": "k_dnj_requeue", "nj_argmin": "k_nj_argmin", "nj_pop": "k_nj_pop", "exact_sum": "k_exact_sum"}


def rocprof_mean_us(kernel):
    """Mean kernel duration of `kernel` in the committed rocprofv3
    --kernel-trace --stats summary (begin to end of the dispatch)."""
    import csv
    sym = KSYM.get(kernel)
    try:
        with open(KERNEL_STATS) as f:
            for r in csv.DictReader(f):
                if sym and r["Name"].replace("void ", "").startswith(sym + "<"):
                    return round(float(r["AverageNs"]) / 1e3, 3)
    except (OSError, KeyError, ValueError):
        pass
    return None


def refrule_scan(stats, n, s, launches, sec_per_launch):
    """The scan's rate by SURVEY 8(d)'s unit: the cells the reference's own
    minQpair rule rescans (the engine counts them from its replay decisions,
    stats[11 + 2 NKSTAT]) instead of the engine's speculative cells."""
    K = len(KNAMES)
    if len(stats) < 12 + 2 * K or not stats[11 + 2 * K]:
        return {}
    ab = algorithmic_bytes_total("dnj_scan_ref", n, s, 0, stats[11 + 2 * K]) / launches
    return {"reference_rule_rows": int(stats[10 + 2 * K]), "reference_rule_cells": int(stats[11 + 2 * K]),
            "engine_cells": int(stats[4 + 2 * K] + stats[5 + 2 * K]),
            "engine_over_reference_cells": round((stats[4 + 2 * K] + stats[5 + 2 * K]) / stats[11 + 2 * K], 3),
            "algorithmic_bytes_per_launch_reference_rule": round(ab, 1),
            "frac_reference_rule": round(ab / sec_per_launch / 1e9 / HBM_PEAK_GBS, 5)}


def roofline(stats, n, s):
    """Dominant kernel (largest total device time) of a profiled run."""
    per = {}
    for c, name in enumerate(KNAMES):
        cnt, ns = stats[4 + 2 * c], stats[5 + 2 * c]
        if cnt:
            per[name] = (cnt, ns)
    name = max(per, key=lambda k: per[k][1])
    cnt, ns = per[name]
    K = len(KNAMES)
    ch = stats[8 + 2 * K] if len(stats) > 8 + 2 * K else 0   # single engine only (sharded: init bytes)
    tot = algorithmic_bytes_total(name, n, s, stats[4 + 2 * K], stats[5 + 2 * K], ch)
    avg_s = ns / cnt / 1e9
    achieved = tot / cnt / avg_s / 1e9
    shares = {k: round(v[1] / sum(x[1] for x in per.values()), 4) for k, v in per.items()}
    kernels = {}
    for k, (c, t) in per.items():   # every kernel class: algorithmic bytes, HIP-event and rocprof rates, PMC bytes
        if k == "init":
            continue
        ab = algorithmic_bytes_total(k, n, s, stats[4 + 2 * K], stats[5 + 2 * K], ch) / c
        ev = t / c / 1e9
        rp = rocprof_mean_us(k)
        kernels[k] = {"algorithmic_bytes_per_launch": round(ab, 1), "avg_launch_us": round(ev * 1e6, 3),
                      "frac": round(ab / ev / 1e9 / HBM_PEAK_GBS, 5), "traffic": pmc_traffic(k)[0]}
        if rp:
            kernels[k]["rocprof_mean_us"] = rp
            kernels[k]["frac_rocprof_duration"] = round(ab / (rp * 1e-6) / 1e9 / HBM_PEAK_GBS, 5)
        if k == "dnj_scan":
            kernels[k].update(refrule_scan(stats, n, s, c, ev))
    traffic, src = pmc_traffic(name)
    out = {"kernel": name, "bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
           "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
           "traffic": traffic, "avg_launch_us": round(avg_s * 1e6, 3), "launches": cnt,
           "algorithmic_bytes_per_launch": round(tot / cnt, 1), "time_shares": shares, "kernels": kernels}
    if src:
        out["traffic_source"] = src
    rp = rocprof_mean_us(name)
    if rp:
        # HIP events on the engine stream are stamped when the previous event
        # and the kernel complete, so avg_launch_us also holds the dependent
        # dispatch gap before the kernel (2-4 us here); rocprofv3 times the
        # dispatch from begin to end.  frac uses the event time (conservative).
        out["rocprof_mean_us"] = rp
        out["frac_rocprof_duration"] = round(tot / cnt / (rp * 1e-6) / 1e9 / HBM_PEAK_GBS, 5)
        out["timing_note"] = ("avg_launch_us: HIP events around each launch on the engine stream (includes the "
                              "dispatch gap after the previous kernel); rocprof_mean_us: rocprofv3 --kernel-trace "
                              "--stats mean of the same kernel (profiles/r02_kernel_stats.csv)")
    return out


def cpu_baseline(D, n, tmpdir, threads=None, method="dnj"):
    """The reference binary (oracle/_ref, built from /root/reference by
    oracle/Makefile) on the same matrix written as Phylip, with 1 and all
    host pthreads (`-t`); the faster is the baseline.  Falls back to the
    oracle's C restatement in-process."""
    if threads is None:
        threads = sorted({1, effective_cores()})
    ref = os.path.join(ROOT, "oracle", "_ref", "ccphylo")
    if os.path.exists(ref):
        from ccphylo_amd import native
        path = os.path.join(tmpdir, "bench_ref.phy")
        native.write_phylip(path, D, n, [f"t{k}" for k in range(n)])
        runs = {}
        for t in threads:
            t0 = time.perf_counter()
            p = subprocess.run([ref, "tree", "-i", path, "-m", method, "-t", str(t), "-o",
                                os.path.join(tmpdir, "ref.nwk" if method == "dnj" else f"ref_{method}.nwk")],
                               capture_output=True, text=True, timeout=900)
            wall = time.perf_counter() - t0
            # the reference reports clock() (CPU time summed over threads), so
            # the construction rate uses the process wall clock minus its load
            ld = re.search(r"loading matrix: ([0-9.]+) s", p.stderr)
            load = float(ld.group(1)) if ld else 0.0
            cons = max(wall - load, 1e-9) if t > 1 else None
            m = re.search(r"Constructing tree: ([0-9.]+) s", p.stderr)
            if cons is None:
                cons = float(m.group(1)) if m else wall
            runs[t] = (cons, wall, load)
        os.unlink(path)
        best = min(runs, key=lambda t: runs[t][0])
        cons, wall, load = runs[best]
        desc = "; ".join(f"-t {t}: construction {c:.2f} s, load {l:.2f} s, wall {w:.2f} s"
                         for t, (c, w, l) in sorted(runs.items()))
        ncpu, quota = host_cpus()
        return {"value": round((n - 2) / cons, 2), "unit": "NJ joins/s", "cores": best, "kind": "reference",
                "host_cpus": ncpu, "cgroup_cpu_quota": quota,
                "sample": f"full N={n} {method.upper()} tree, reference ccphylo 0.8.5 `tree -m {method}` on the same matrix "
                          f"(Phylip %.9f), best of {list(threads)} pthreads ({desc}); 1-thread time is the "
                          f"reference's own 'Constructing tree' report, multi-thread time is process wall "
                          f"minus its 'loading matrix' report"}
    from oracle import pyoracle
    t0 = time.perf_counter()
    j, _, _ = pyoracle.tree(D, n, method=1)
    dt = time.perf_counter() - t0
    return {"value": round(len(j) / dt, 2), "unit": "NJ joins/s", "cores": 1, "kind": "port",
            "sample": f"full N={n} DNJ tree with the oracle's serial C restatement (reference binary absent)"}


def cpu_baseline_dist(tmpdir, sizes=(1024, 2048), L=20_000, threads=None):
    """The reference's `ccphylo dist` (oracle/_ref, -t <host CPUs>) on random MSAs of
    `sizes` taxa x L bp (FASTA text, seeded; the data of the GPU dist leg).  The process wall time is
    parse + compare; with two sizes, t = a n + b n^2 separates the quadratic
    (compare) term, whose rate is reported as nt-comparisons/s."""
    import numpy as np
    ref = os.path.join(ROOT, "oracle", "_ref", "ccphylo")
    if not os.path.exists(ref):
        return None
    ncpu, quota = host_cpus()
    threads = threads or effective_cores()
    rng = np.random.default_rng(11)
    lut = np.frombuffer(b"ACGT", dtype=np.uint8)
    walls = {}
    for n in sizes:
        path = os.path.join(tmpdir, f"cpu_dist_{n}.fsa")
        with open(path, "wb") as f:   # random MSA, as the GPU dist leg (every word pair differs)
            for k in range(n):
                f.write(b">t%d\n" % k + lut[rng.integers(0, 4, L)].tobytes() + b"\n")
        t0 = time.perf_counter()
        subprocess.run([ref, "dist", "-i", path, "-t", str(threads), "-o", os.path.join(tmpdir, "d.phy")],
                       capture_output=True, timeout=900, check=True)
        walls[n] = time.perf_counter() - t0
        os.unlink(path)
    (n1, t1), (n2, t2) = sorted(walls.items())
    b = (t2 / n2 - t1 / n1) / (n2 - n1)          # t/n = a + b n
    pairs_s = 0.5 / b if b > 0 else None         # pairs ~ n^2 / 2
    return {"value": round(pairs_s * L, 1) if pairs_s else None, "unit": "nt-comparisons/s",
            "taxa_pairs_per_s": round(pairs_s, 1) if pairs_s else None, "cores": threads, "kind": "reference",
            "host_cpus": ncpu, "cgroup_cpu_quota": quota,
            "sample": f"reference ccphylo 0.8.5 `dist -t {threads}` on random MSAs of {list(sizes)} taxa x {L} "
                      f"bp (FASTA); walls " + ", ".join(f"n={n}: {w:.2f} s" for n, w in sorted(walls.items())) +
                      "; the rate is the quadratic (compare) term of t = a n + b n^2"}


def dist_extra(dev, torch, n=8192, L=1_000_000, reps=3, rank=0, world=1, dist=None, pair=False):
    """SNP distances (non-pair, double) with device-resident packed input.
    With world > 1 the LT rows are sharded over the ranks (SURVEY 8(e):
    pairs are independent, so no data-path collective): rank g computes rows
    shard.lt_row_ranges(n, world)[g] of the same matrix; the rate is all
    pairs over the max time over ranks (strong scaling of one matrix)."""
    from ccphylo_amd import shard
    W = L // 32 + 1
    g = torch.Generator(device="cuda").manual_seed(3)
    seqs = torch.randint(-2**62, 2**62, (n, W), dtype=torch.int64, device="cuda", generator=g)
    incs = torch.full((n, W) if pair else (W,), -1, dtype=torch.int32, device="cuda")
    incs[..., (L + 31) // 32:] = 0
    if L % 32:
        incs[..., (L + 31) // 32 - 1] = ((0xFFFFFFFF << (32 - L % 32)) & 0xFFFFFFFF) - (1 << 32)
    if pair:   # per-taxon masks with ~1/16 of the positions excluded
        incs &= torch.randint(-2**31, 2**31, incs.shape, dtype=torch.int32, device="cuda", generator=g) | 0x7FFF7FFF
    m = n * (n - 1) // 2
    r0, r1 = shard.lt_row_ranges(n, world)[rank]
    Dd = torch.empty(m, dtype=torch.float64, device="cuda")
    Nd = torch.empty(m, dtype=torch.float64, device="cuda") if pair else None
    kw = dict(row_range=(r0, r1), pair=pair, N_ptr=Nd.data_ptr() if pair else None)
    torch.cuda.synchronize()
    dev.snp_ltd_dev(seqs.data_ptr(), incs.data_ptr(), n, L, W, Dd.data_ptr(), **kw)
    times = []
    for _ in range(reps):
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        dev.snp_ltd_dev(seqs.data_ptr(), incs.data_ptr(), n, L, W, Dd.data_ptr(), **kw)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        times.append(shard.reduce_max(dt, dist) if dist is not None else dt)
    dt = min(times)
    words = (L + 31) // 32
    opw = OPS_PER_WORD_PAIR_PAIRMODE if pair else OPS_PER_WORD_PAIR
    ops = m * words * opw / world   # per GPU
    mode_env = os.environ.get("CCG_DIST_MFMA", "2")
    mfma = mode_env != "0"
    del seqs, incs, Dd, Nd
    mode = "pair mode -f 3, D and N" if pair else "non-pair"
    return {"taxa_pairs_per_s": round(m / dt, 1), "nt_comparisons_per_s": m * L / dt, "seconds": round(dt, 4),
            "config": f"N={n} x L={L} random MSA ({mode}, double), input in HBM, LT rows sharded over {world} GPU(s)",
            "kernel": (("k_snp_mfma_pair" if mode_env == "1" else "k_snp_mfma2_pair") if pair
                       else dist_kernel_name()) if mfma
            else ("k_snp_tile_pair" if pair else "k_snp_tile"),
            "roofline": mfma_roofline(m * L / world, dt, 8.0 if pair else FLOPS_PER_POSITION_PAIR) if mfma
            else valu_roofline(ops, dt, opw)}


def mfma_roofline(position_pairs, dt, flops_per_pp=FLOPS_PER_POSITION_PAIR):
    """dist on the matrix cores: 6 flops (3 MX-fp4 MACs) per position pair
    (pair mode: 8, the mask is a fourth component) against the MX-fp4 dense
    peak, and beside it the register-fed issue rate measured on this box."""
    tf = flops_per_pp * position_pairs / dt / 1e12
    return {"bound": "mfma", "achieved": round(tf, 1), "peak": MFMA_FP4_DENSE_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tf / MFMA_FP4_DENSE_TFLOPS, 4), "measured_issue_peak": MFMA_FP4_MEASURED_TFLOPS,
            "frac_of_measured_peak": round(tf / MFMA_FP4_MEASURED_TFLOPS, 4),
            "form": "tetrahedron (+-1)^3 MX-fp4 operands, v_mfma_scale_f32_32x32x64_f8f6f4, dist = (3 L - dot) / 4",
            "evidence": "profiles/r02_mfma_fp4.txt (tools/micro/mfma_fp4: lane map), profiles/r06_mfma_valu.txt "
                        "(tools/micro/mfma_valu: register-fed rate, VALU per MFMA)"}


def valu_roofline(ops, dt, opw):
    """dist: integer VALU issue (instruction-lanes/s) against the nominal
    peak, and against the measured ceiling of the kernel's instruction mix."""
    return {"bound": "valu-int", "achieved": round(ops / dt / 1e12, 3), "peak": round(VALU_NOMINAL_LANE_OPS / 1e12, 2),
            "unit": "T int instruction-lanes/s", "frac": round(ops / dt / VALU_NOMINAL_LANE_OPS, 4),
            "int32_wave64_ceiling": round(VALU_INT32_CEILING / 1e12, 2),
            "frac_of_int32_ceiling": round(ops / dt / VALU_INT32_CEILING, 4), "ops_per_word_pair": opw,
            "ceiling_evidence": "profiles/r02_valu_mix.txt (v_xor / v_or / v_bitop3 / v_bcnt alone and mixed: ~4 cycles "
                                "per wave64 instruction per SIMD) and profiles/r02_pmc_dist.json (k_snp_tile: "
                                "SQ_INSTS_VALU = 1.035 x the algorithmic 3 per word pair, 3.66 cycles per "
                                "instruction per SIMD at the 2.35 GHz GRBM_GUI_ACTIVE clock)"}


def packed_rows_to_fasta(path, words, L, masked_words):
    """FASTA text of packed 2-bit rows (qseq2nibble layout, MSB-first, codes
    0..3 = A C G T, qseqs.c:60), the positions of `masked_words` written as N
    in the first taxon only (the non-pair dist ANDs every taxon's include
    mask, cdist.c:273, so those positions drop out for all pairs)."""
    lut = np.frombuffer(b"ACGT", dtype=np.uint8)
    shifts = (62 - 2 * np.arange(32, dtype=np.uint64)).astype(np.uint64)
    with open(path, "wb") as f:
        for t in range(words.shape[0]):
            codes = ((words[t][:, None] >> shifts[None, :]) & np.uint64(3)).astype(np.uint8).reshape(-1)[:L]
            txt = lut[codes]
            if t == 0:
                txt = txt.reshape(-1)
                for w in masked_words:
                    txt[32 * w:32 * w + 32] = ord("N")
            f.write(b">t%d\n" % t + txt.tobytes() + b"\n")


def read_phylip_values(path):
    """The LT cells of a (relaxed) Phylip file as floats, row by row."""
    vals = []
    with open(path) as f:
        n = int(f.readline())
        for i in range(n):
            parts = f.readline().split()
            vals.extend(float(x) for x in parts[1:1 + i])
    return n, np.array(vals)


def headline_cpu_baseline(dev, seqs_host, incs_host, L, gpu_cells, tmpdir, m=256):
    """The reference binary's own pipeline on the first `m` taxa of the
    headline alignment (written as FASTA): `ccphylo dist -t <host CPUs>`
    then `ccphylo tree` (DNJ; its threads do not speed DNJ up, so -t 1).
    value = m(m-1)/2 / (dist wall + tree wall).  The reference's distances
    are compared with the GPU's LT cells of those taxa, and its Newick with
    the Newick the GPU builds from the same sub-matrix."""
    import ccphylo_amd as cg
    from ccphylo_amd import native
    ref = os.path.join(ROOT, "oracle", "_ref", "ccphylo")
    if not os.path.exists(ref):
        return {"error": "reference binary absent (oracle/_ref not built)"}
    ncpu, quota = host_cpus()
    cores = effective_cores()
    masked = [w for w in range((L + 31) // 32) if incs_host[w] == 0]
    fa = os.path.join(tmpdir, "head.fsa")
    phy = os.path.join(tmpdir, "head.phy")
    nwk = os.path.join(tmpdir, "head.nwk")
    packed_rows_to_fasta(fa, seqs_host[:m], L, masked)
    t0 = time.perf_counter()
    subprocess.run([ref, "dist", "-i", fa, "-t", str(cores), "-o", phy], capture_output=True, timeout=900, check=True)
    t1 = time.perf_counter()
    # -x 3: the reference's formNode (nwck.c:52-53, :75) reserves 32 bytes for
    # "(" + two ":%.*f" lengths + ",)"; at the default 9 digits a length of
    # 1000 or more overruns the buffer (heap corruption, glibc aborts on this
    # alignment's SNP counts), so both Newicks are written with 3 digits
    subprocess.run([ref, "tree", "-i", phy, "-o", nwk, "-x", "3"], capture_output=True, timeout=900, check=True)
    t2 = time.perf_counter()
    os.unlink(fa)
    nn, vals = read_phylip_values(phy)
    k = m * (m - 1) // 2
    mism = int(nn != m) + int((vals != gpu_cells[:k]).sum())
    # the GPU tree of the same sub-matrix (its LT block is the first m rows)
    trees = cg.newick_from_phylip(phy, lambda D_, n_: dev.tree(np.asarray(gpu_cells[:k], dtype=np.float64), n_,
                                                              method=cg.CCG_TREE_DNJ, exact=True)[:3], precision=3)
    with open(nwk, "rb") as f:
        same_tree = ("\n".join(trees) + "\n").encode() == f.read()
    os.unlink(phy)
    os.unlink(nwk)
    pairs = m * (m - 1) / 2
    return {"value": round(pairs / (t2 - t0), 2),
            "unit": "taxa-pairs/s (dist + DNJ tree, end to end, FASTA parse included; a sample rate)",
            "cores": cores, "host_cpus": ncpu, "cgroup_cpu_quota": quota, "kind": "reference",
            "dist_s": round(t1 - t0, 3), "tree_s": round(t2 - t1, 3),
            "dist_nt_comparisons_per_s": round(pairs * L / (t1 - t0), 1),
            "parity_mismatched_cells": mism, "parity_newick_identical": same_tree,
            "sample": f"SAMPLE RATE: reference ccphylo 0.8.5 `dist -t {cores}` + `tree -x 3` (DNJ) on the first {m} "
                      f"of the {L / 1e6:g} Mbp headline alignment's taxa (a {m * L / 4e9:.2f} GB FASTA written and "
                      f"parsed inside the time); the GPU's LT cells and Newick for the same taxa are compared with "
                      f"the reference's"}


def make_headline_alignment(torch, n, L, seed=3):
    """configs[2]: tools/config3.make_packed's tree-like alignment (512 clades,
    ~0.8% of codes flipped per taxon) on this GPU, every 10th word excluded
    (the 'N columns'); the same bytes on every rank."""
    from tools.config3 import make_packed
    W = L // 32 + 1
    seqs = make_packed(torch, n, W, seed=seed)
    incs = torch.full((W,), -1, dtype=torch.int32, device="cuda")
    incs[::10] = 0
    incs[(L + 31) // 32:] = 0
    if L % 32:
        incs[(L + 31) // 32 - 1] &= ((0xFFFFFFFF << (32 - L % 32)) & 0xFFFFFFFF) - (1 << 32)
    torch.cuda.synchronize()
    return seqs, incs, W


def pipeline_leg(dev, torch, rank, world, dist, coll, n, L, steps, warmup, barrier, profile_tree=True, capture_k=0,
                 tree_mode="shard", pg=None, tree_cus=0, tree_layout="low", seed=3):
    """The headline: dist + exact DNJ of one n x L alignment per step.
    world 1: ccg_snp_ltd_dev into the full double LT, ccg_tree_dev in place;
    world > 1, tree_mode "shard": ccg_snp_ltd_shard_dev into this rank's band
    shard, ccg_tree_shard_dev over `coll` (RCCL);
    world > 1, tree_mode "gather": each rank's dist over its contiguous LT
    row range (shard.lt_row_ranges, equal cells), the ranges sent to GPU 0
    (RCCL point-to-point on the process group `pg`, straight into place in
    its packed LT), and the single-GPU engine builds the tree there while the
    other ranks wait (at this n a join is a latency-bound chain
    that the sharded engine's per-join collectives only lengthen).
    Returns (timed result, the last step's joins, profiled-step stats or None,
    alignment, the first capture_k LT cells of the first step (world 1)).
    world 1 with tree_cus > 0: the pipelined form (pipelined_leg, alignments
    of seeds 3 and 4 in turn); otherwise the alignment of `seed`."""
    if world == 1 and tree_cus > 0:
        return pipelined_leg(dev, torch, n, L, steps, warmup, barrier, tree_cus, profile_tree, capture_k, tree_layout)
    if world > 1 and tree_mode == "gather-pipelined":
        return gather_pipelined_leg(dev, torch, rank, world, dist, n, L, steps, warmup, barrier, pg, profile_tree)
    import hashlib
    import ccphylo_amd as cg
    from ccphylo_amd import native as nt
    from ccphylo_amd import shard as shd
    seqs, incs, W = make_headline_alignment(torch, n, L, seed=seed)
    m = n * (n - 1) // 2
    gather = world > 1 and tree_mode == "gather"
    ranges = shd.lt_row_ranges(n, world) if gather else None
    if gather:
        r0, r1 = ranges[rank]
        elems = m if rank == 0 else r1 * (r1 - 1) // 2 - r0 * (r0 - 1) // 2
    else:
        elems = m if world == 1 else nt.shard_elems(n, rank, world)
    D = torch.empty(max(elems, 1), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    cap = []

    def step(profile=False):
        t0 = time.perf_counter()
        if world == 1:
            inc = dev.snp_ltd_dev(seqs.data_ptr(), incs.data_ptr(), n, L, W, D.data_ptr())
        elif gather:
            # rows [r0, r1) land at their packed offsets: rank 0 in its whole LT,
            # the others in a buffer that starts at row r0's offset
            base = D.data_ptr() - (0 if rank == 0 else 8 * (r0 * (r0 - 1) // 2))
            inc = dev.snp_ltd_dev(seqs.data_ptr(), incs.data_ptr(), n, L, W, base, row_range=(r0, r1))
        else:
            inc = dev.snp_ltd_shard_dev(seqs.data_ptr(), incs.data_ptr(), n, L, W, D.data_ptr(), rank, world)
        dms = dev.last_dist_ms()
        if gather and pg is not None:   # every range to GPU 0 at once (RCCL over xGMI)
            ops = []
            if rank == 0:
                for g in range(1, world):
                    a0, a1 = ranges[g]
                    o0, o1 = a0 * (a0 - 1) // 2, a1 * (a1 - 1) // 2
                    if o1 > o0:
                        ops.append(dist.P2POp(dist.irecv, D[o0:o1], g, pg))
            elif elems:
                ops.append(dist.P2POp(dist.isend, D[:elems], 0, pg))
            for w_ in (dist.batch_isend_irecv(ops) if ops else []):
                w_.wait()
            torch.cuda.synchronize()
        elif gather:   # gloo rehearsal (several ranks on one GPU): host-staged, rank by rank
            torch.cuda.synchronize()
            if rank == 0:
                for g in range(1, world):
                    a0, a1 = ranges[g]
                    o0, o1 = a0 * (a0 - 1) // 2, a1 * (a1 - 1) // 2
                    if o1 > o0:
                        buf = torch.empty(o1 - o0, dtype=torch.float64)
                        dist.recv(buf, src=g)
                        D[o0:o1].copy_(buf)
            elif elems:
                dist.send(D[:elems].cpu(), dst=0)
            torch.cuda.synchronize()
        t1 = time.perf_counter()
        if capture_k and not cap and world == 1:   # untimed: only in the first (warmup) step
            cap.append(D[:capture_k].cpu().numpy())
            t1 = time.perf_counter()
        if world == 1 or (gather and rank == 0):
            j, fn, fd, st = dev.tree_dev(D.data_ptr(), n, method=cg.CCG_TREE_DNJ, exact=True, profile=profile)
        elif gather:   # the tree runs on GPU 0; this rank's part of the step is done
            j, fn, fd, st = np.zeros(0, dtype=nt.JOIN_DTYPE), 0, 0.0, [0] * (12 + 2 * nt.NKSTAT)
        else:
            j, fn, fd, st = dev.tree_shard_dev(D.data_ptr(), n, coll, method=cg.CCG_TREE_DNJ, exact=True,
                                               profile=profile)
        t2 = time.perf_counter()
        return t1 - t0, t2 - t1, dms, (j, fn, fd), st, inc

    for w in range(warmup):
        r = step()
        log(f"  warmup step {w}: dist {r[0]:.2f} s, tree {r[1]:.2f} s")
    barrier()
    t0 = time.perf_counter()
    parts = []
    for k in range(steps):
        parts.append(step())
        log(f"  step {k}: dist {parts[-1][0]:.2f} s, tree {parts[-1][1]:.2f} s")
    barrier()
    dt = shard_max(time.perf_counter() - t0, dist)
    dist_s = shard_max(sum(p[0] for p in parts) / steps, dist)
    tree_s = shard_max(sum(p[1] for p in parts) / steps, dist)
    dist_kernel_ms = shard_max(sum(p[2] for p in parts) / steps, dist)
    joins, st, inc = parts[-1][3], parts[-1][4], parts[-1][5]
    jj, fn, fd = joins
    sha = hashlib.sha256(np.ascontiguousarray(jj).tobytes() + np.array([fn, fd]).tobytes()).hexdigest()[:16]
    pst = None
    if profile_tree:
        pst = step(profile=True)[4]   # HIP events around every tree kernel (an extra, untimed step)
    res = {"dt": dt, "dist_s": dist_s, "tree_s": tree_s, "dist_kernel_ms": dist_kernel_ms, "joins": len(jj),
           "joins_sha256": sha, "rows_rescanned": int(st[0]), "cells_rescanned": int(st[1]),
           "included_positions": inc}
    del D
    torch.cuda.empty_cache()
    return res, joins, pst, (seqs, incs, W), (cap[0] if cap else None)


def tree_cu_set(ncu, k, layout):
    """The tree context's compute units.  Mask bit c runs on XCD c % 8 (slot
    c // 8 there; tools/micro/cu_mask.hip, profiles/r06_cu_mask_map.txt), so
    "low" (bits 0 .. k-1) gives every XCD k / 8 CUs.  "xcd" (round 5: bits
    0 .. k/8 - 1 of each 32-bit word) puts them on XCDs 0 .. k/8 - 1 only:
    below k = 64 it leaves XCDs empty, which would run unmasked, and
    ccg_ctx_configure refuses it; at 64 it equals "low".  Inside an XCD the
    slots interleave its 4 shader engines and blocks are dealt round-robin
    over them, so a context runs like 32 x (its fewest CUs per engine): k
    should be a multiple of 32 (56 CUs run like 32, profiles/r06_tree_cus.jsonl)."""
    if layout == "xcd":
        per = max(1, k // 8)
        return [g * (ncu // 8) + i for g in range(8) for i in range(per)]
    return list(range(k))


def pipelined_leg(dev, torch, n, L, steps, warmup, barrier, tree_cus, profile_tree=True, capture_k=0, layout="low"):
    """The headline on one GPU as a pipeline over a stream of alignments: two
    engine contexts on disjoint compute units (ccg_ctx_configure: the tree's
    stream on CUs [0, tree_cus), 8 per XCD, the dist's on the rest, neither
    waiting for the whole device) and two LT buffers, so that step k builds
    the tree of matrix k while the dist of matrix k + 1 fills the other
    buffer.  The stream alternates two distinct alignments (seeds 3 and 4):
    matrix k is alignment k % 2's, so consecutive steps really are different
    matrices.  The dist of matrix 0 runs before the warmup; every timed step
    holds one whole dist and one whole tree (K of each in K steps), so the
    rate is matrices completed per second in steady state.  tree_s / dist_s
    are each context's device time (HIP events on its own stream); the thread
    walls are reported beside them.  Same return value as pipeline_leg, plus
    res["alignments"] (both) and res["joins_sha256_by_alignment"]."""
    import hashlib
    import threading
    import ccphylo_amd as cg
    aligns = [make_headline_alignment(torch, n, L, seed=3), make_headline_alignment(torch, n, L, seed=4)]
    W = aligns[0][2]
    m = n * (n - 1) // 2
    gpu = torch.cuda.current_device()
    ncu = torch.cuda.get_device_properties(gpu).multi_processor_count
    tree_cus = max(1, min(tree_cus, ncu - 1))
    tset = tree_cu_set(ncu, tree_cus, layout)
    ddev, tdev = cg.Device(gpu), cg.Device(gpu)
    ddev.configure(cu_mask=[c for c in range(ncu) if c not in set(tset)], nosync=True)
    tdev.configure(cu_mask=tset, nosync=True)
    tree_cus = len(tset)
    Ds = [torch.empty(m, dtype=torch.float64, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()
    s0, i0, _ = aligns[0]
    inc0 = ddev.snp_ltd_dev(s0.data_ptr(), i0.data_ptr(), n, L, W, Ds[0].data_ptr())   # matrix 0
    cap = Ds[0][:capture_k].cpu().numpy() if capture_k else None

    def step(k, profile=False):
        res, err = {}, []

        def run_d():
            try:
                sq, ic, _ = aligns[(k + 1) % 2]
                t0 = time.perf_counter()
                inc = ddev.snp_ltd_dev(sq.data_ptr(), ic.data_ptr(), n, L, W, Ds[(k + 1) % 2].data_ptr())
                res["d"] = (time.perf_counter() - t0, ddev.last_dist_ms(), inc)
            except Exception as e:  # noqa: BLE001
                err.append(e)

        def run_t():
            try:
                t0 = time.perf_counter()
                j, fn, fd, st = tdev.tree_dev(Ds[k % 2].data_ptr(), n, method=cg.CCG_TREE_DNJ, exact=True,
                                              profile=profile)
                res["t"] = (time.perf_counter() - t0, (j, fn, fd), st)
            except Exception as e:  # noqa: BLE001
                err.append(e)
        th = [threading.Thread(target=run_d), threading.Thread(target=run_t)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        if err:
            raise err[0]
        # walls, the dist's kernel ms, joins, stats, included positions, the tree's device s (HIP events)
        return (res["d"][0], res["t"][0], res["d"][1], res["t"][1], res["t"][2], res["d"][2],
                res["t"][2][3] / 1e6)

    def sha_of(joins):
        jj, fn, fd = joins
        return hashlib.sha256(np.ascontiguousarray(jj).tobytes() + np.array([fn, fd]).tobytes()).hexdigest()[:16]

    k = 0
    for w in range(warmup):
        r = step(k)
        k += 1
        log(f"  warmup step {w}: dist {r[0]:.2f} s beside tree {r[1]:.2f} s (device {r[6]:.2f} s)")
    barrier()
    t0 = time.perf_counter()
    parts = []
    shas = {}
    for s_ in range(steps):
        parts.append(step(k))
        shas.setdefault(k % 2, set()).add(sha_of(parts[-1][3]))
        k += 1
        log(f"  step {s_}: dist {parts[-1][0]:.2f} s beside tree {parts[-1][1]:.2f} s "
            f"(tree device {parts[-1][6]:.2f} s, dist kernels {parts[-1][2] / 1e3:.2f} s)")
    barrier()
    dt = time.perf_counter() - t0
    joins, st, inc = parts[-1][3], parts[-1][4], parts[-1][5]
    # the line's sha: alignment 0's (the sequential form's default matrix)
    sha = sorted(shas[0])[0] if 0 in shas else sha_of(joins)
    pst = step(k, profile=True)[4] if profile_tree else None   # an extra, untimed pipelined step
    res = {"dt": dt, "dist_s": sum(p[2] for p in parts) / steps / 1e3, "tree_s": sum(p[6] for p in parts) / steps,
           "dist_wall_s": sum(p[0] for p in parts) / steps, "tree_wall_s": sum(p[1] for p in parts) / steps,
           "dist_kernel_ms": sum(p[2] for p in parts) / steps, "joins": len(joins[0]), "joins_sha256": sha,
           "joins_sha256_by_alignment": {str(a): sorted(v) for a, v in shas.items()},
           "rows_rescanned": int(st[0]), "cells_rescanned": int(st[1]), "included_positions": inc,
           "alignments": aligns,
           "pipelined": {"tree_cus": tree_cus, "dist_cus": ncu - tree_cus, "layout": layout,
                         "matrix0_included_positions": inc0, "alignment_seeds": [3, 4]}}
    del Ds
    ddev.close()
    tdev.close()
    torch.cuda.empty_cache()
    return res, joins, pst, aligns[0], cap


def gather_pipelined_leg(dev, torch, rank, world, dist, n, L, steps, warmup, barrier, pg, profile_tree=True):
    """The headline at N > 1 as a pipeline over a stream of alignments: rank 0
    builds the tree of matrix k on its whole chip while ranks 1 .. N-1
    compute the dist of matrix k + 1 over contiguous LT row ranges of equal
    cells (shard.lt_row_ranges over N - 1 ranks) and send them into rank 0's
    other LT buffer (RCCL point-to-point on `pg`; gloo host-staged when pg is
    None).  Every timed step holds one whole dist and one whole tree.  Rank
    0's context does not wait for the whole device at its entry points
    (ccg_ctx_configure nosync): the receives run beside the tree.  Same
    return value as pipeline_leg; the dist figures are rank 1's."""
    import hashlib
    import threading
    import ccphylo_amd as cg
    from ccphylo_amd import native as nt
    from ccphylo_amd import shard as shd
    seqs, incs, W = make_headline_alignment(torch, n, L)
    m = n * (n - 1) // 2
    ranges = [(0, 0)] + shd.lt_row_ranges(n, world - 1)   # rank 0: the tree only

    def off(r):
        return r * (r - 1) // 2 if r > 0 else 0
    r0, r1 = ranges[rank]
    elems = off(r1) - off(r0)
    if rank == 0:
        dev.configure(nosync=True)
        Ds = [torch.empty(m, dtype=torch.float64, device="cuda") for _ in range(2)]
    else:
        Dl = torch.empty(max(elems, 1), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    cur = torch.cuda.current_stream()

    def dist_part():
        t0 = time.perf_counter()
        inc = dev.snp_ltd_dev(seqs.data_ptr(), incs.data_ptr(), n, L, W, Dl.data_ptr() - 8 * off(r0),
                              row_range=(r0, r1))
        return time.perf_counter() - t0, dev.last_dist_ms(), inc

    def transfer(k):   # matrix k's row ranges into rank 0's buffer k % 2
        if pg is not None:
            ops = []
            if rank == 0:
                for g in range(1, world):
                    a0, a1 = ranges[g]
                    if off(a1) > off(a0):
                        ops.append(dist.P2POp(dist.irecv, Ds[k % 2][off(a0):off(a1)], g, pg))
            elif elems:
                ops.append(dist.P2POp(dist.isend, Dl[:elems], 0, pg))
            for w_ in (dist.batch_isend_irecv(ops) if ops else []):
                w_.wait()
            cur.synchronize()   # this stream only: rank 0's tree runs on the engine's own stream
        elif rank == 0:
            for g in range(1, world):
                a0, a1 = ranges[g]
                if off(a1) > off(a0):
                    buf = torch.empty(off(a1) - off(a0), dtype=torch.float64)
                    dist.recv(buf, src=g)
                    Ds[k % 2][off(a0):off(a1)].copy_(buf)
            cur.synchronize()
        elif elems:
            dist.send(Dl[:elems].cpu(), dst=0)

    def step(k, profile=False):
        """tree of matrix k (rank 0) beside the dist and transfer of matrix k + 1"""
        if rank == 0:
            res, err = {}, []

            def run_t():
                try:
                    t0 = time.perf_counter()
                    j, fn, fd, st = dev.tree_dev(Ds[k % 2].data_ptr(), n, method=cg.CCG_TREE_DNJ, exact=True,
                                                 profile=profile)
                    res["t"] = (time.perf_counter() - t0, (j, fn, fd), st)
                except Exception as e:  # noqa: BLE001
                    err.append(e)
            th = threading.Thread(target=run_t)
            th.start()
            transfer(k + 1)
            th.join()
            if err:
                raise err[0]
            return 0.0, res["t"][0], 0.0, res["t"][1], res["t"][2], 0
        ds, dms, inc = dist_part()
        transfer(k + 1)
        return ds, 0.0, dms, (np.zeros(0, dtype=nt.JOIN_DTYPE), 0, 0.0), [0] * (12 + 2 * nt.NKSTAT), inc

    if rank != 0:
        dist_part()
    transfer(0)   # matrix 0
    k = 0
    for w in range(warmup):
        r = step(k)
        k += 1
        log(f"  warmup step {w}: dist {r[0]:.2f} s beside tree {r[1]:.2f} s")
    barrier()
    t0 = time.perf_counter()
    parts = []
    for s_ in range(steps):
        parts.append(step(k))
        k += 1
        log(f"  step {s_}: dist {parts[-1][0]:.2f} s beside tree {parts[-1][1]:.2f} s")
    barrier()
    dt = shard_max(time.perf_counter() - t0, dist)
    joins, st = parts[-1][3], parts[-1][4]
    jj, fn, fd = joins
    sha = hashlib.sha256(np.ascontiguousarray(jj).tobytes() + np.array([fn, fd]).tobytes()).hexdigest()[:16]
    pst = step(k, profile=True)[4] if profile_tree else None
    barrier()
    # rank 1's dist figures (the ranks' shares are equal) for rank 0's line
    mine = [sum(p[0] for p in parts) / steps, sum(p[2] for p in parts) / steps, parts[-1][5], elems,
            sum(p[1] for p in parts) / steps]
    allv = [None] * world
    dist.all_gather_object(allv, mine)
    d1 = allv[1]
    tree_s = allv[0][4]   # rank 0's (every rank reports the same line fields)
    res = {"dt": dt, "dist_s": d1[0], "tree_s": tree_s, "dist_kernel_ms": d1[1], "joins": len(jj),
           "joins_sha256": sha, "rows_rescanned": int(st[0]), "cells_rescanned": int(st[1]),
           "included_positions": d1[2], "dist_elems": d1[3],
           "gather_pipelined": {"dist_ranks": world - 1, "tree_rank": 0}}
    if rank == 0:
        del Ds
        dev.configure()   # the extras after this leg order their inputs by device-wide waits again
    else:
        del Dl
    torch.cuda.empty_cache()
    return res, joins, pst, (seqs, incs, W), None


def refrule_cells(dev, torch, seqs, incs, n, L, W, prefix, threads):
    """DNJ's algorithmic bytes count the cells the REFERENCE's
    minQpair rescans (dnj.c:43-128), not the engine's speculative ones.  The
    oracle (the reference's rule, serial) and the engine run the same first
    `prefix` joins of the headline matrix; their rescanned rows / cells."""
    import ccphylo_amd as cg
    from oracle import pyoracle
    m = n * (n - 1) // 2
    D = torch.empty(m, dtype=torch.float64, device="cuda")
    dev.snp_ltd_dev(seqs.data_ptr(), incs.data_ptr(), n, L, W, D.data_ptr())
    host = D.cpu().numpy()
    j, fn, fd, st = dev.tree_dev(D.data_ptr(), n, method=cg.CCG_TREE_DNJ, exact=True, max_joins=prefix,
                                 profile=True)
    K = len(KNAMES)
    del D
    torch.cuda.empty_cache()
    t0 = time.perf_counter()
    rj, _, _, rst = pyoracle.tree(host, n, method=cg.CCG_TREE_DNJ, max_joins=prefix, threads=threads, copy=False,
                                  stats=True)
    dt = time.perf_counter() - t0
    same = len(rj) == len(j) and bool((rj == j).all())
    del host
    return {"joins": prefix, "engine_rows": int(st[0]), "engine_cells": int(st[1]),
            "reference_rule_rows": int(rst[0]), "reference_rule_cells": int(rst[1]),
            "engine_over_reference_cells": round(int(st[1]) / max(int(rst[1]), 1), 3),
            "engine_counter_equals_oracle": (int(st[10 + 2 * K]), int(st[11 + 2 * K])) == (int(rst[0]), int(rst[1])),
            "joins_identical_to_oracle": same, "oracle_s": round(dt, 1)}


def kma_extra(dev, torch, n=1024, L=50_000, reps=3, metric="cos"):
    """Count-matrix (KMA *.mat) distances, ccg_kma_ltd_dev: n samples x L
    positions of synthetic depth-~30 counts (views built on the GPU; the
    file loader is not timed).  Rate = sample pairs x positions / s."""
    g = torch.Generator(device="cuda").manual_seed(5)
    base = torch.randint(0, 4, (L,), device="cuda", generator=g)
    cnt = torch.randint(0, 3, (n, L, 6), device="cuda", generator=g, dtype=torch.int32)
    dom = torch.randint(15, 45, (n, L), device="cuda", generator=g, dtype=torch.int32)
    cnt.scatter_add_(2, base.view(1, L, 1).expand(n, L, 1), dom.unsqueeze(2))
    tot = cnt.sum(2)
    rec = torch.zeros((n, L, 4), dtype=torch.int32, device="cuda")
    rec[:, :, 0] = cnt[:, :, 0] | (cnt[:, :, 1] << 16)
    rec[:, :, 1] = cnt[:, :, 2] | (cnt[:, :, 3] << 16)
    rec[:, :, 2] = cnt[:, :, 4] | (cnt[:, :, 5] << 16)
    rec[:, :, 3] = tot
    rec1 = torch.zeros((n, L + 1, 4), dtype=torch.int32, device="cuda")
    rec1[:, :L] = rec
    len1 = torch.full((n,), L + 1, dtype=torch.int32, device="cuda")   # stripMat without insertions
    len2 = torch.full((n,), L, dtype=torch.int32, device="cuda")
    m = n * (n - 1) // 2
    D = torch.empty(m, dtype=torch.float64, device="cuda")
    args = (n, rec1.data_ptr(), len1.data_ptr(), L + 1, rec.data_ptr(), len2.data_ptr(), L, D.data_ptr())
    dev.kma_ltd_dev(*args, metric=metric)
    times = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dev.kma_ltd_dev(*args, metric=metric)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    dt = min(times)
    del rec, rec1, cnt, D
    return {"sample_pairs_per_s": round(m / dt, 1), "position_pairs_per_s": m * L / dt, "seconds": round(dt, 4),
            "config": f"{n} KMA count matrices x {L} positions, -d {metric}, double, views in HBM"}


def nj_shard_extra(dev, torch, rank=0, world=1, dist=None, coll=None, n=100_000, joins=64):
    """NJ on ONE n-taxon matrix (n = 100k, double: 40 GB): world 1 the
    single-GPU engine; world > 1 the row-sharded engine (rank g holds the row
    bands g, g + world, ...; ccg_tree_shard_dev) over `coll`
    (RCCL) -- strong scaling of one tree.  Timed: the first `joins` joins
    (each a full initQ scan of the whole matrix), as time(joins + 1) -
    time(1) so the exact initSummaD and the setup are excluded."""
    import ccphylo_amd as cg
    from tools.synth import euclid_shard_dev
    loc = euclid_shard_dev(torch, n, rank, world)
    work = torch.empty_like(loc)

    def run(k, profile=False):
        work.copy_(loc)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        j, fn, fd, st = dev.tree_shard_dev(work.data_ptr(), n, coll, method=cg.CCG_TREE_NJ, exact=False,
                                           profile=profile, max_joins=k)
        dt = time.perf_counter() - t0
        assert len(j) == k, (len(j), k)
        dt = shard_max(dt, dist)
        return dt, st

    t1, _ = run(1)
    tk, _ = run(joins + 1)
    _, pst = run(joins + 1, profile=True)
    dt = tk - t1
    # algorithmic bytes of the argmin of the timed joins: every LT cell once (s = 8) + sD
    cells = sum((m * (m - 1) // 2) for m in range(n - joins, n))
    gb = (8.0 * cells + 8.0 * n * joins) / dt / 1e9
    cnt, ns = pst[4 + 2 * 3], pst[5 + 2 * 3]
    kern_gb = (8.0 * cells / world + 8.0 * n * joins) / (ns / 1e9) / 1e9 if ns else None
    del loc, work
    torch.cuda.empty_cache()
    return {"joins_per_s": round(joins / dt, 2), "ms_per_join": round(1000 * dt / joins, 3), "joins": joins,
            "n": n, "world": world, "seconds": round(dt, 4),
            "config": f"NJ (-m nj) on one N={n} Euclidean matrix (double, {8 * n * (n - 1) / 2 / 1e9:.1f} GB), " +
                      ("the single-GPU engine" if world == 1 else f"its LT row bands dealt over {world} GPUs") +
                      f"; first {joins} joins; fast row sums",
            "hbm_GBps_aggregate": round(gb, 1), "hbm_frac_aggregate": round(gb / (HBM_PEAK_GBS * world), 4),
            "argmin_kernel_GBps_per_gpu": round(kern_gb, 1) if kern_gb else None,
            "coll_us_per_join": round(pst[5 + 2 * 8] / 1e3 / (joins + 1), 2) if pst[4 + 2 * 8] else 0.0}


def dnj_shard_extra(dev, torch, rank=0, world=1, dist=None, coll=None, n=200_000, joins=0, exact=True,
                    profile_joins=2000):
    """configs[3]: DNJ on ONE n-taxon Euclidean matrix (n = 200k, float =
    `-p`: 80 GB), the WHOLE tree (joins = 0) with exact row sums.  world 1:
    the single-GPU engine on the packed LT (ccg_tree_shard_dev at world 1);
    world > 1: rank g holds the row bands g, g + world, ... and the ranks
    exchange over `coll` (RCCL) -- strong scaling of one tree.  A second,
    profiled run of the first `profile_joins` joins gives each rank's device
    time per join by kernel class (HIP events on the engine stream; the
    collectives' class is their device time on that stream), reported for
    rank 0 and as the max over ranks; the aggregate HBM fraction counts the
    cells every rank's scans loaded (4 B each) plus the O(n) vectors."""
    import hashlib
    import ccphylo_amd as cg
    from ccphylo_amd import native as nt
    from tools.synth import euclid_shard_dev
    loc = euclid_shard_dev(torch, n, rank, world, dtype=torch.float32)
    work = torch.empty_like(loc) if profile_joins else None
    if work is not None:
        work.copy_(loc)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    j, fn, fd, st = dev.tree_shard_dev(loc.data_ptr(), n, coll, etype=4, method=cg.CCG_TREE_DNJ, exact=exact,
                                       max_joins=joins)
    dt = shard_max(time.perf_counter() - t0, dist)
    del loc
    sha = hashlib.sha256(np.ascontiguousarray(j).tobytes() + np.array([fn, fd]).tobytes()).hexdigest()[:16]
    cells_all = float(st[1]) if dist is None else shard_sum(float(st[1]), dist)
    # algorithmic bytes: the cells the scans loaded + per join ~ (4 s + 40) n of vectors and line updates
    algo = 4.0 * cells_all + sum(56.0 * (n - k) for k in range(len(j)))
    res = {"joins_per_s": round(len(j) / dt, 2), "ms_per_join": round(1000 * dt / max(len(j), 1), 4),
           "joins": len(j), "n": n, "world": world, "seconds": round(dt, 3), "joins_sha256": sha,
           "rows_rescanned_rank0": int(st[0]), "cells_rescanned_rank0": int(st[1]),
           "cells_rescanned_all_ranks": int(cells_all),
           "hbm_GBps_aggregate": round(algo / dt / 1e9, 1),
           "hbm_frac_aggregate": round(algo / dt / 1e9 / (HBM_PEAK_GBS * world), 4),
           "row_sums": "exact" if exact else "fast",
           "config": f"configs[3]: DNJ (-m dnj) on one N={n} Euclidean matrix (float, "
                     f"{4 * n * (n - 1) / 2 / 1e9:.0f} GB), " +
                     ("the single-GPU engine" if world == 1 else f"its LT row bands dealt over {world} GPUs (RCCL)") +
                     f"; {'the whole tree' if not joins else f'first {joins} joins'}, init included"}
    if work is not None:
        pj = min(profile_joins, len(j)) if len(j) else profile_joins
        if dist is not None:
            dist.barrier()
        _, _, _, ps = dev.tree_shard_dev(work.data_ptr(), n, coll, etype=4, method=cg.CCG_TREE_DNJ, exact=exact,
                                         max_joins=pj, profile=True)
        per, mx = {}, {}
        for c, nm in enumerate(KNAMES):   # every class on every rank, in one order (the max is a collective)
            us = ps[5 + 2 * c] / 1e3 / pj if ps[4 + 2 * c] else 0.0
            m_ = shard_max(us, dist)
            if nm != "init" and m_ > 0:
                per[nm], mx[nm] = round(us, 2), round(m_, 2)
        res["device_us_per_join_rank0"] = {"joins": pj, **per}
        res["device_us_per_join_max_over_ranks"] = mx
        res["device_us_per_join_total_rank0"] = round(sum(per.values()), 2)
        del work
    torch.cuda.empty_cache()
    return res


def shard_max(x, dist):
    if dist is None:
        return x
    from ccphylo_amd import shard
    return shard.reduce_max(x, dist)


def shard_sum(x, dist):
    if dist is None:
        return x
    from ccphylo_amd import shard
    return shard.reduce_sum(x, dist)


def reference_tree_parity(D, n, exact_joins, fast_joins, td):
    """Checks in the cpu_baseline leg: the reference binary's Newick for the
    bench matrix against the GPU's exact-mode tree (byte identity), and the
    fast-sum tree against the exact one (join identity, splits differing)."""
    import ccphylo_amd as cg
    from ccphylo_amd import native
    from tools.parity_large import splits
    out = {}
    ref_nwk = os.path.join(td, "ref.nwk")
    path = os.path.join(td, "bench_ref.phy")
    if os.path.exists(ref_nwk):
        native.write_phylip(path, D, n, [f"t{k}" for k in range(n)])
        ej, efn, efd = exact_joins
        trees = cg.newick_from_phylip(path, lambda _D, _n: (ej, efn, efd))
        os.unlink(path)
        with open(ref_nwk, "rb") as f:
            out["exact_newick_identical_to_reference"] = ("\n".join(trees) + "\n").encode() == f.read()
    if fast_joins is not None:
        fj, ffn, _ = fast_joins
        ej, efn, _ = exact_joins
        same = len(fj) == len(ej) and bool((fj["i"] == ej["i"]).all() and (fj["j"] == ej["j"]).all())
        out["fast_joins_identical"] = same
        out["fast_splits_differing"] = len(splits(fj, n, ffn) ^ splits(ej, n, efn)) // 2
    return out


HEADLINE_STATS = _latest("r06_kernel_stats_headline.csv", "r05_kernel_stats_headline.csv", "r04_kernel_stats_headline.csv", "r03_kernel_stats_headline.csv")
def dist_kernel_name():
    """The non-pair dist kernel the engine launches (snp.hip: k_snp_mfma3, the
    LDS-DMA staged form, unless CCG_DIST_GLDS=0 or CCG_DIST_KC=16; CCG_DIST_MFMA
    1 / 0: the 128x128 MFMA / VALU tiles)."""
    mode = os.environ.get("CCG_DIST_MFMA", "2")
    if mode == "0":
        return "k_snp_tile"
    if mode == "1":
        return "k_snp_mfma"
    if os.environ.get("CCG_DIST_GLDS") == "0" or os.environ.get("CCG_DIST_KC") == "16":
        return "k_snp_mfma2"
    return "k_snp_mfma3"


HSYM = {"dist": (dist_kernel_name(),), "dnj_scan": ("k_dnj_scan_v", "k_dnj_scan_w", "k_dnj_scan", "k_dnj_scan_g"),
        "dnj_find": ("k_dnj_plan",), "update": ("k_dnj_join_pf", "k_dnj_join"), "dnj_requeue": ("k_dnj_requeue",),
        "exact_sum": ("k_exact_sum",), "dnj_select": ("k_dnj_select",), "init": ("k_init_rows",)}


def _base_symbol(name):
    return re.match(r"(?:void )?([A-Za-z_]\w*)", name).group(1)


def headline_profile_evidence(kernel):
    """rocprofv3 mean duration (us) and PMC HBM bytes per launch of a headline
    kernel, from the committed profiles of the same workload (if present)."""
    import csv
    out = {}
    syms = HSYM.get(kernel, (kernel,))
    try:   # launch-weighted over the class's kernel forms (e.g. the three scan forms)
        calls = ns = 0
        with open(HEADLINE_STATS) as f:
            for r in csv.DictReader(f):
                if _base_symbol(r["Name"]) in syms:
                    calls += int(r["Calls"])
                    ns += float(r["TotalDurationNs"])
        if calls:
            out["rocprof_mean_us"] = round(ns / calls / 1e3, 3)
            out["rocprof_calls"] = calls
    except (OSError, KeyError, ValueError):
        pass
    try:
        with open(PMC_HEADLINE) as f:
            d = json.load(f)
        ks = [d["kernels"][s] for s in syms if s in d["kernels"]]
        launches = sum(k["launches"] for k in ks)
        if launches:
            out["traffic"] = round(sum(k["hbm_bytes_per_launch"] * k["launches"] for k in ks) / launches, 1)
            out["traffic_source"] = d.get("source")
    except (OSError, KeyError, ValueError):
        pass
    return out


def headline_roofline(n, L, positions, elems, dist_kernel_ms, dist_launches, pst, world, single_tree=False):
    """Every kernel of the headline step with its roofline; the dominant one
    (largest device time per step) is the line's `roofline`.
    dist: 6 flops (3 MX-fp4 MACs) per position pair, this rank's cells x the
    positions the kernel compares (the included ones: k_planes compacts the
    excluded words away, so the MFMAs never see them), against the MX-fp4
    dense peak; tree kernels: SURVEY 8(d) bytes (the engine's own rescanned
    cells for the scans), against 8 TB/s."""
    kernels = {}
    fl = FLOPS_PER_POSITION_PAIR * elems * float(positions)
    tf = fl / (dist_kernel_ms / 1e3) / 1e12
    d = {"kernel": dist_kernel_name(), "bound": "mfma", "achieved": round(tf, 1),
         "peak": MFMA_FP4_DENSE_TFLOPS, "unit": "TFLOP/s", "frac": round(tf / MFMA_FP4_DENSE_TFLOPS, 4),
         "frac_of_measured_issue_peak": round(tf / MFMA_FP4_MEASURED_TFLOPS, 4),
         "step_ms": round(dist_kernel_ms, 2), "launches": dist_launches,
         "avg_launch_ms": round(dist_kernel_ms / dist_launches, 3),
         "flops_per_launch": fl / dist_launches,
         "algorithm": f"6 flops per position pair (tetrahedron MX-fp4 form, dist = (3 L - dot) / 4), "
                      f"position pairs = LT cells x {positions} included positions (of L = {L})"}
    d.update(headline_profile_evidence("dist"))
    if d.get("rocprof_mean_us"):   # the same count over the committed rocprofv3 mean of the same command
        d["frac_rocprof_duration"] = round(fl / dist_launches / (d["rocprof_mean_us"] * 1e-6) / 1e12 /
                                           MFMA_FP4_DENSE_TFLOPS, 4)
    kernels["dist"] = d
    if pst is not None:
        cs, cr = pst[4 + 2 * len(KNAMES)], pst[5 + 2 * len(KNAMES)]
        ch = pst[8 + 2 * len(KNAMES)] if world == 1 or single_tree else 0   # plan helpers' S cells (single engine)
        for c, name in enumerate(KNAMES):
            cnt, ns = pst[4 + 2 * c], pst[5 + 2 * c]
            if not cnt or name == "coll":
                continue
            ab = algorithmic_bytes_total(name, n, 8, cs, cr, ch) / (world if name in ("init",) else 1)
            gbs = ab / (ns / 1e9) / 1e9
            k = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": round(gbs / HBM_PEAK_GBS, 5), "step_ms": round(ns / 1e6, 2), "launches": cnt,
                 "avg_launch_us": round(ns / cnt / 1e3, 3), "algorithmic_bytes_per_launch": round(ab / cnt, 1)}
            k.update(headline_profile_evidence(name))
            if name == "dnj_scan":
                k.update(refrule_scan(pst, n, 8, cnt, ns / cnt / 1e9))
            kernels[name] = k
        if pst[4 + 2 * 8]:
            kernels["coll"] = {"step_ms": round(pst[5 + 2 * 8] / 1e6, 2), "launches": pst[4 + 2 * 8],
                               "note": "collective enqueue / host-staged round trips"}
    dom = max((k for k in kernels if k != "coll"), key=lambda k: kernels[k]["step_ms"])
    out = {key: kernels[dom][key] for key in ("bound", "achieved", "peak", "unit", "frac")}
    out["traffic"] = kernels[dom].get("traffic")
    out["kernel"] = kernels[dom].get("kernel", KSYM.get(dom, dom))
    out["step_ms"] = kernels[dom]["step_ms"]
    for key in ("rocprof_mean_us", "traffic_source", "avg_launch_ms", "avg_launch_us", "flops_per_launch",
                "algorithmic_bytes_per_launch"):
        if key in kernels[dom]:
            out[key] = kernels[dom][key]
    out["timing"] = "HIP events on the engine stream (dist: ccg_last_dist_ms; tree: a profiled step)"
    out["kernels"] = kernels
    return out


def config1_extras(dev, torch, td, n=10_000, steps=3, cpu=True, threads=16):
    """configs[1]: an N=10k synthetic Phylip matrix (Euclidean U[0,1)^8, seed
    1, %.9f-quantized), `tree -m dnj` exact (steps-timed, one fresh device
    copy per tree), fast sums, NJ, HNJ; the reference binary's DNJ on the
    same matrix and its NJ on the first 4000 taxa (NJ is O(n^3) on the CPU);
    the reference-rule rescanned cells (oracle) vs the engine's."""
    import ccphylo_amd as cg
    from oracle import pyoracle
    D = euclid_ltd(n, seed=1)
    nbytes = D.nbytes
    bufs = [dev.malloc(nbytes) for _ in range(steps + 1)]
    for b in bufs:
        dev.h2d(b, D)
    dev.tree_dev(bufs[0], n, method=cg.CCG_TREE_DNJ, exact=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    joins = 0
    for k in range(steps):
        j, fn, fd, st = dev.tree_dev(bufs[1 + k], n, method=cg.CCG_TREE_DNJ, exact=True)
        joins += len(j)
    dt = time.perf_counter() - t0
    for b in bufs:
        dev.free(b)
    exact_joins = (j, fn, fd)
    out = {"config": f"configs[1]: N={n} Euclidean Phylip matrix (%.9f), f64, one GPU",
           "dnj_exact": {"joins_per_s": round(joins / dt, 2), "ms_per_tree": round(1000 * dt / steps, 2),
                         "steps": steps, "rows_rescanned": int(st[0]), "cells_rescanned": int(st[1])}}
    pb = dev.malloc(nbytes)
    fast_joins = None
    for label, method, ex in (("dnj_fast_sums", cg.CCG_TREE_DNJ, False), ("nj", cg.CCG_TREE_NJ, True),
                              ("hnj", cg.CCG_TREE_HNJ, True)):
        dev.h2d(pb, D)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        j2, fn2, fd2, _ = dev.tree_dev(pb, n, method=method, exact=ex)
        t2 = time.perf_counter() - t1
        out[label] = {"joins_per_s": round(len(j2) / t2, 2), "seconds": round(t2, 4),
                      "row_sums": "exact" if ex else "fast"}
        if label == "dnj_fast_sums":
            fast_joins = (j2, fn2, fd2)
    dev.h2d(pb, D)
    _, _, _, pst = dev.tree_dev(pb, n, method=cg.CCG_TREE_DNJ, exact=True, profile=True)
    out["dnj_exact"]["roofline"] = roofline(pst, n, 8)
    dev.h2d(pb, D)
    _, _, _, nst = dev.tree_dev(pb, n, method=cg.CCG_TREE_NJ, exact=True, profile=True)
    out["nj"]["roofline"] = roofline(nst, n, 8)
    dev.free(pb)
    # the reference rule's rescans on the same tree (the oracle, serial)
    rj, _, _, rst = pyoracle.tree(D, n, method=cg.CCG_TREE_DNJ, stats=True, threads=threads)
    out["dnj_exact"]["reference_rule"] = {
        "rows_rescanned": int(rst[0]), "cells_rescanned": int(rst[1]),
        "engine_over_reference_cells": round(out["dnj_exact"]["cells_rescanned"] / max(int(rst[1]), 1), 3),
        "engine_counter_equals_oracle": (int(pst[10 + 2 * len(KNAMES)]), int(pst[11 + 2 * len(KNAMES)])) ==
                                        (int(rst[0]), int(rst[1])),
        "joins_identical_to_oracle": bool(len(rj) == len(j) and (rj == j).all())}
    if cpu:
        out["dnj_exact"]["cpu_baseline"] = cpu_baseline(D, n, td)
        try:
            par = reference_tree_parity(D, n, exact_joins, fast_joins, td)
            out["dnj_exact"]["cpu_baseline"]["parity"] = par
            out["dnj_fast_sums"]["parity_vs_exact"] = {k: v for k, v in par.items() if k.startswith("fast")}
        except Exception as e:  # noqa: BLE001
            out["dnj_exact"]["cpu_baseline"]["parity"] = {"error": str(e)}
        # NJ on the host: the reference's -m nj on the first 4000 taxa, the GPU on the same matrix
        m4 = 4000
        D4 = D[:m4 * (m4 - 1) // 2].copy()
        nj_cpu = cpu_baseline(D4, m4, td, threads=[1], method="nj")
        t1 = time.perf_counter()
        dev.tree(D4, m4, method=cg.CCG_TREE_NJ, exact=True)
        t2 = time.perf_counter() - t1
        nj_cpu["gpu_joins_per_s_same_matrix"] = round((m4 - 2) / t2, 2)
        out["nj"]["cpu_baseline"] = nj_cpu
    return out


def spawn_ranks(world):
    """One child process per rank (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT as torch.distributed.run sets them), each running
    this script with the same arguments.  Returns the largest exit code."""
    import socket
    import subprocess
    with socket.socket() as so:   # a free port for the rendezvous store
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c != 0]
    return (max(bad, key=abs) if bad else 0) & 0xFF


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", "--taxa", dest="n", type=int, default=50_000,
                    help="headline taxa (configs[2]; --taxa under torchrun, whose own options take --n)")
    ap.add_argument("--L", type=int, default=5_000_000, help="headline alignment length (configs[2])")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--c1-n", type=int, default=10_000)
    ap.add_argument("--refrule-prefix", type=int, default=150)
    ap.add_argument("--shard-n", type=int, default=100_000)
    ap.add_argument("--shard-joins", type=int, default=64)
    ap.add_argument("--dnj-shard-n", type=int, default=200_000)
    ap.add_argument("--dnj-shard-joins", type=int, default=20_000,
                    help="joins of the configs[3] tree to time (0: the whole tree; the rescans per join grow "
                         "along this tree, DESIGN.md 4)")
    ap.add_argument("--shard-transport", choices=["rccl", "gloo"], default="rccl",
                    help="gloo: host-staged (rehearsal of several ranks on one GPU)")
    ap.add_argument("--tree-mode", choices=["gather-pipelined", "gather", "shard"], default="gather-pipelined",
                    help="N > 1: GPU 0 builds each matrix's tree while GPUs 1 .. N-1 compute the next matrix's "
                         "dist and send it over (default, gather_pipelined_leg); gather: every GPU's dist rows "
                         "gathered to GPU 0, then its tree, step by step; shard: the row-sharded tree over RCCL "
                         "(DESIGN.md 6)")
    ap.add_argument("--tree-cus", type=int, default=64,
                    help="N = 1: the pipelined headline (pipelined_leg) with the tree on this many compute units and "
                         "the next matrix's dist on the rest (64: tools/overlap.py, 50k x 5 Mbp per matrix 7.59 s "
                         "against 7.71-7.90 s at 32-56 CUs); 0: dist then tree on the whole chip, step by step")
    ap.add_argument("--tree-layout", choices=["low", "xcd"], default="low",
                    help="which CUs the pipelined tree takes: mask bits 0 .. --tree-cus - 1 (--tree-cus / 8 CUs "
                         "per XCD), or the first --tree-cus / 8 bits of each 32-bit mask word (round 5's form: "
                         "XCDs 0 .. --tree-cus/8 - 1 only; refused below 64)")
    ap.add_argument("--headline-seed", type=int, default=3,
                    help="the alignment's seed in the sequential forms (the pipelined one alternates 3 and 4)")
    args = ap.parse_args()
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # `python bench.py --gpus N` without a launcher: start the N rank
        # processes here, before this process touches any GPU, and exit with
        # the worst of their codes (rank 0 prints the line)
        sys.exit(spawn_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world} (the launcher's world must match)")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
    # one GPU per rank; on a smaller box (rehearsals) ranks share the devices
    gpu = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    import ccphylo_amd as cg
    from ccphylo_amd import native as nt
    ncpu, quota = host_cpus()
    oracle_threads = max(1, min(16, int(quota) if quota else ncpu))
    dev = cg.Device(gpu)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    coll, transport = None, "none (one GPU)"
    if world > 1:
        try:
            coll = nt.RcclColl(dev, dist) if args.shard_transport == "rccl" else nt.HostColl(dist)
            transport = args.shard_transport
        except Exception as e:  # noqa: BLE001
            coll, transport = nt.HostColl(dist), f"gloo (host-staged; RCCL unavailable: {e})"

    if rank == 0:
        start_heartbeat()
    n, L = args.n, args.L
    m = n * (n - 1) // 2
    pg = None
    if world == 1:
        elems = m
    elif args.tree_mode.startswith("gather"):   # this rank's dist cells: its contiguous row range
        from ccphylo_amd import shard as shd
        r0_, r1_ = shd.lt_row_ranges(n, world)[rank]
        elems = r1_ * (r1_ - 1) // 2 - r0_ * (r0_ - 1) // 2
        if args.shard_transport == "rccl":
            pg = dist.new_group(backend="nccl")   # RCCL point-to-point for the ranges
        else:
            pg = None   # gloo: the default group (host-staged rehearsal)
    else:
        elems = nt.shard_elems(n, rank, world)
    log(f"headline: configs[2] pipeline {n} x {L}, world {world}, {args.warmup} warmup + {args.steps} steps")
    hwd = None
    if world > 1:   # a collective that never completes ends the run with a line saying so, not a hang
        import threading

        def _headline_timeout():
            if rank == 0:
                print(json.dumps({"metric": "taxa-pairs/sec (dist) + NJ iterations/sec at N taxa, 1/2/4/8 MI355X",
                                  "value": None, "n_gpus": world, "error": f"sharded headline did not finish in "
                                  f"{HEADLINE_TIMEOUT_S} s (transport {transport})"}), flush=True)
            os._exit(3)
        hwd = threading.Timer(HEADLINE_TIMEOUT_S, _headline_timeout)
        hwd.daemon = True
        hwd.start()
    head, joins, pst, (seqs, incs, W), cells = pipeline_leg(
        dev, torch, rank, world, dist if world > 1 else None, coll, n, L, args.steps, args.warmup, barrier,
        capture_k=256 * 255 // 2 if (world == 1 and not args.no_cpu) else 0, tree_mode=args.tree_mode, pg=pg,
        tree_cus=args.tree_cus if world == 1 else 0, tree_layout=args.tree_layout, seed=args.headline_seed)
    if hwd is not None:
        hwd.cancel()
    dt = head["dt"]
    # dist launches per call (snp_launch_mfma2: 256 x 256 tiles in batches of
    # 65536; no split-K at the headline's tile count)
    tiles = (-(-n // 256)) * (-(-n // 256) + 1) // 2 // world
    roof = headline_roofline(n, L, head["included_positions"], head.get("dist_elems", elems), head["dist_kernel_ms"],
                             max(1, -(-tiles // 65536)), pst, world, single_tree=args.tree_mode.startswith("gather"))
    pipe = head.get("pipelined")
    if pipe:   # the dist kernel ran on the dist context's share of the CUs
        dk = roof["kernels"]["dist"]
        dk["cus"] = pipe["dist_cus"]
        dk["frac_of_cu_share"] = round(dk["frac"] * (pipe["dist_cus"] + pipe["tree_cus"]) / pipe["dist_cus"], 4)
        if roof.get("kernel", "").startswith("k_snp_mfma"):
            roof["cus"], roof["frac_of_cu_share"] = dk["cus"], dk["frac_of_cu_share"]
    result = {
        "metric": "taxa-pairs/sec (dist) + NJ iterations/sec at N taxa, 1/2/4/8 MI355X",
        "value": round(m * args.steps / dt, 1),
        "unit": "taxa-pairs/s (dist + exact DNJ tree of the same matrix, end to end)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * dt / args.steps, 1),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u2 packed codes -> MX-fp4 MFMA (exact integer counts), f64 LT and tree",
        "data": f"synthetic: {n} taxa x {L} bp tree-like alignment (512 clades, ~0.8% of codes flipped per taxon, "
                f"every 10th 32-position word excluded), generated packed in HBM",
        "config": {"workload": f"configs[2]: ccphylo dist (MSA, non-pair) + ccphylo tree -m dnj (exact row sums) "
                               f"on {n} taxa x {L / 1e6:g} Mbp, one matrix per step",
                   "n_taxa": n, "alignment_length": L, "lt": "double",
                   "parallelism": (f"one GPU, pipelined: tree of matrix k on {pipe['tree_cus']} CUs "
                                   f"({pipe['layout']} layout) beside the dist of matrix k + 1 on the other "
                                   f"{pipe['dist_cus']}" if pipe else "one GPU")
                   if world == 1 else
                   (f"pipelined: GPU 0 builds the tree of matrix k (single-GPU engine) while GPUs 1..{world - 1} "
                    f"compute the dist of matrix k + 1 over LT row ranges and send them to GPU 0 over "
                    f"{args.shard_transport} point-to-point" if args.tree_mode == "gather-pipelined" else
                    f"dist: LT row ranges over {world} GPUs, gathered to GPU 0 over {args.shard_transport} "
                    f"point-to-point; tree: GPU 0 (single-GPU engine)" if args.tree_mode == "gather" else
                    f"LT row bands over {world} GPUs ({transport})")},
        "split": {"dist_s": round(head["dist_s"], 3), "tree_s": round(head["tree_s"], 3),
                  "overlap": "dist and tree run concurrently (pipelined); dist_s / tree_s: each context's device "
                             "time (HIP events on its stream)" if pipe else
                             "dist and tree walls run concurrently (pipelined)"
                             if head.get("gather_pipelined") else "sequential",
                  "dist_taxa_pairs_per_s": round(m / max(head["dist_s"], 1e-9), 1),
                  "dist_nt_comparisons_per_s": m * float(L) / max(head["dist_s"], 1e-9),
                  "tree_nj_iterations_per_s": round(head["joins"] / max(head["tree_s"], 1e-9), 1),
                  "joins": head["joins"], "joins_sha256": head["joins_sha256"],
                  **({"dist_wall_s": round(head["dist_wall_s"], 3), "tree_wall_s": round(head["tree_wall_s"], 3),
                      "joins_sha256_by_alignment": head["joins_sha256_by_alignment"]} if pipe else {}),
                  "rows_rescanned": head["rows_rescanned"], "cells_rescanned": head["cells_rescanned"],
                  "included_positions": head["included_positions"]},
        "roofline": roof,
    }
    if pst is not None and pst[11 + 2 * len(KNAMES)]:   # the whole tree, counted in the profiled step
        result["split"]["reference_rule_rows"] = int(pst[10 + 2 * len(KNAMES)])
        result["split"]["reference_rule_cells"] = int(pst[11 + 2 * len(KNAMES)])
        result["split"]["engine_over_reference_cells"] = round(head["cells_rescanned"] /
                                                               int(pst[11 + 2 * len(KNAMES)]), 3)
    log(f"headline: {result['value']:.4g} taxa-pairs/s, {result['ms_per_step']} ms per step")
    if rank == 0 and world == 1 and not args.no_cpu:
        log("headline cpu_baseline (reference dist + tree on 256 taxa)")
        try:
            with tempfile.TemporaryDirectory(dir="/tmp") as td:
                host = seqs[:256].cpu().numpy().view(np.uint64)
                result["cpu_baseline"] = headline_cpu_baseline(dev, host, incs.cpu().numpy().view(np.uint32), L,
                                                               cells, td)
        except Exception as e:  # noqa: BLE001
            result["cpu_baseline"] = {"error": str(e)}
    extras = result.setdefault("extras", {}) if not args.no_extras else None
    if extras is not None and world == 1 and pipe:
        # the same matrix step by step on the whole chip (dist, then tree): one matrix's latency
        log("headline, sequential form (each alignment once, whole chip)")
        try:
            D1 = torch.empty(m, dtype=torch.float64, device="cuda")
            seq = {}
            for a_, (sq_, ic_, _) in enumerate(head["alignments"]):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                dev.snp_ltd_dev(sq_.data_ptr(), ic_.data_ptr(), n, L, W, D1.data_ptr())
                t1 = time.perf_counter()
                j1, fn1, fd1, _ = dev.tree_dev(D1.data_ptr(), n, method=cg.CCG_TREE_DNJ, exact=True)
                t2 = time.perf_counter()
                sha1 = hashlib.sha256(np.ascontiguousarray(j1).tobytes() +
                                      np.array([fn1, fd1]).tobytes()).hexdigest()[:16]
                seq[str(a_)] = {"s_per_matrix": round(t2 - t0, 3), "dist_s": round(t1 - t0, 3),
                                "tree_s": round(t2 - t1, 3), "joins_sha256": sha1}
            del D1
            torch.cuda.empty_cache()
            pipe_sha = head["joins_sha256_by_alignment"]
            s_mean = sum(v["s_per_matrix"] for v in seq.values()) / len(seq)
            extras["headline_sequential"] = {
                "s_per_matrix": round(s_mean, 3), "taxa_pairs_per_s": round(m / s_mean, 1),
                "dist_s": seq["0"]["dist_s"], "tree_s": seq["0"]["tree_s"], "joins_sha256": seq["0"]["joins_sha256"],
                "by_alignment": seq,
                "pipelined_joins_match": all(pipe_sha.get(a_, [v["joins_sha256"]]) == [v["joins_sha256"]]
                                             for a_, v in seq.items()),
                "note": "one matrix's latency, dist then tree on all CUs, for each of the two alignments; the "
                        "line's value is the pipelined steady state (each step one whole dist and one whole tree, "
                        "on disjoint CUs, the matrices alternating between the two alignments)"}
        except Exception as e:  # noqa: BLE001
            extras["headline_sequential"] = {"error": str(e)}
    if extras is not None and rank == 0 and world == 1:
        log(f"reference-rule cells on a {args.refrule_prefix}-join prefix of the headline tree (oracle)")
        try:
            extras["refrule_config2_prefix"] = refrule_cells(dev, torch, seqs, incs, n, L, W, args.refrule_prefix,
                                                             oracle_threads)
        except Exception as e:  # noqa: BLE001
            extras["refrule_config2_prefix"] = {"error": str(e)}
    del seqs, incs
    head.pop("alignments", None)
    torch.cuda.empty_cache()
    if extras is not None:
        if rank == 0 and world == 1:
            log("configs[1] extras")
            try:
                with tempfile.TemporaryDirectory(dir="/tmp") as td:
                    extras["config1"] = config1_extras(dev, torch, td, n=args.c1_n, cpu=not args.no_cpu,
                                                       threads=oracle_threads)
            except Exception as e:  # noqa: BLE001
                extras["config1"] = {"error": str(e)}
            log("dist / kma extras")
            try:
                extras["dist_pair"] = dist_extra(dev, torch, pair=True)
            except Exception as e:  # noqa: BLE001
                extras["dist_pair"] = {"error": str(e)}
            try:
                extras["kma_cos"] = kma_extra(dev, torch)
            except Exception as e:  # noqa: BLE001
                extras["kma_cos"] = {"error": str(e)}
            torch.cuda.empty_cache()
        # every rank takes part (row-sharded dist); rank 0 reports
        try:
            extras["dist"] = dist_extra(dev, torch, rank=rank, world=world, dist=dist if world > 1 else None)
        except Exception as e:  # noqa: BLE001
            extras["dist"] = {"error": str(e)}
        if rank == 0 and world == 1 and not args.no_cpu:
            try:
                with tempfile.TemporaryDirectory(dir="/tmp") as td:
                    extras["dist"]["cpu_baseline"] = cpu_baseline_dist(td)
            except Exception as e:  # noqa: BLE001
                extras["dist"]["cpu_baseline"] = {"error": str(e)}
        torch.cuda.empty_cache()
        # the sharded legs last, under a watchdog: a collective that never
        # completes must not cost the whole line
        import threading

        def _timeout():
            # a hung collective: the line (with the legs marked) still prints,
            # and the process fails, so the driver's rc says so
            if rank == 0:
                for leg in ("dnj_sharded", "nj_sharded"):
                    extras.setdefault(leg, {"error": f"timed out after {SHARD_LEG_TIMEOUT_S} s"})
                print(json.dumps(result), flush=True)
            sys.stderr.write(f"bench.py: a sharded leg did not finish in {SHARD_LEG_TIMEOUT_S} s\n")
            sys.stderr.flush()
            os._exit(4)
        wd = threading.Timer(SHARD_LEG_TIMEOUT_S, _timeout)
        wd.daemon = True
        wd.start()
        log(f"configs[3]: DNJ on one 200k float matrix ({args.dnj_shard_joins or 'all'} joins)")
        try:
            extras["dnj_sharded"] = dnj_shard_extra(dev, torch, rank=rank, world=world,
                                                    dist=dist if world > 1 else None, coll=coll,
                                                    n=args.dnj_shard_n, joins=args.dnj_shard_joins)
        except Exception as e:  # noqa: BLE001
            extras["dnj_sharded"] = {"error": str(e)}
        torch.cuda.empty_cache()
        log("NJ on one 100k matrix")
        try:
            extras["nj_sharded"] = nj_shard_extra(dev, torch, rank=rank, world=world,
                                                  dist=dist if world > 1 else None, coll=coll, n=args.shard_n,
                                                  joins=args.shard_joins)
        except Exception as e:  # noqa: BLE001
            extras["nj_sharded"] = {"error": str(e)}
        wd.cancel()
    log("done")
    if coll is not None and hasattr(coll, "close"):
        coll.close()
    dev.close()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
