#!/usr/bin/env python3
"""bench.py -- headline benchmark of ccphylo_amd (driver contract).

Metric (BASELINE.json): "taxa-pairs/sec (dist) + NJ iterations/sec at N taxa".
`value` is NJ iterations (joins) per second of `ccphylo tree -m dnj` (the
reference's default method, which yields the exact NJ join sequence) on
configs[1]: an N=10,000-taxon distance matrix, one full tree per step, the
packed LT already resident in HBM when the timed region starts (one fresh
device copy per step; the engine consumes its input).  Row sums are exact
(the CLI default): the join list and the Newick bytes equal the reference's,
checked in the cpu_baseline leg against the reference binary's own output.
extras.dnj_fast_sums is the non-default --fast_sums mode with its parity
status at this config (join list identical or not, splits differing).

extras.config3: configs[2], the largest single-GPU configuration: a 50k taxa
x 5 Mbp synthetic tree-like alignment, packed in HBM -> dist -> exact DNJ in
place, steps-timed, with its own roofline (dist: VALU issue; tree: HBM) and
cpu_baseline (the reference's `dist -t <threads>` on row subsamples of the
same alignment written as FASTA, whose distances are also compared with the
GPU's cells).

Multi-GPU (torchrun, one process per GPU): every rank builds its own N=10k
tree on its own GPU ("replicas") -> scaling "weak", value = all ranks' joins
divided by the max over ranks of the timed span.  One N=10k tree does not
gain from more GPUs (a join is ~35 us of dependent steps); the sharded path is
measured where it pays, in extras.nj_sharded: ONE N=100k matrix (40 GB) with
its LT row bands dealt over all ranks, NJ joins with RCCL exchanges
(ccg_tree_shard_dev), strong scaling; and extras.dnj_sharded,
configs[3]: ONE N=200k matrix (float, 80 GB) sharded the same way, DNJ joins.

Also reported: the dominant kernel's roofline (HIP-event timing of every
kernel in one profiled extra step on the engine stream; algorithmic bytes as
defined in DESIGN.md; `traffic` from the committed rocprofv3 PMC summary of
the same kernel, profiles/r02_pmc.json, when present), the reference CPU path
on the same matrix (rank 0, N=1), and extras (exact-row-sum mode, -m nj, and
SNP `dist` throughput).
"""
import argparse
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
# dist roofline: 32-bit integer VALU issue.  A 32-position word pair costs 3
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
# (MI355X_MICROARCH.md); tools/micro/mfma_fp4 (profiles/r02_mfma_fp4.txt)
# issues 3.55e15 MAC/s = 7.1 PF from registers on this box.
MFMA_FP4_DENSE_TFLOPS = 10000.0
MFMA_FP4_MEASURED_TFLOPS = 7098.0
FLOPS_PER_POSITION_PAIR = 6.0
VALU_INT32_CEILING = 256 * 4 * 16 * 2.4e9
OPS_PER_WORD_PAIR = 3.0
OPS_PER_WORD_PAIR_PAIRMODE = 6.0   # v_and (masks), v_xor, v_bitop3, v_and, 2x v_bcnt (dist and n)
KNAMES = ["init", "dnj_select", "dnj_scan", "nj_argmin", "update", "dnj_requeue", "nj_pop", "dnj_find", "coll",
          "exact_sum"]
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r02_pmc.json")
SHARD_LEG_TIMEOUT_S = 480


from tools.synth import euclid as euclid_ltd  # noqa: E402


def algorithmic_bytes_total(kernel, n, s, cells_select, cells_scan):
    """Compulsory HBM bytes of all launches of one class over a whole tree
    (joins at matrix sizes n .. 3); DESIGN.md, 'Roofline accounting'.
    s = bytes per D element; the n-vectors are f64 (sD, Q) and i32 (N, P)."""
    sizes = range(3, n + 1)
    sn = float(sum(sizes))
    if kernel == "dnj_select":      # (sharded engine) rescanned D cells of S + the sD vector once
        return s * cells_select + 8.0 * sn
    if kernel == "dnj_scan":        # one GPU: every rescanned D cell (S and the rows below it) + the sD vector once
        return s * (cells_select + cells_scan) + 8.0 * sn
    if kernel == "dnj_find":        # k_dnj_plan: Q of every row; P, the partner cell, sD of row and partner
        return 8.0 * sn + (20.0 + s) * float(sum(min(k - 1, 960) for k in sizes))   # for the top rows
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


KERNEL_STATS = os.path.join(ROOT, "profiles", "r02_kernel_stats.csv")
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


def roofline(stats, n, s):
    """Dominant kernel (largest total device time) of a profiled run."""
    per = {}
    for c, name in enumerate(KNAMES):
        cnt, ns = stats[4 + 2 * c], stats[5 + 2 * c]
        if cnt:
            per[name] = (cnt, ns)
    name = max(per, key=lambda k: per[k][1])
    cnt, ns = per[name]
    tot = algorithmic_bytes_total(name, n, s, stats[4 + 2 * len(KNAMES)], stats[5 + 2 * len(KNAMES)])
    avg_s = ns / cnt / 1e9
    achieved = tot / cnt / avg_s / 1e9
    shares = {k: round(v[1] / sum(x[1] for x in per.values()), 4) for k, v in per.items()}
    kernels = {}
    for k, (c, t) in per.items():   # every kernel class: algorithmic bytes, HIP-event and rocprof rates, PMC bytes
        if k == "init":
            continue
        ab = algorithmic_bytes_total(k, n, s, stats[4 + 2 * len(KNAMES)], stats[5 + 2 * len(KNAMES)]) / c
        ev = t / c / 1e9
        rp = rocprof_mean_us(k)
        kernels[k] = {"algorithmic_bytes_per_launch": round(ab, 1), "avg_launch_us": round(ev * 1e6, 3),
                      "frac": round(ab / ev / 1e9 / HBM_PEAK_GBS, 5), "traffic": pmc_traffic(k)[0]}
        if rp:
            kernels[k]["rocprof_mean_us"] = rp
            kernels[k]["frac_rocprof_duration"] = round(ab / (rp * 1e-6) / 1e9 / HBM_PEAK_GBS, 5)
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


def cpu_baseline(D, n, tmpdir, threads=(1, 16)):
    """The reference binary (oracle/_ref, built from /root/reference by
    oracle/Makefile) on the same matrix written as Phylip, with 1 and 16
    pthreads (`-t`, the box's CPU share); the faster is the baseline.  Falls
    back to the oracle's C restatement in-process."""
    ref = os.path.join(ROOT, "oracle", "_ref", "ccphylo")
    if os.path.exists(ref):
        from ccphylo_amd import native
        path = os.path.join(tmpdir, "bench_ref.phy")
        native.write_phylip(path, D, n, [f"t{k}" for k in range(n)])
        runs = {}
        for t in threads:
            t0 = time.perf_counter()
            p = subprocess.run([ref, "tree", "-i", path, "-m", "dnj", "-t", str(t), "-o",
                                os.path.join(tmpdir, "ref.nwk")], capture_output=True, text=True, timeout=900)
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
        return {"value": round((n - 2) / cons, 2), "unit": "NJ joins/s", "cores": best, "kind": "reference",
                "sample": f"full N={n} DNJ tree, reference ccphylo 0.8.5 `tree -m dnj` on the same matrix "
                          f"(Phylip %.9f), best of {list(threads)} pthreads ({desc}); 1-thread time is the "
                          f"reference's own 'Constructing tree' report, multi-thread time is process wall "
                          f"minus its 'loading matrix' report"}
    from oracle import pyoracle
    t0 = time.perf_counter()
    j, _, _ = pyoracle.tree(D, n, method=1)
    dt = time.perf_counter() - t0
    return {"value": round(len(j) / dt, 2), "unit": "NJ joins/s", "cores": 1, "kind": "port",
            "sample": f"full N={n} DNJ tree with the oracle's serial C restatement (reference binary absent)"}


def cpu_baseline_dist(tmpdir, sizes=(1024, 2048), L=20_000, threads=16):
    """The reference's `ccphylo dist` (oracle/_ref, -t 16) on random MSAs of
    `sizes` taxa x L bp (FASTA text, seeded; the data of the GPU dist leg).  The process wall time is
    parse + compare; with two sizes, t = a n + b n^2 separates the quadratic
    (compare) term, whose rate is reported as nt-comparisons/s."""
    import numpy as np
    ref = os.path.join(ROOT, "oracle", "_ref", "ccphylo")
    if not os.path.exists(ref):
        return None
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
    mfma = os.environ.get("CCG_DIST_MFMA", "1") != "0"
    del seqs, incs, Dd, Nd
    mode = "pair mode -f 3, D and N" if pair else "non-pair"
    return {"taxa_pairs_per_s": round(m / dt, 1), "nt_comparisons_per_s": m * L / dt, "seconds": round(dt, 4),
            "config": f"N={n} x L={L} random MSA ({mode}, double), input in HBM, LT rows sharded over {world} GPU(s)",
            "kernel": ("k_snp_mfma_pair" if pair else "k_snp_mfma") if mfma else ("k_snp_tile_pair" if pair else "k_snp_tile"),
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
            "evidence": "profiles/r02_mfma_fp4.txt (tools/micro/mfma_fp4: lane map, register-fed rate)"}


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


def config3_cpu_baseline(seqs_host, L, masked_words, tmpdir, gpu_cells, sizes=(96, 192), threads=16):
    """The reference's `ccphylo dist -t <threads>` (oracle/_ref, built from
    the reference's sources) on the first 96 and 192 taxa of the configs[2]
    alignment written as FASTA.  Wall = parse + compare; t = a n + b n^2
    separates the compare term.  The reference's distances for those taxa are
    compared with the GPU's LT cells (same rows)."""
    ref = os.path.join(ROOT, "oracle", "_ref", "ccphylo")
    if not os.path.exists(ref):
        return {"error": "reference binary absent (oracle/_ref not built)"}
    walls, mism = {}, 0
    for m in sizes:
        path = os.path.join(tmpdir, f"c3_{m}.fsa")
        packed_rows_to_fasta(path, seqs_host[:m], L, masked_words)
        out = os.path.join(tmpdir, f"c3_{m}.phy")
        t0 = time.perf_counter()
        subprocess.run([ref, "dist", "-i", path, "-t", str(threads), "-o", out], capture_output=True, timeout=900,
                       check=True)
        walls[m] = time.perf_counter() - t0
        os.unlink(path)
        nn, vals = read_phylip_values(out)
        os.unlink(out)
        k = m * (m - 1) // 2
        mism += int(nn != m) + int((vals != gpu_cells[:k]).sum())
    (n1, t1), (n2, t2) = sorted(walls.items())
    b = (t2 / n2 - t1 / n1) / (n2 - n1)          # t / n = a + b n
    pairs_s = 0.5 / b if b > 0 else None
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count()
    return {"value": round(pairs_s, 2) if pairs_s else None, "unit": "taxa-pairs/s", "cores": threads,
            "host_cpus_available": ncpu, "kind": "reference",
            "nt_comparisons_per_s": round(pairs_s * L, 1) if pairs_s else None,
            "parity_mismatched_cells": mism,
            "sample": f"reference ccphylo 0.8.5 `dist -t {threads}` on the first {list(sizes)} taxa of the same "
                      f"{L / 1e6:g} Mbp alignment (FASTA); walls " +
                      ", ".join(f"{m} taxa: {w:.2f} s" for m, w in sorted(walls.items())) +
                      "; the rate is the quadratic (compare) term of t = a n + b n^2; its distances equal the GPU's "
                      "LT cells of the same taxa when parity_mismatched_cells is 0"}


def config3_leg(dev, torch, tmpdir, n=50_000, L=5_000_000, steps=1, cpu=True):
    """configs[2]: N=50k taxa x L=5 Mbp synthetic tree-like alignment on one
    GPU, end to end in HBM: packed sequences (62.5 GB) -> ccg_snp_ltd_dev
    (double LT, 10 GB) -> ccg_tree_dev DNJ with exact row sums, in place.  A
    step = dist + tree (steps-timed); the alignment is generated once."""
    import ccphylo_amd as cg
    from tools.config3 import make_packed
    W = L // 32 + 1
    seqs = make_packed(torch, n, W)
    incs = torch.full((W,), -1, dtype=torch.int32, device="cuda")
    masked_words = list(range(0, (L + 31) // 32, 10))
    incs[::10] = 0
    incs[(L + 31) // 32:] = 0
    m = n * (n - 1) // 2
    D = torch.empty(m, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    t_dist, t_tree, joins, cells, rows = [], [], 0, 0, 0
    first_cells = None
    for k in range(steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        inc = dev.snp_ltd_dev(seqs.data_ptr(), incs.data_ptr(), n, L, W, D.data_ptr())
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if first_cells is None:   # the LT block of the first 192 taxa, for the reference check
            first_cells = D[:192 * 191 // 2].cpu().numpy()
            torch.cuda.synchronize()
            t1b = time.perf_counter()
        else:
            t1b = t1
        j, fn, fd, st = dev.tree_dev(D.data_ptr(), n, method=cg.CCG_TREE_DNJ, exact=True)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        t_dist.append(t1 - t0)
        t_tree.append(t2 - t1b)
        joins, rows, cells = len(j), int(st[0]), int(st[1])
    dist_s, tree_s = sum(t_dist) / steps, sum(t_tree) / steps
    words = (L + 31) // 32
    ops = m * words * OPS_PER_WORD_PAIR
    # tree HBM bytes: initSummaD + initHNJ (two LT passes), the rescanned cells,
    # and per join the O(n) update / requeue / row-sum traffic
    sizes_sum = n * (n + 1) / 2.0
    tree_bytes = 2.0 * 8 * m + 8.0 * cells + (7 * 8 + 48) * sizes_sum
    res = {"n": n, "L": L, "steps": steps, "ms_per_step": round(1000 * (dist_s + tree_s), 1),
           "dist_s": round(dist_s, 3), "tree_s": round(tree_s, 3),
           "taxa_pairs_per_s": round(m / dist_s, 1), "nt_comparisons_per_s": m * L / dist_s,
           "joins_per_s": round(joins / tree_s, 1), "joins": joins, "rows_rescanned": rows,
           "cells_rescanned": cells, "included_positions": inc, "row_sums": "exact",
           "roofline": {"dist": mfma_roofline(m * L, dist_s) if os.environ.get("CCG_DIST_MFMA", "1") != "0"
                        else valu_roofline(ops, dist_s, OPS_PER_WORD_PAIR),
                        "tree": {"bound": "hbm", "achieved": round(tree_bytes / tree_s / 1e9, 1),
                                 "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": round(tree_bytes / tree_s / 1e9 / HBM_PEAK_GBS, 4),
                                 "algorithmic_bytes": tree_bytes,
                                 "note": "2 LT passes (init) + 8 B per rescanned cell + ~104 B per active taxon per "
                                         "join; latency-bound joins, see DESIGN.md 4"}},
           "tree_parity": "exact row sums; tests/test_gpu_large.py::test_config2_dist_and_dnj_prefix pins this "
                          "configuration's dist cells (fsacmp) and DNJ join prefix against the oracle"}
    del D, incs
    torch.cuda.empty_cache()
    if cpu:
        try:
            host = seqs[:192].cpu().numpy().view(np.uint64)
            res["cpu_baseline"] = config3_cpu_baseline(host, L, masked_words, tmpdir, first_cells)
        except Exception as e:  # noqa: BLE001
            res["cpu_baseline"] = {"error": str(e)}
    del seqs
    torch.cuda.empty_cache()
    return res


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


def nj_shard_extra(dev, torch, rank=0, world=1, dist=None, n=100_000, joins=64, transport="rccl"):
    """NJ with the LT rows sharded over the ranks (ccg_tree_shard_dev; SURVEY
    8(e)): rank g holds the row bands g, g + world, ... of ONE n-taxon matrix
    (n = 100k, double: 40 GB in all), collectives over RCCL (world > 1) --
    strong scaling of one tree.  Timed: the first `joins` joins (each a full
    initQ scan of the whole matrix), as time(joins + 1) - time(1) so the exact
    initSummaD and the setup are excluded.  Every rank takes part."""
    import ccphylo_amd as cg
    from ccphylo_amd import native as nt
    from tools.synth import euclid_shard_dev
    coll = None
    if world > 1:
        coll = nt.RcclColl(dev, dist) if transport == "rccl" else nt.HostColl(dist)
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

    try:
        t1, _ = run(1)
        tk, _ = run(joins + 1)
        _, pst = run(joins + 1, profile=True)
    finally:
        if coll is not None and transport == "rccl":
            coll.close()
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
            "config": f"NJ (-m nj) on one N={n} Euclidean matrix (double, {8 * n * (n - 1) / 2 / 1e9:.1f} GB) with "
                      f"its LT row bands dealt over {world} GPU(s) ({transport if world > 1 else 'no'} transport); "
                      f"first {joins} joins; fast row sums",
            "hbm_GBps_aggregate": round(gb, 1), "hbm_frac_aggregate": round(gb / (HBM_PEAK_GBS * world), 4),
            "argmin_kernel_GBps_per_gpu": round(kern_gb, 1) if kern_gb else None,
            "coll_us_per_join": round(pst[5 + 2 * 8] / 1e3 / (joins + 1), 2) if pst[4 + 2 * 8] else 0.0}


def dnj_shard_extra(dev, torch, rank=0, world=1, dist=None, n=200_000, joins=4000, transport="rccl"):
    """configs[3]: DNJ with the LT rows sharded over the ranks (ccg_tree_shard_dev
    with CCG_TREE_DNJ): ONE n-taxon Euclidean matrix (n = 200k,
    float = `-p`: 80 GB in all), rank g holding the row bands g, g + world, ...;
    collectives over RCCL (world > 1).  Timed: the first `joins` joins, as
    time(joins + 1) - time(1), so the exact initSummaD, initHNJ and the setup
    are excluded.  Every rank takes part."""
    import ccphylo_amd as cg
    from ccphylo_amd import native as nt
    from tools.synth import euclid_shard_dev
    coll = None
    if world > 1:
        coll = nt.RcclColl(dev, dist) if transport == "rccl" else nt.HostColl(dist)
    loc = euclid_shard_dev(torch, n, rank, world, dtype=torch.float32)
    work = torch.empty_like(loc)

    def run(k):
        work.copy_(loc)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        j, fn, fd, st = dev.tree_shard_dev(work.data_ptr(), n, coll, etype=4, method=cg.CCG_TREE_DNJ, exact=False,
                                           max_joins=k)
        dt = time.perf_counter() - t0
        assert len(j) == k, (len(j), k)
        return shard_max(dt, dist), st

    try:
        t1, _ = run(1)
        tk, st = run(joins + 1)
    finally:
        if coll is not None and transport == "rccl":
            coll.close()
    dt = tk - t1
    del loc, work
    torch.cuda.empty_cache()
    return {"joins_per_s": round(joins / dt, 2), "ms_per_join": round(1000 * dt / joins, 4), "joins": joins,
            "n": n, "world": world, "seconds": round(dt, 4),
            "rows_rescanned_rank0": int(st[0]), "cells_rescanned_rank0": int(st[1]),
            "config": f"configs[3]: DNJ (-m dnj) on one N={n} Euclidean matrix (float, "
                      f"{4 * n * (n - 1) / 2 / 1e9:.0f} GB) with its LT row bands dealt over {world} GPU(s) "
                      f"({transport if world > 1 else 'no'} transport); first {joins} joins; fast row sums"}


def shard_max(x, dist):
    if dist is None:
        return x
    from ccphylo_amd import shard
    return shard.reduce_max(x, dist)


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=10000)
    ap.add_argument("--sums", choices=["fast", "exact"], default="exact")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--no-config3", action="store_true", help="skip the 50k x 5M dist+tree leg (~1 min)")
    ap.add_argument("--c3-steps", type=int, default=1)
    ap.add_argument("--shard-n", type=int, default=100_000)
    ap.add_argument("--shard-joins", type=int, default=64)
    ap.add_argument("--dnj-shard-n", type=int, default=200_000)
    ap.add_argument("--dnj-shard-joins", type=int, default=4000)
    ap.add_argument("--shard-transport", choices=["rccl", "gloo"], default="rccl",
                    help="gloo: host-staged (rehearsal of several ranks on one GPU)")
    args = ap.parse_args()

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

    n = args.n
    s = 8
    D = euclid_ltd(n, seed=1)
    dev = cg.Device(gpu)
    exact = args.sums == "exact"
    nbytes = D.nbytes
    bufs = [dev.malloc(nbytes) for _ in range(args.steps + args.warmup)]
    for b in bufs:
        dev.h2d(b, D)
    for w in range(args.warmup):
        dev.tree_dev(bufs[w], n, method=cg.CCG_TREE_DNJ, exact=exact)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    joins = 0
    for k in range(args.steps):
        j, fn, fd, st = dev.tree_dev(bufs[args.warmup + k], n, method=cg.CCG_TREE_DNJ, exact=exact)
        joins += len(j)
    barrier()
    dt = time.perf_counter() - t0
    main_joins = (j, fn, fd)
    if world > 1:
        t = torch.tensor([dt])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t[0])
        jt = torch.tensor([joins], dtype=torch.float64)
        dist.all_reduce(jt, op=dist.ReduceOp.SUM)
        joins_all = float(jt[0])
    else:
        joins_all = float(joins)
    for b in bufs:
        dev.free(b)

    # one profiled extra step (HIP events around every kernel, engine stream)
    pb = dev.malloc(nbytes)
    dev.h2d(pb, D)
    _, _, _, pst = dev.tree_dev(pb, n, method=cg.CCG_TREE_DNJ, exact=exact, profile=True)
    dev.free(pb)
    roof = roofline(pst, n, s)
    roof["row_sums_serial_order"] = int(pst[6 + 2 * len(KNAMES)])
    roof["row_sums_by_serial_chain"] = int(pst[7 + 2 * len(KNAMES)])

    result = {
        "metric": "taxa-pairs/sec (dist) + NJ iterations/sec at N taxa, 1/2/4/8 MI355X",
        "value": round(joins_all / dt, 2),
        "unit": "NJ iterations (joins)/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * dt / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": f"synthetic: N={n} Euclidean distances of U[0,1)^8 points (seed 1), quantized to 9 decimals "
                f"as a %.9f Phylip would be; one full tree per step per GPU",
        "config": {"workload": f"ccphylo tree -m dnj (configs[1]: N={n} synthetic Phylip matrix, NJ/DNJ on 1 "
                               f"MI355X per rank)", "n_taxa": n, "method": "dnj", "elem": "double",
                   "row_sums": args.sums, "parallelism": f"replicas x{world}"},
        "roofline": roof,
    }
    fast_joins = None
    if rank == 0 and world == 1 and not args.no_extras:
        extras = {}
        pb = dev.malloc(nbytes)
        other = "dnj_exact_sums" if not exact else "dnj_fast_sums"
        for label, method, ex in ((other, cg.CCG_TREE_DNJ, not exact),
                                  ("nj", cg.CCG_TREE_NJ, exact), ("hnj", cg.CCG_TREE_HNJ, exact)):
            dev.h2d(pb, D)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            j2, fn2, fd2, st = dev.tree_dev(pb, n, method=method, exact=ex)
            t2 = time.perf_counter() - t1
            extras[label] = {"joins_per_s": round(len(j2) / t2, 2), "seconds": round(t2, 4),
                             "row_sums": "exact" if ex else "fast"}
            if label == "dnj_fast_sums":
                fast_joins = (j2, fn2, fd2)
        dev.h2d(pb, D)
        _, _, _, nst = dev.tree_dev(pb, n, method=cg.CCG_TREE_NJ, exact=exact, profile=True)
        extras["nj"]["roofline"] = roofline(nst, n, s)
        dev.free(pb)
        result["extras"] = extras
    if not args.no_extras:
        # every rank takes part (row-sharded dist); rank 0 reports
        try:
            d = dist_extra(dev, torch, rank=rank, world=world, dist=dist if world > 1 else None)
        except Exception as e:  # noqa: BLE001
            d = {"error": str(e)}
        result.setdefault("extras", {})["dist"] = d
        if world == 1:
            try:
                result["extras"]["dist_pair"] = dist_extra(dev, torch, pair=True)
            except Exception as e:  # noqa: BLE001
                result["extras"]["dist_pair"] = {"error": str(e)}
            try:
                result["extras"]["kma_cos"] = kma_extra(dev, torch)
            except Exception as e:  # noqa: BLE001
                result["extras"]["kma_cos"] = {"error": str(e)}
            if not args.no_config3:
                # configs[2]: N=50k x L=5M tree-like alignment -> dist -> exact DNJ, all in HBM
                try:
                    torch.cuda.empty_cache()
                    with tempfile.TemporaryDirectory(dir="/tmp") as td:
                        c3 = config3_leg(dev, torch, td, steps=args.c3_steps, cpu=not args.no_cpu)
                    c3["config"] = ("configs[2]: 50k taxa x 5 Mbp synthetic tree-like alignment (512 clades, ~0.8% "
                                    "codes flipped per taxon), packed in HBM -> ccg_snp_ltd_dev (double LT, 10 GB) "
                                    "-> ccg_tree_dev DNJ with exact row sums")
                    result["extras"]["config3"] = c3
                except Exception as e:  # noqa: BLE001
                    result["extras"]["config3"] = {"error": str(e)}
                torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_cpu:
        with tempfile.TemporaryDirectory(dir="/tmp") as td:
            result["cpu_baseline"] = cpu_baseline(D, n, td)
            if exact:
                try:
                    par = reference_tree_parity(D, n, main_joins, fast_joins, td)
                    result["cpu_baseline"]["parity"] = par
                    if "dnj_fast_sums" in result.get("extras", {}):
                        result["extras"]["dnj_fast_sums"]["parity_vs_exact"] = {
                            k: v for k, v in par.items() if k.startswith("fast")}
                except Exception as e:  # noqa: BLE001
                    result["cpu_baseline"]["parity"] = {"error": str(e)}
            if not args.no_extras and isinstance(result.get("extras", {}).get("dist"), dict):
                try:
                    result["extras"]["dist"]["cpu_baseline"] = cpu_baseline_dist(td)
                except Exception as e:  # noqa: BLE001
                    result["extras"]["dist"]["cpu_baseline"] = {"error": str(e)}
    if not args.no_extras:
        # last, under a watchdog: a collective that never completes (e.g. an
        # RCCL bootstrap failure on one rank) must not cost the whole line
        import threading

        def _timeout():
            if rank == 0:
                for leg in ("nj_sharded", "dnj_sharded"):
                    result["extras"].setdefault(leg, {"error": f"timed out after {SHARD_LEG_TIMEOUT_S} s"})
                print(json.dumps(result), flush=True)
            os._exit(0)
        wd = threading.Timer(SHARD_LEG_TIMEOUT_S, _timeout)
        wd.daemon = True
        wd.start()
        try:
            d = nj_shard_extra(dev, torch, rank=rank, world=world, dist=dist if world > 1 else None, n=args.shard_n,
                               joins=args.shard_joins, transport=args.shard_transport)
        except Exception as e:  # noqa: BLE001
            d = {"error": str(e)}
        result["extras"]["nj_sharded"] = d
        torch.cuda.empty_cache()
        try:
            d = dnj_shard_extra(dev, torch, rank=rank, world=world, dist=dist if world > 1 else None,
                                n=args.dnj_shard_n, joins=args.dnj_shard_joins, transport=args.shard_transport)
        except Exception as e:  # noqa: BLE001
            d = {"error": str(e)}
        wd.cancel()
        result["extras"]["dnj_sharded"] = d
    dev.close()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
