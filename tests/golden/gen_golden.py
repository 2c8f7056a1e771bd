#!/usr/bin/env python3
"""Generates the golden vectors of tests/golden/ by running the REFERENCE
ccphylo 0.8.5 binary built by oracle/Makefile (oracle/_ref/ccphylo) on
synthetic inputs made here with fixed seeds, plus the reference's own bundled
fixture test.phy.gz.  Run in the build container (needs /root/reference):

    make -C oracle && python tests/golden/gen_golden.py

Outputs (all data, committed): inputs *.fsa / *.phy(.gz) and expected outputs
*.out, listed with their command lines in golden.json.
"""
import gzip
import hashlib
import json
import os
import random
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(ROOT, "oracle", "_ref", "ccphylo")


def msa(path, n, L, seed, mut=0.03, nrate=0.002, gaps=True, lower=True, iupac=True, crlf=False, wrap=60,
        exclude=1, tree_like=True):
    """Writes a FASTA MSA.  Taxa descend from random ancestors (tree_like) so
    the distance matrix has real structure and many ties."""
    rng = random.Random(seed)
    base = [rng.choice("ACGT") for _ in range(L)]
    pool = [base]
    seqs = []
    for t in range(n):
        parent = rng.choice(pool) if tree_like else base
        s = list(parent)
        for p in range(L):
            if rng.random() < mut:
                s[p] = rng.choice("ACGT")
        if tree_like and rng.random() < 0.3:
            pool.append(s[:])
        for p in range(L):
            r = rng.random()
            if r < nrate:
                s[p] = "N"
            elif gaps and r < 2 * nrate:
                s[p] = "-"
            elif iupac and r < 2.5 * nrate:
                s[p] = rng.choice("RYSWKMBDHVX")
            elif lower and r < 3.5 * nrate:
                s[p] = s[p].lower()
        seqs.append(s)
    for t in range(exclude):   # mostly-N taxa: excluded by minCov (cdist.c:270)
        k = rng.randrange(n)
        for p in range(L):
            if rng.random() < 0.7:
                seqs[k][p] = "N"
    nl = "\r\n" if crlf else "\n"
    with open(path, "w", newline="") as f:
        for t, s in enumerate(seqs):
            f.write(f">taxon_{t:03d} sample/{t}{nl}")
            txt = "".join(s)
            for k in range(0, L, wrap):
                f.write(txt[k:k + wrap] + nl)


def euclid_phy(path, n, seed, dim=8, fmt="%.9f", gz=False):
    rng = random.Random(seed)
    pts = [[rng.random() for _ in range(dim)] for _ in range(n)]
    op = gzip.open if gz else open
    with op(path, "wt") as f:
        f.write("%10d\n" % n)
        for i in range(n):
            row = [f"e{i}"]
            for j in range(i):
                d = sum((a - b) ** 2 for a, b in zip(pts[i], pts[j])) ** 0.5
                row.append(fmt % d)
            f.write("\t".join(row) + "\n")


def kma_sample(path, templates, seed, depth=30, ins=0.0, gz=True, skip=(), trunc=None):
    """A KMA count matrix (*.mat[.gz]): per template "#name", one row per
    position "ref A C G T N -" (tab separated), a blank line at the end.
    `ins` adds insertion rows (ref '-'); `trunc` cuts a template short."""
    rng = random.Random(seed)
    op = gzip.open if gz else open
    with op(path, "wt") as f:
        for name, ref in templates:
            if name in skip:
                continue
            f.write(f"#{name}\n")
            rows = ref if not trunc or name not in trunc else ref[:trunc[name]]
            for b in rows:
                dep = max(0, int(rng.gauss(depth, depth / 3)))
                c = [0] * 6
                base = "ACGT".index(b) if rng.random() > 0.02 else rng.randrange(4)
                for _ in range(dep):
                    r = rng.random()
                    if r < 0.9:
                        c[base] += 1
                    elif r < 0.97:
                        c[rng.randrange(4)] += 1
                    elif r < 0.985:
                        c[4] += 1
                    else:
                        c[5] += 1
                f.write(b + "\t" + "\t".join(map(str, c)) + "\n")
                if ins and rng.random() < ins:
                    c = [0] * 6
                    c[rng.randrange(4)] = rng.randrange(1, 20)
                    c[5] = rng.randrange(0, 10)
                    f.write("-\t" + "\t".join(map(str, c)) + "\n")
            f.write("\n")


def run(args, out):
    p = subprocess.run([REF] + args, capture_output=True, check=True)
    with open(out, "wb") as f:
        f.write(p.stdout)
    return hashlib.md5(p.stdout).hexdigest()


def main():
    if not os.path.exists(REF):
        sys.exit("build the reference first: make -C oracle")
    os.chdir(HERE)
    cases = []

    def case(name, args, out, kind):
        md5 = run(args, out)
        cases.append({"name": name, "kind": kind, "args": args, "out": out, "md5": md5})

    # (i) the reference's bundled fixture
    shutil.copyfile("/root/reference/test.phy.gz", "test.phy.gz")
    for m in ("dnj", "nj"):
        case(f"test_{m}", ["tree", "-i", "test.phy.gz", "-m", m], f"test_{m}.out", "tree")
    case("test_dnj_p", ["tree", "-i", "test.phy.gz", "-p"], "test_dnj_p.out", "tree")
    case("test_dnj_f1", ["tree", "-i", "test.phy.gz", "-f", "1"], "test_dnj_f1.out", "tree")
    case("test_dnj_f2", ["tree", "-i", "test.phy.gz", "-f", "2"], "test_dnj_f2.out", "tree")
    case("test_dnj_x4", ["tree", "-i", "test.phy.gz", "-x", "4"], "test_dnj_x4.out", "tree")
    case("test_dnj_s", ["tree", "-i", "test.phy.gz", "-s", "1000"], "test_dnj_s.out", "tree")
    case("test_nj_b", ["tree", "-i", "test.phy.gz", "-m", "nj", "-b", "100"], "test_nj_b.out", "tree")

    # (ii) MSAs -> dist
    msa("msa64.fsa", 64, 3000, seed=1)
    msa("msa_crlf.fsa", 40, 2500, seed=2, crlf=True, wrap=70)
    msa("msa_odd.fsa", 33, 1027, seed=3, exclude=2)      # len % 32 != 0, two excluded taxa
    msa("msa_word.fsa", 48, 2048, seed=4, exclude=0)     # len % 32 == 0
    for f in ("msa64.fsa", "msa_crlf.fsa", "msa_odd.fsa", "msa_word.fsa"):
        b = f[:-4]
        case(f"{b}_f1", ["dist", "-i", f], f"{b}_f1.out", "dist")
        case(f"{b}_f3", ["dist", "-i", f, "-f", "3"], f"{b}_f3.out", "dist")
    b = "msa64"
    case(f"{b}_f0", ["dist", "-i", "msa64.fsa", "-f", "0"], f"{b}_f0.out", "dist")
    case(f"{b}_f9", ["dist", "-i", "msa64.fsa", "-f", "9"], f"{b}_f9.out", "dist")
    case(f"{b}_f33", ["dist", "-i", "msa64.fsa", "-f", "33"], f"{b}_f33.out", "dist")
    case(f"{b}_f11", ["dist", "-i", "msa64.fsa", "-f", "11"], f"{b}_f11.out", "dist")
    case(f"{b}_W", ["dist", "-i", "msa64.fsa", "-W", "1000"], f"{b}_W.out", "dist")
    case(f"{b}_f3W", ["dist", "-i", "msa64.fsa", "-f", "3", "-W", "1000"], f"{b}_f3W.out", "dist")
    case(f"{b}_p", ["dist", "-i", "msa64.fsa", "-p"], f"{b}_p.out", "dist")
    case(f"{b}_f3pW", ["dist", "-i", "msa64.fsa", "-f", "3", "-p", "-W", "999"], f"{b}_f3pW.out", "dist")
    case(f"{b}_s", ["dist", "-i", "msa64.fsa", "-s", "10"], f"{b}_s.out", "dist")
    case(f"{b}_f3sW", ["dist", "-i", "msa64.fsa", "-f", "3", "-s", "2", "-W", "100"], f"{b}_f3sW.out", "dist")
    case(f"{b}_b", ["dist", "-i", "msa64.fsa", "-b"], f"{b}_b.out", "dist")
    case(f"{b}_P", ["dist", "-i", "msa64.fsa", "-P", "10"], f"{b}_P.out", "dist")
    case(f"{b}_P2", ["dist", "-i", "msa_odd.fsa", "-P", "2"], f"msa_odd_P2.out", "dist")
    # pair mode with proximity masking (maskProxi, fsacmp.c:355)
    case("msa64_f3P10", ["dist", "-i", "msa64.fsa", "-f", "3", "-P", "10"], "msa64_f3P10.out", "dist")
    case("msa_odd_f3P2", ["dist", "-i", "msa_odd.fsa", "-f", "3", "-P", "2"], "msa_odd_f3P2.out", "dist")
    case("msa_word_f3P40W", ["dist", "-i", "msa_word.fsa", "-f", "3", "-P", "40", "-W", "1000"],
         "msa_word_f3P40W.out", "dist")
    case("msa64_f3P5pn", ["dist", "-i", "msa64.fsa", "-f", "3", "-P", "5", "-p", "-n", "/dev/null"],
         "msa64_f3P5pn.out", "dist")
    case("msa_crlf_f3P100s", ["dist", "-i", "msa_crlf.fsa", "-f", "3", "-P", "100", "-s", "10"],
         "msa_crlf_f3P100s.out", "dist")
    case("msa64_f11P7", ["dist", "-i", "msa64.fsa", "-f", "11", "-P", "7"], "msa64_f11P7.out", "dist")
    case(f"{b}_L", ["dist", "-i", "msa64.fsa", "-f", "3", "-L", "2978", "-C", "0"], f"{b}_L.out", "dist")
    case(f"{b}_n", ["dist", "-i", "msa64.fsa", "-f", "3", "-n", "/dev/null"], f"{b}_n.out", "dist")
    case(f"{b}_x3", ["dist", "-i", "msa64.fsa", "-W", "7", "-x", "3"], f"{b}_x3.out", "dist")

    # (iii) trees on an integer SNP matrix (tie-heavy) and a Euclidean one
    msa("msa300.fsa", 300, 2000, seed=5, exclude=0, mut=0.01)
    run(["dist", "-i", "msa300.fsa"], "snp300.phy")
    for m in ("dnj", "nj"):
        case(f"snp300_{m}", ["tree", "-i", "snp300.phy", "-m", m], f"snp300_{m}.out", "tree")
    case("snp300_s", ["tree", "-i", "snp300.phy", "-s"], "snp300_s.out", "tree")
    case("snp300_b", ["tree", "-i", "snp300.phy", "-b"], "snp300_b.out", "tree")
    euclid_phy("euc400.phy.gz", 400, seed=6, gz=True)
    for m in ("dnj", "nj"):
        case(f"euc400_{m}", ["tree", "-i", "euc400.phy.gz", "-m", m], f"euc400_{m}.out", "tree")
    case("euc400_p", ["tree", "-i", "euc400.phy.gz", "-p"], "euc400_p.out", "tree")

    # HNJ (-m hnj, hclust.c:1671): the heuristic NJ on the same inputs
    case("test_hnj", ["tree", "-i", "test.phy.gz", "-m", "hnj"], "test_hnj.out", "tree")
    case("test_hnj_p", ["tree", "-i", "test.phy.gz", "-m", "hnj", "-p"], "test_hnj_p.out", "tree")
    case("test_hnj_f1", ["tree", "-i", "test.phy.gz", "-m", "hnj", "-f", "1"], "test_hnj_f1.out", "tree")
    case("test_hnj_f2", ["tree", "-i", "test.phy.gz", "-m", "hnj", "-f", "2"], "test_hnj_f2.out", "tree")
    case("snp300_hnj", ["tree", "-i", "snp300.phy", "-m", "hnj"], "snp300_hnj.out", "tree")
    case("snp300_hnj_b", ["tree", "-i", "snp300.phy", "-m", "hnj", "-b"], "snp300_hnj_b.out", "tree")
    case("snp300_hnj_s", ["tree", "-i", "snp300.phy", "-m", "hnj", "-s"], "snp300_hnj_s.out", "tree")
    case("euc400_hnj", ["tree", "-i", "euc400.phy.gz", "-m", "hnj"], "euc400_hnj.out", "tree")

    # (iv) missing data: pairwise distances with -1 where the overlap is short
    msa("msa_miss.fsa", 80, 1500, seed=7, nrate=0.12, exclude=0, gaps=False, iupac=False, lower=False)
    run(["dist", "-i", "msa_miss.fsa", "-f", "3", "-L", "1150", "-C", "0"], "miss80.phy")
    for m in ("dnj", "nj"):
        case(f"miss80_{m}", ["tree", "-i", "miss80.phy", "-m", m], f"miss80_{m}.out", "tree")
    case("miss80_p", ["tree", "-i", "miss80.phy", "-p"], "miss80_p.out", "tree")
    case("miss80_hnj", ["tree", "-i", "miss80.phy", "-m", "hnj"], "miss80_hnj.out", "tree")

    # multi-matrix Phylip with a comment header (tree.c:101-104, phy.c:275)
    with open("multi.phy", "w") as f:
        for k, fn in enumerate(("snp300.phy", "miss80.phy")):
            f.write(f"#matrix{k}\n")
            f.write(open(fn).read())
    case("multi_dnj", ["tree", "-i", "multi.phy"], "multi_dnj.out", "tree")
    case("multi_hnj", ["tree", "-i", "multi.phy", "-m", "hnj"], "multi_hnj.out", "tree")

    # (v) KMA count matrices (B1/B2): 9 samples x 2 templates -- insertion rows
    # (s2, s5: stripMat's 7-short stride), a low-depth sample (s3), a missing
    # template (s4), a truncated one (s7: cmpMats' early -1), a plain file (s8)
    rng = random.Random(8)
    t1 = "".join(rng.choice("ACGT") for _ in range(3000))
    t2 = "".join(rng.choice("ACGT") for _ in range(1500))
    kfiles = []
    for k in range(9):
        fn = f"kma{k}.mat" + ("" if k == 8 else ".gz")
        kma_sample(fn, [("tmpl_one", t1), ("tmpl_two", t2)], seed=k + 10, depth=8 if k == 3 else 30,
                   ins=0.01 if k in (2, 5) else 0.0, skip=("tmpl_two",) if k == 4 else (), gz=k != 8,
                   trunc={"tmpl_one": 2900} if k == 7 else None)
        kfiles.append(fn)
    for m in ("cos", "c", "l1", "l2", "linf", "chi2", "nchi2", "nc", "bc", "nbc", "nl1", "nl2", "nlinf", "l3",
              "nl3"):
        case(f"kma_{m}", ["dist", "-i"] + kfiles + ["-r", "tmpl_one", "-d", m], f"kma_{m}.out", "kma")
    case("kma_t2", ["dist", "-i"] + kfiles + ["-r", "tmpl_two"], "kma_t2.out", "kma")
    case("kma_t2_c", ["dist", "-i"] + kfiles + ["-r", "tmpl_two", "-d", "c"], "kma_t2_c.out", "kma")
    case("kma_W", ["dist", "-i"] + kfiles + ["-r", "tmpl_one", "-W", "1000"], "kma_W.out", "kma")
    case("kma_p", ["dist", "-i"] + kfiles + ["-r", "tmpl_one", "-p"], "kma_p.out", "kma")
    case("kma_s", ["dist", "-i"] + kfiles + ["-r", "tmpl_one", "-s", "100"], "kma_s.out", "kma")
    case("kma_b", ["dist", "-i"] + kfiles + ["-r", "tmpl_one", "-b", "0.5"], "kma_b.out", "kma")
    case("kma_E5", ["dist", "-i"] + kfiles + ["-r", "tmpl_one", "-E", "5"], "kma_E5.out", "kma")
    case("kma_CL", ["dist", "-i"] + kfiles + ["-r", "tmpl_two", "-C", "10", "-L", "100"], "kma_CL.out", "kma")
    case("kma_n", ["dist", "-i"] + kfiles + ["-r", "tmpl_one", "-n", "-", "-d", "l1"], "kma_n.out", "kma")
    case("kma_f5", ["dist", "-i"] + kfiles + ["-r", "tmpl_one", "-f", "5", "-x", "4"], "kma_f5.out", "kma")

    # (vi) multi-file FASTA with -r (cdist.c:36 ltdFsaMatrix_get): one file
    # per sample holding two template entries; ff3 lacks "gene_b", ff5's
    # gene_b is mostly N (excluded), so cmpFsaThrd's `&&` pair order shows
    rng = random.Random(9)
    ga = [rng.choice("ACGT") for _ in range(2500)]
    gb = [rng.choice("ACGT") for _ in range(1337)]
    ffiles = []
    for k in range(7):
        fn = f"ff{k}.fsa"
        with open(fn, "w") as f:
            for name, base in (("gene_a", ga), ("gene_b", gb)):
                if name == "gene_b" and k == 3:
                    continue
                s_ = list(base)
                for p_ in range(len(s_)):
                    r_ = rng.random()
                    if r_ < 0.02:
                        s_[p_] = rng.choice("ACGT")
                    elif r_ < 0.025:
                        s_[p_] = "N"
                    elif (name == "gene_b" and k == 5) and r_ < 0.7:
                        s_[p_] = "N"
                f.write(f">{name}\n")
                txt = "".join(s_)
                for q in range(0, len(txt), 60):
                    f.write(txt[q:q + 60] + "\n")
        ffiles.append(fn)
    case("ff_a", ["dist", "-i"] + ffiles + ["-r", "gene_a"], "ff_a.out", "fsafiles")
    case("ff_b", ["dist", "-i"] + ffiles + ["-r", "gene_b"], "ff_b.out", "fsafiles")
    case("ff_b_W", ["dist", "-i"] + ffiles + ["-r", "gene_b", "-W", "1000", "-f", "5"], "ff_b_W.out", "fsafiles")
    case("ff_b_f3", ["dist", "-i"] + ffiles + ["-r", "gene_b", "-f", "3", "-n", "-"], "ff_b_f3.out", "fsafiles")
    case("ff_a_f3s", ["dist", "-i"] + ffiles + ["-r", "gene_a", "-f", "3", "-s", "10"], "ff_a_f3s.out", "fsafiles")
    case("ff_b_f3P", ["dist", "-i"] + ffiles + ["-r", "gene_b", "-f", "3", "-P", "6"], "ff_b_f3P.out", "fsafiles")

    with open("golden.json", "w") as f:
        json.dump({"reference": "ccphylo 0.8.5 (oracle/_ref/ccphylo, built by oracle/Makefile)",
                   "cases": cases}, f, indent=1)
    print(f"{len(cases)} golden cases")


if __name__ == "__main__":
    main()
