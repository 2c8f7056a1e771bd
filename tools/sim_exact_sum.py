"""CPU model of the exact-mode row sum (ccg_tree_common.h exact_sum_w), used
to validate the algorithm before the HIP version: the reference's serial sum
s_k = fl(s_{k-1} + c_k) (nj.c:911) of non-negative c_k, computed as exact
integer sums of per-element increments RN_u(c_k) inside runs where s keeps
one binade [2^e, 2^(e+1)) (u = 2^(e-52)), with the real add only at the
elements where the binade changes, and half-ulp ties resolved from the
parity of the running total.  Chunks play the role of the GPU's lanes /
waves.  Compares against Python's serial float sum on random, %.9f-like,
dyadic (tie-heavy) and wide-range inputs.

    python tools/sim_exact_sum.py
"""
# Simulation of the binade-segmented exact serial sum (validation before the HIP version)
import math, random, sys
import numpy as np

def binade(x):  # exponent e with 2^e <= x < 2^(e+1); None for 0
    if x == 0: return None
    m, e = math.frexp(x)  # x = m*2^e, 0.5<=m<1
    return e - 1

def serial(c):
    s = 0.0
    for x in c: s += x
    return s

def par_sum(c, NT=16):
    n = len(c)
    E = (n + NT - 1) // NT
    for x in c:
        if not (x >= 0 and x < math.inf): return None
    # pass 1: thread sums, exclusive scan (approximate)
    ts = [sum(c[t*E:min(n,(t+1)*E)]) for t in range(NT)]  # any order ok (approx)
    pbase = [0.0]*NT
    acc = 0.0
    for t in range(NT): pbase[t] = acc; acc += ts[t]
    crosses = []   # (k, c, e_new) in order
    ties = []      # (k, seg, pi)
    runs = []      # per thread list of (seg, sum, parity)
    # we need global crossing indices: do per-thread pass computing local crossings, then scan
    per_thread = []
    for t in range(NT):
        P = pbase[t]
        loc_cross = []; loc_runs = []; loc_ties = []
        run_sum = 0.0; run_par = 0
        for k in range(t*E, min(n,(t+1)*E)):
            x = c[k]
            ep = binade(P)
            Pn = P + x
            en = binade(Pn)
            if ep != en and x > 0:
                loc_runs.append((run_sum, run_par)); run_sum = 0.0; run_par = 0
                loc_cross.append((k, x, en))
            elif ep is not None:
                y = math.ldexp(x, 52 - ep)
                B = math.floor(y); f = y - B
                if f == 0.5:
                    loc_ties.append((k, len(loc_cross), (run_par + int(B)) & 1))
                    inc = B
                else:
                    inc = B + (1 if f > 0.5 else 0)
                run_sum += inc; run_par = (run_par + int(inc)) & 1
            P = Pn
        loc_runs.append((run_sum, run_par))
        per_thread.append((loc_cross, loc_runs, loc_ties))
    # global crossing numbering
    cb = 0
    nseg_sum = {}
    thread_of_cross = []
    cbases = []
    for t in range(NT):
        loc_cross, loc_runs, loc_ties = per_thread[t]
        cbases.append(cb)
        for r, (rs, rp) in enumerate(loc_runs):
            nseg_sum[cb + r] = nseg_sum.get(cb + r, 0.0) + rs
        for x in loc_cross: crosses.append(x); thread_of_cross.append(t)
        cb += len(loc_cross)
    ncross = cb
    # XOR scan of last-run parity
    X = [0]*(NT+1)
    for t in range(NT): X[t+1] = X[t] ^ per_thread[t][1][-1][1]
    for t in range(NT):
        loc_cross, loc_runs, loc_ties = per_thread[t]
        for (k, lseg, lpar) in loc_ties:
            seg = cbases[t] + lseg
            if lseg > 0:
                pi = lpar
            else:
                # segment started in an earlier thread (the thread holding crossing seg-1), or at 0
                if seg == 0: pi = lpar   # should not happen (zeros)
                else:
                    tc = thread_of_cross[seg - 1]
                    pi = (X[t] ^ X[tc] ^ per_thread[tc][1][-1][1] ^ lpar) & 1 if tc < t else lpar
                    # X[t]^X[tc] = xor of last-run parities of threads tc..t-1 (includes tc)
                    pi = (X[t] ^ X[tc] ^ lpar) & 1
            ties.append((k, seg, pi))
    ties.sort(); STATS["ties"] += len(ties); STATS["cross"] += ncross
    # walker
    S = 0.0; tp = 0
    for s in range(ncross + 1):
        if s > 0:
            e = crosses[s-1][2]
            ue = e - 52
            if ue < -1022: return None
            T0 = math.ldexp(S, -ue)
            assert T0 == math.floor(T0)
            x = int(T0) & 1
            ups = 0
            while tp < len(ties) and ties[tp][1] == s:
                up = (x + ties[tp][2] + ups) & 1; ups += up; tp += 1
            T = T0 + nseg_sum.get(s, 0.0) + ups
            if T >= 2.0**53: return None
            S = math.ldexp(T, ue)
        else:
            if nseg_sum.get(0, 0.0) != 0: return None
        if s < ncross:
            Sn = S + crosses[s][1]
            if binade(Sn) != crosses[s][2]: return None
            S = Sn
    return S

STATS={"ties":0,"cross":0}
random.seed(1)
bad = fb = 0
tests = 0
for trial in range(3000):
    n = random.randint(1, 400)
    kind = trial % 5
    if kind == 0: c = [random.random() for _ in range(n)]
    elif kind == 1: c = [round(random.random()*1e9)/1e9 for _ in range(n)]
    elif kind == 2: c = [random.randint(0, 8) * 0.5**random.randint(0, 60) for _ in range(n)]  # tie heavy
    elif kind == 3: c = [random.choice([0.0, 1e-3, 0.1, 3.0, 1e5]) * (1 + random.random()*2**-40) for _ in range(n)]
    else: c = [random.randint(0, 2**53) * 2.0**random.randint(-80, -30) for _ in range(n)]
    for z in range(random.randint(0, 3)):
        c[random.randrange(n)] = 0.0
    if trial % 7 == 0: c[0] = 0.0; 
    r = par_sum(c, NT=random.choice([1, 2, 4, 16, 64]))
    tests += 1
    if r is None: fb += 1
    elif r != serial(c) or math.copysign(1, r) != math.copysign(1, serial(c)): bad += 1; print("BAD", kind, n, r, serial(c))
print("tests", tests, "bad", bad, "fallback", fb)
print(STATS)
