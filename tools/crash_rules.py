#!/usr/bin/env python3
"""Crash-start working-set rules on the CPU (config B): the paired kernel's rule (every violated
bound in, negative multipliers out, at most 12 with kept bounds first) against variants that add
only part of the violated bounds -- the most violated ones of the first set or of every set, or at
most a few per set.  Replays the rule in numpy on the oracle's own H_FF / g (J = L^-T, x0 the
unconstrained minimum); the plain rule's set counts must equal the oracle's iteration counts.
Usage:  python tools/crash_rules.py [batch]   (CPU only; DESIGN.md section 4, crash start)"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'mpc-limx-control_amd'))
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
import mpcqp, oracle
TOL = 1e-11
p = mpcqp.model_params("B")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
batch = mpcqp.make_batch(p, B, seed=5)
pc = dict(p); pc["crash"] = (12, 8)
o = oracle.srbm_batch(pc, batch["x0"], batch["xref"], batch["lin"], batch["contact"], want_hf=True, nthreads=8)
probs = []
for i in range(B):
    lb, ub = oracle.srbm_bounds(p, int(batch["contact"][i]))
    F = np.flatnonzero(lb != ub)
    H = o["H"][i][np.ix_(F, F)]; g = o["f"][i][F]
    L = np.linalg.cholesky(H); J = np.linalg.inv(L).T
    x0 = -J @ (J.T @ g)
    probs.append((J, x0, lb[F], ub[F]))

ADD_ONLY = [0, 0, 0, 0]  # later sets that only append, all later sets, their rows, all rows


def crash(J, x0, lo, hi, rule, kmax=12, pmax=8):
    n = len(x0); side = np.zeros(n, int); lam = np.zeros(n); xc = x0.copy()
    sets = []
    it = 0
    while True:
        nw = side.copy()
        viol = np.zeros(n)
        for j in range(n):
            if side[j] == 0:
                if xc[j] - lo[j] < -TOL * (1 + abs(lo[j])): nw[j] = 1; viol[j] = lo[j] - xc[j]
                elif -xc[j] + hi[j] < -TOL * (1 + abs(hi[j])): nw[j] = -1; viol[j] = xc[j] - hi[j]
            elif lam[j] < 0: nw[j] = 0
        if (nw == side).all(): return sets, True
        if it >= pmax: return sets, False
        new = np.flatnonzero((side == 0) & (nw != 0))
        if rule[0] == "frac" and len(new):
            vmax = viol[new].max()
            for j in new:
                if viol[j] < rule[1] * vmax: nw[j] = 0
        if rule[0] == "cap" and len(new) > rule[1]:
            order = new[np.argsort(-viol[new], kind="stable")]
            for j in order[rule[1]:]: nw[j] = 0
        if rule[0] == "capid" and len(new) > rule[1]:
            for j in new[rule[1]:]: nw[j] = 0
        if rule[0] == "first" and it == 0 and len(new):
            vmax = viol[new].max()
            for j in new:
                if viol[j] < rule[1] * vmax: nw[j] = 0
        cnt = (nw != 0).sum()
        if cnt > kmax:
            kept = ((side != 0) & (nw != 0)).sum(); room = kmax - kept
            for j in range(n):
                if side[j] == 0 and nw[j] != 0:
                    if room > 0: room -= 1
                    else: nw[j] = 0
        if rule == ("none",) and it > 0 and (side != 0).any():
            drops = ((side != 0) & (nw == 0)).any()
            ADD_ONLY[0] += not drops
            ADD_ONLY[1] += 1
            ADD_ONLY[2] += (nw != 0).sum() if not drops else 0
        if rule == ("none",):
            ADD_ONLY[3] += (nw != 0).sum()
        side = nw; it += 1
        A = np.flatnonzero(side)
        if len(A) == 0: xc = x0.copy(); lam[:] = 0; continue
        sets.append(len(A))
        b = np.where(side[A] > 0, lo[A], hi[A])
        JA = J[A]; M = JA @ JA.T
        w = np.linalg.solve(M, x0[A] - b)
        xc = x0 - J @ (JA.T @ w); xc[A] = b
        lam[:] = 0; lam[A] = -side[A] * w

rules = [("none",), ("first", 0.5), ("first", 0.25), ("frac", 0.5), ("frac", 0.25), ("cap", 4), ("cap", 6),
         ("cap", 8), ("capid", 6), ("capid", 8)]

t0=time.time()
res = {}
for rule in rules:
    nsets = []; ksum = []; fails = 0
    for (J, x0, lo, hi) in probs:
        sets, ok = crash(J, x0, lo, hi, rule)
        fails += not ok
        nsets.append(len(sets)); ksum.append(sum(sets))
    nsets = np.array(nsets); ksum = np.array(ksum)
    pairmax = np.maximum(nsets[0::2], nsets[1::2])
    pairk = np.maximum(ksum[0::2], ksum[1::2])
    print(f"{str(rule):16s} sets mean {nsets.mean():.3f} max {nsets.max()}  pair-max mean {pairmax.mean():.3f}  sum-k mean {ksum.mean():.2f} pair-max-k mean {pairk.mean():.2f} max {pairk.max()}  give-ups {fails}")
    if rule == ("none",):
        it = o["iters"]
        print("   oracle iters == sets:", np.mean(it == nsets))
print(f"kept rule: {ADD_ONLY[0]} of {ADD_ONLY[1]} later sets only append bounds; their rows "
      f"are {ADD_ONLY[2]} of the {ADD_ONLY[3]} rows solved")
print("%.1fs" % (time.time()-t0))
