#!/usr/bin/env python3
"""Config C friction QPs (oracle H, f, bounds, pyramid rows over the free forces): does the
primal-dual active-set iteration of gi_crash_reg.hpp converge from the optimum's own active set
(|slack| < 1e-8) and from the empty set?  Dependent rows (pivot below 1e-12 of the diagonal) are
skipped.  CPU only (the checker library).  Usage: python tools/crash_sim_friction.py"""
import sys, numpy as np
import os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, 'mpc-limx-control_amd')); sys.path.insert(0, os.path.join(R, 'oracle'))
import mpcqp, oracle as orc
p = mpcqp.model_params("C")
B = 256
b = mpcqp.make_batch(p, B, seed=3)
ref = orc.srbm_batch(p, b["x0"], b["xref"], b["lin"], b["contact"], want_hf=True)
NU, N, mu = p["nu"], p["N"], p["mu"]
nV = NU * N
def qp(i):
    H = ref["H"][i]; f = ref["f"][i]; ct = int(b["contact"][i])
    lb, ub = orc.srbm_bounds(p, ct)
    free = np.where(lb != ub)[0]
    # constraints over free vars: list of (normal over free idx, b)
    pos = {v: j for j, v in enumerate(free)}
    cons = []
    for j, v in enumerate(free):
        isfz = (v % NU) % 3 == 2
        if not (isfz and mu > 0 and lb[v] <= 0):  # elided fz lower bound
            if lb[v] > -1e19: n = np.zeros(len(free)); n[j] = 1; cons.append((n, lb[v], ('lo', v)))
        if ub[v] < 1e19: n = np.zeros(len(free)); n[j] = -1; cons.append((n, -ub[v], ('hi', v)))
    for k in range(N):
        for s in range(2):
            if (ct >> (2 * k + s)) & 1:
                vz = k * NU + 3 * s + 2
                for t in range(4):
                    vt = vz - 2 + (t >> 1); sg = 1.0 if t & 1 else -1.0
                    n = np.zeros(len(free)); n[pos[vz]] = mu; n[pos[vt]] = sg
                    cons.append((n, 0.0, ('row', vz, t)))
    Hf = H[np.ix_(free, free)]; gf = f[free] + H[np.ix_(free, np.setdiff1d(np.arange(nV), free))] @ np.zeros(nV - len(free))
    return Hf, f[free], cons, free
def crash(Hf, g, cons, seed, P=6, K=16, tol=1e-11):
    x0 = -np.linalg.solve(Hf, g)
    Hi = np.linalg.inv(Hf)
    sel = set(); neg = set(); xc = x0
    for it in range(100):
        nsel = set()
        for a, (n, bb, _) in enumerate(cons):
            s = n @ xc - bb
            if a in sel:
                if a not in neg: nsel.add(a)
            elif s < -tol * (1 + abs(bb)) or (it == 0 and a in seed): nsel.add(a)
        if nsel == sel: return True, it, xc
        if it >= P: return False, it, None
        sel = nsel
        A = sorted(sel)
        if len(A) > K: return False, it, None
        if not A: xc = x0; neg = set(); continue
        Nm = np.array([cons[a][0] for a in A]).T
        bv = np.array([cons[a][1] for a in A])
        M = Nm.T @ Hi @ Nm
        r = Nm.T @ x0 - bv
        # Gauss-Jordan without pivoting; a pivot below 1e-12 of its original diagonal = a row
        # dependent on the earlier ones: skipped (its w = 0)
        Mw = M.copy(); rw = r.copy(); k = len(A); skip = np.zeros(k, bool)
        for j in range(k):
            piv = Mw[j, j]
            if not (piv > 1e-12 * M[j, j]): skip[j] = True; continue
            for rr_ in range(k):
                if rr_ != j:
                    l = Mw[rr_, j] / piv
                    Mw[rr_] -= l * Mw[j]; rw[rr_] -= l * rw[j]
        w = np.where(skip, 0.0, rw / np.where(skip, 1.0, np.diag(Mw)))
        xc = x0 - Hi @ Nm @ w
        neg = set(a for a, wa in zip(A, w) if wa > 0)
    return False, 100, None
ok = 0; its = []; okc = 0
for i in range(B):
    Hf, g, cons, free = qp(i)
    x = ref["U"][i][free]
    act = set(a for a, (n, bb, _) in enumerate(cons) if abs(n @ x - bb) < 1e-8)
    s, it, xc = crash(Hf, g, cons, act)
    if s:
        ok += 1; its.append(it)
        assert np.abs(xc - x).max() < 1e-6 * max(1, np.abs(x).max()), (i, np.abs(xc - x).max())
    s2, it2, _ = crash(Hf, g, cons, set())
    okc += s2
print(f"perfect seed: {ok}/{B} converge, sets {np.bincount(its)}; cold: {okc}/{B}")
