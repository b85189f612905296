#!/usr/bin/env python3
"""Warm-start A/B for the Goldfarb-Idnani dual solver,
on the CPU oracle (the same algorithm, constraint order and tolerances as the GPU kernels).

A dual active-set solve adds one constraint per pass and drops one per pass, so a cold solve
that ends with the active set A takes  iters = |A| + 2 * drops  passes (every dropped
constraint was added once before).  The best a warm start can do -- hot-starting from the
previous tick's active set when it equals this tick's -- is |A| passes (each constraint of A
re-added once; J, R have to be rebuilt for this tick's H), so its saving is bounded by
2 * drops / iters.  This tool measures |A| (bounds at a bound, friction rows at equality) and the
drops of every instance of a seeded batch, cold, and reports that bound.
Usage: python tools/warm_start_ab.py [--config C] [--batch 4096] [--gait alternating]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def active_count(p, U, contact, tol=1e-9):
    import oracle
    lb, ub = oracle.srbm_bounds(p, int(contact))
    free = lb < ub
    n = int(np.sum(free & ((np.abs(U - lb) <= tol * (1 + np.abs(lb))) |
                           (np.abs(U - ub) <= tol * (1 + np.abs(ub))))))
    if p["constraints"]:
        nu, N = p["nu"], p["N"]
        for k in range(N):
            for s in range(2):
                if not (int(contact) >> (2 * k + s)) & 1:
                    continue
                b = k * nu + 3 * s
                fz = U[b + 2]
                for t in range(2):
                    for sg in (-1.0, 1.0):
                        if abs(p["mu"] * fz + sg * U[b + t]) <= tol * (1 + abs(fz)):
                            n += 1
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--gait", default="alternating")
    a = ap.parse_args()
    import mpcqp
    import oracle
    p = mpcqp.model_params(a.config)
    b = mpcqp.make_batch(p, a.batch, gait=a.gait)
    ref = oracle.srbm_batch(p, b["x0"], b["xref"], b["lin"], b["contact"])
    ok = ref["status"] == 0
    A = np.array([active_count(p, ref["U"][i], b["contact"][i]) for i in range(a.batch)])
    it = ref["iters"].astype(float)
    drops = (it - A) / 2.0
    print(f"config {a.config} gait {a.gait} batch {a.batch}: solved {ok.mean():.4f}")
    print(f"  mean passes (cold) {it[ok].mean():.3f}; mean |A| {A[ok].mean():.3f}; "
          f"mean drops {drops[ok].mean():.3f}; instances with a drop {np.mean(drops[ok] > 0):.3f}")
    print(f"  perfect warm start: {A[ok].mean():.3f} passes -> saves at most "
          f"{100 * (1 - A[ok].sum() / it[ok].sum()):.1f}% of the dual-loop passes")
    bad = np.abs(drops - np.round(drops)) > 1e-9
    if bad.any():
        print(f"  note: {bad.sum()} instances with a non-integer drop count (degenerate actives)")


if __name__ == "__main__":
    main()
