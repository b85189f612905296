#!/usr/bin/env python3
"""Warm vs cold closed loop (mpcqp_set_warm_start): per-tick iteration totals
(crash working sets + dual passes) of K ticks of solve_gait -> select_state -> plant on one
context, for configs B (paired kernel: the crash seeded) and C (one-QP kernel: the dual loop's
guesses).  Usage: python tools/warm_iters.py [--configs B,C] [--states 64] [--ticks 8]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))
import numpy as np  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--configs", default="B,C")
ap.add_argument("--states", type=int, default=64)
ap.add_argument("--cands", type=int, default=16)
ap.add_argument("--ticks", type=int, default=8)
args = ap.parse_args()
import mpcqp  # noqa: E402
from mpcqp.engine import BatchEngine  # noqa: E402


def run(p, g, warm):
    eng = BatchEngine(p)
    eng.set_warm_start(warm)
    dg = eng.upload_gait(g)
    tot, ms = [], []
    for _ in range(args.ticks):
        eng.enable_timing(True)
        eng.solve_gait(dg)
        eng.select_state(dg)
        eng.sync()
        ms.append(eng.last_kernel_ms(1))
        tot.append(int(dg["iters"].cpu().numpy().sum()))
        eng.plant(dg)
    eng.close()
    return np.array(tot), np.array(ms)


for cfg in args.configs.split(","):
    p = mpcqp.model_params(cfg)
    g = mpcqp.make_gait_states(p, args.states, seed=11, candidates=args.cands)
    w, wm = run(p, g, True)
    c, cm = run(p, g, False)
    print(f"{cfg}: ticks 1-{args.ticks - 1} iterations warm {w[1:].sum()} cold {c[1:].sum()} "
          f"({w[1:].sum() / max(1, c[1:].sum()):.3f}x); tick 0 {w[0]} / {c[0]}; "
          f"solve ms warm {wm[1:].mean():.4f} cold {cm[1:].mean():.4f}", flush=True)
    print(f"   per tick warm {w.tolist()}\n   per tick cold {c.tolist()}", flush=True)
