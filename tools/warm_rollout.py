#!/usr/bin/env python3
"""Closed-loop rollout at config C (65,536 = 4,096 states x 16 gait candidates, K ticks of
solve_gait -> select_state -> plant on one context): mean dual passes per instance and the
gait-solve kernel time per tick, cold vs warm-started (mpcqp_set_warm_start).  GPU box.
Usage: python tools/warm_rollout.py [--config C] [--states 4096] [--ticks 20]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))


def run(p, g, K, warm):
    import torch
    from mpcqp.engine import BatchEngine
    eng = BatchEngine(p)
    eng.set_warm_start(warm)
    dg = eng.upload_gait(g)
    eng.reserve(dg["B"])
    it, ms = [], []
    stream = torch.cuda.current_stream()
    for _ in range(K):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        eng.solve_gait(dg)
        e1.record(stream)
        eng.select_state(dg)
        eng.plant(dg)
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
        it.append(float(dg["iters"].float().mean().item()))
    eng.close()
    return np.array(it), np.array(ms)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C")
    ap.add_argument("--states", type=int, default=4096)
    ap.add_argument("--ticks", type=int, default=20)
    a = ap.parse_args()
    import mpcqp
    p = mpcqp.model_params(a.config)
    g = mpcqp.make_gait_states(p, a.states, seed=11, candidates=16)
    ic, mc = run(p, g, a.ticks, False)
    iw, mw = run(p, g, a.ticks, True)
    print(f"config {a.config}, {a.states} states x 16 candidates, {a.ticks} ticks")
    print("tick  cold_iters  warm_iters  cold_ms  warm_ms")
    for k in range(a.ticks):
        print(f"{k:4d}  {ic[k]:10.3f}  {iw[k]:10.3f}  {mc[k]:7.3f}  {mw[k]:7.3f}")
    print(f"ticks 1..: mean iters cold {ic[1:].mean():.3f} warm {iw[1:].mean():.3f} "
          f"({100 * (1 - iw[1:].mean() / ic[1:].mean()):.1f}% fewer); kernel ms cold "
          f"{mc[1:].mean():.3f} warm {mw[1:].mean():.3f}")


if __name__ == "__main__":
    main()
