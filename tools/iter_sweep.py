#!/usr/bin/env python3
"""k_mpc time vs the solver's iteration cap (config B): the slope is the cost of one dual-loop
pass at full occupancy.  Usage: python tools/iter_sweep.py [--batch 65536] [--caps 1,2,3,5,10,100]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))
import numpy as np  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="B")
ap.add_argument("--batch", type=int, default=65536)
ap.add_argument("--caps", default="1,2,3,4,6,10,100")
ap.add_argument("--reps", type=int, default=10)
args = ap.parse_args()
import mpcqp  # noqa: E402
from mpcqp.engine import BatchEngine  # noqa: E402

for cap in [int(c) for c in args.caps.split(",")]:
    p = mpcqp.model_params(args.config)
    p["max_iter"] = cap
    eng = BatchEngine(p)
    d = eng.upload(mpcqp.make_batch(p, args.batch))
    eng.enable_timing(True)
    ts = []
    for r in range(args.reps + 2):
        eng.solve(d)
        eng.sync()
        if r >= 2:
            ts.append(eng.last_kernel_ms(1))
    it = d["iters"].cpu().numpy().reshape(-1, 2)
    print(f"cap {cap:4d}: {np.median(ts):.4f} ms  mean iters {it.mean():.3f}  "
          f"mean pair max {it.max(1).mean():.3f}", flush=True)
    eng.close()
