#!/usr/bin/env python3
"""Median k_mpc time over repeated launches for a config (library from $MPCQP_LIB)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))
import numpy as np  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--configs", default="B,C,L")
ap.add_argument("--batch", type=int, default=65536)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--gait", default="alternating")
ap.add_argument("--max-free", type=int, default=None)
ap.add_argument("--b2b", action="store_true",
                help="launches back to back (no sync between them, as bench.py's steps), the "
                     "one-wave kernel's mean by the library's events (slot 2) after 50 warm-up calls")
args = ap.parse_args()
import mpcqp  # noqa: E402
from mpcqp.engine import BatchEngine  # noqa: E402
print("lib", os.environ.get("MPCQP_LIB", "default"))
for cfg in args.configs.split(","):
    p = mpcqp.model_params(cfg)
    if args.max_free is not None:
        p["max_free"] = args.max_free
    eng = BatchEngine(p)
    d = eng.upload(mpcqp.make_batch(p, args.batch, gait=args.gait))
    if args.b2b:
        for _ in range(50):
            eng.solve(d)
        eng.sync()
        eng.enable_timing(True)
        for _ in range(args.reps):
            eng.solve(d)
        eng.sync()
        ms, n = eng.kernel_ms_sum(2)
        st = d["status"].cpu().numpy()
        print(f"  {cfg}: {ms / n:.4f} ms  ({args.batch / (ms / n) / 1e3:.2f} M QP/s)  solved "
              f"{np.mean(st == 0):.4f}  (back to back, {n} launches)")
        eng.close()
        continue
    eng.enable_timing(True)
    ts = []
    for r in range(args.reps + 3):
        eng.solve(d)
        eng.sync()
        if r >= 3:
            ts.append(eng.last_kernel_ms(1))
    st = d["status"].cpu().numpy()
    print(f"  {cfg}: {np.median(ts):.4f} ms  ({args.batch / np.median(ts) / 1e3:.2f} M QP/s)  "
          f"solved {np.mean(st == 0):.4f}")
    eng.close()
