#!/usr/bin/env python3
"""Run the batched solve a few times (profiling driver for tools/phase_pmc.sh)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="B")
ap.add_argument("--batch", type=int, default=65536)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--max-iter", type=int, default=0, help="solver iteration cap (0 = default)")
ap.add_argument("--max-free", type=int, default=None, help="max_free (30: no overflow launch)")
args = ap.parse_args()
import mpcqp  # noqa: E402
from mpcqp.engine import BatchEngine  # noqa: E402
p = mpcqp.model_params(args.config)
p["max_iter"] = args.max_iter
if args.max_free is not None:
    p["max_free"] = args.max_free
eng = BatchEngine(p)
d = eng.upload(mpcqp.make_batch(p, args.batch))
for _ in range(args.reps):
    eng.solve(d)
eng.sync()
eng.close()
