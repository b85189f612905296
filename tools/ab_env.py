#!/usr/bin/env python3
"""Alternating A/B of one library under two environment settings read at context creation
(e.g. MPCQP_CRASH_P=0 vs the default): both contexts live in one process, launches alternate
in rounds, each kernel timed by the library's own HIP events (slot 2: the one-wave kernel).
Usage:  python tools/ab_env.py --env MPCQP_CRASH_P=0 --env MPCQP_CRASH_P= [--batches 512,4096]
(an empty value unsets the variable)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))
import numpy as np  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--env", action="append", required=True)
ap.add_argument("--config", default="B")
ap.add_argument("--gait", default="alternating")
ap.add_argument("--batches", default="512,4096,8192,65536")
ap.add_argument("--rounds", type=int, default=8)
ap.add_argument("--per", type=int, default=16)
ap.add_argument("--slot", type=int, default=2,
                help="library timing slot: 2 the one-wave kernel, 3 the workgroup kernel, 1 the "
                     "whole solve call (dense contexts: 1)")
args = ap.parse_args()
import mpcqp  # noqa: E402
from mpcqp.engine import BatchEngine  # noqa: E402

p = mpcqp.model_params(args.config)
for B in [int(b) for b in args.batches.split(",")]:
    batch = mpcqp.make_batch(p, B, gait=args.gait)
    engs = []
    for spec in args.env:
        k, v = spec.split("=", 1)
        if v:
            os.environ[k] = v
        else:
            os.environ.pop(k, None)
        e = BatchEngine(p)
        engs.append((spec, e, e.upload(batch)))
    for _, e, d in engs:
        e.enable_timing(True)
        for _ in range(40):
            e.solve(d)
        e.sync()
        e.kernel_ms_sum(args.slot)
    res = {spec: [] for spec, _, _ in engs}
    for _ in range(args.rounds):
        for spec, e, d in engs:
            for _ in range(args.per):
                e.solve(d)
            e.sync()
            ms, n = e.kernel_ms_sum(args.slot)
            res[spec].append(ms / max(1, n))
    line = [f"{args.config}@{B} ({args.gait})"]
    for spec, e, d in engs:
        it = d["iters"].cpu().numpy()
        r = np.array(res[spec])
        line.append(f"[{spec or 'default'}] {np.median(r) * 1e3:8.1f} us (spread "
                    f"{(r.max() - r.min()) / np.median(r) * 100:4.1f} %) iters mean "
                    f"{it.mean():.2f} max {it.max()}")
        e.close()
    print("  ".join(line), flush=True)
