#!/usr/bin/env python3
"""Per-step GPU time of the headline solve right after a short warm-up (the driver's 5): HIP
events around each of the first K steps after the warm-up's synchronize, and the host time of
each call -- where a short timed region's fixed offset comes from.
Usage: python tools/step_profile.py [--steps 20] [--warmup 5] [--batch 65536]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mpcqp  # noqa: E402
from mpcqp.engine import BatchEngine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--batch", type=int, default=65536)
ap.add_argument("--preheat", default="", help="before the profiled engine: 'same-kernel' (the "
                "headline on another engine and batch) or a config name (C, E), for ~1 s")
args = ap.parse_args()
p = mpcqp.model_params("B")
if args.preheat:
    cfg = "B" if args.preheat == "same-kernel" else args.preheat
    pp = mpcqp.model_params(cfg)
    e2 = BatchEngine(pp)
    d2 = e2.upload(mpcqp.make_batch(pp, 65536 if cfg != "E" else 16384, seed=99))
    t1 = time.perf_counter()
    while time.perf_counter() - t1 < 1.0:
        e2.solve(d2)
        e2.sync()
    e2.close()
eng = BatchEngine(p)
d = eng.upload(mpcqp.make_batch(p, args.batch))
rec = torch.zeros(1 + p["nu"] * p["N"], dtype=torch.int64, device="cuda")
for _ in range(args.warmup):
    eng.solve_select(d, rec, index_base=0)
torch.cuda.synchronize()
s = torch.cuda.current_stream()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
host = []
t0 = time.perf_counter()
ev[0].record(s)
for i in range(args.steps):
    h0 = time.perf_counter()
    eng.solve_select(d, rec, index_base=0)
    ev[i + 1].record(s)
    host.append((time.perf_counter() - h0) * 1e6)
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) * 1e3
gpu = [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(args.steps)]
print("gpu us per step:", " ".join(f"{g:.0f}" for g in gpu))
print("host us per call:", " ".join(f"{h:.0f}" for h in host))
print(f"wall {wall:.3f} ms for {args.steps} steps = {wall / args.steps:.4f} ms/step; "
      f"gpu sum {sum(gpu) / 1e3:.3f} ms")
eng.close()
