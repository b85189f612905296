#!/usr/bin/env python3
"""Where the headline kernel's first-launch slowdown comes from (the driver times 20 steps after
5 warm-up; the first ~60 launches of a process run 295 -> 262 us): per-launch k_mpc_pair times
(the library's HIP events, back to back) for
  fresh : the first launches of the process
  idle  : after 50 ms with the GPU idle
  busy  : right after ~300 ms of another kernel (config E) keeping the GPU busy
  newbuf: a fresh engine + upload of new buffers (same data), right after the headline ran
  python tools/ramp_probe.py [--n 80]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))
import numpy as np  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=60)
args = ap.parse_args()
import torch  # noqa: E402
import mpcqp  # noqa: E402
from mpcqp.engine import BatchEngine  # noqa: E402


def launches(eng, d, n):
    eng.enable_timing(True)
    out = []
    for i in range(n):
        eng.solve(d)
        if (i + 1) % 32 == 0 or i + 1 == n:  # (the library's event ring holds 64)
            eng.sync()
            ms, k = eng.kernel_ms_sum(2)
            out.append((k, ms))
            eng.enable_timing(False)
            eng.enable_timing(True)
    eng.enable_timing(False)
    return out


def per_launch(eng, d, n):
    """n launches, each timed on its own (library events), back to back in groups of 8"""
    ts = []
    for g in range(0, n, 8):
        eng.enable_timing(True)
        for _ in range(min(8, n - g)):
            eng.solve(d)
        eng.sync()
        ms, k = eng.kernel_ms_sum(2)
        ts.append(ms / k * 1e3)
        eng.enable_timing(False)
    return ts


p = mpcqp.model_params("B")
batch = mpcqp.make_batch(p, 65536, seed=20250404)
eng = BatchEngine(p)
d = eng.upload(batch)
torch.cuda.synchronize()
print("fresh  (us per launch, groups of 8):", [round(x, 1) for x in per_launch(eng, d, args.n)], flush=True)
time.sleep(0.05)
print("idle   (after 50 ms idle):          ", [round(x, 1) for x in per_launch(eng, d, args.n)], flush=True)
pe = mpcqp.model_params("E")
be = mpcqp.make_batch(pe, 16384, seed=1)
ee = BatchEngine(pe)
de = ee.upload(be)
for _ in range(3):
    ee.solve(de)
torch.cuda.synchronize()
time.sleep(0.05)
for _ in range(64):
    ee.solve(de)
print("busy   (right after ~300 ms of E):  ", [round(x, 1) for x in per_launch(eng, d, args.n)], flush=True)
eng2 = BatchEngine(p)
d2 = eng2.upload(batch)
torch.cuda.synchronize()
for _ in range(16):
    eng.solve(d)
print("newbuf (fresh engine, new buffers): ", [round(x, 1) for x in per_launch(eng2, d2, args.n)], flush=True)
