#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-pointer path (mpcqp_batch_solve_host) at config B: pageable
arrays through the pinned staging vs page-locked caller arrays (mpcqp_host_register, the direct
chunked path), the same call bench.py reports as config.pcie_inclusive_qps(_pageable).
Usage: python tools/host_rate.py [--batches 16384,65536] [--reps 5]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--batches", default="16384,65536")
ap.add_argument("--reps", type=int, default=5)
args = ap.parse_args()
import mpcqp  # noqa: E402
from mpcqp.engine import BatchEngine  # noqa: E402

from bench import host_staged_rate  # noqa: E402

p = mpcqp.model_params("B")
for B in [int(b) for b in args.batches.split(",")]:
    batch = mpcqp.make_batch(p, B)
    eng = BatchEngine(p)
    for _ in range(2):
        lk = host_staged_rate(eng, batch, p, reps=args.reps, locked=True)
        pg = host_staged_rate(eng, batch, p, reps=args.reps)
        print(f"B {B:6d}: page-locked {lk / 1e6:7.2f} M QP/s   pageable {pg / 1e6:7.2f} M QP/s",
              flush=True)
    eng.close()
