#!/usr/bin/env python3
"""A few config-B steps at one batch size, separate then fused selection, for a kernel trace
(rocprofv3 --kernel-trace): the per-step kernel chain and the gaps between its launches.
  rocprofv3 --kernel-trace -d DIR -o run -- python tools/step_trace.py --batch 4096
  python tools/step_trace.py --analyze DIR/.../run_kernel_trace.csv"""
import argparse
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))


def analyze(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    prev_end = None
    for r in rows[-24:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"]
        name = name[name.find("k_"):name.find("(")] if "k_" in name else name[:40]
        gap = (s - prev_end) / 1e3 if prev_end else 0.0
        print(f"  {name[:48]:48s} grid {r['Grid_Size_X']:>8s} dur {(e - s) / 1e3:8.1f} us  gap {gap:7.1f} us")
        prev_end = e


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--analyze", default=None)
    a = ap.parse_args()
    if a.analyze:
        return analyze(a.analyze)
    import torch
    import mpcqp
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params("B")
    eng = BatchEngine(p)
    d = eng.upload(mpcqp.make_batch(p, a.batch, seed=20250404))
    rec = torch.zeros(1 + eng.nV, dtype=torch.int64, device="cuda")
    for _ in range(a.steps):
        eng.solve(d)
        eng.select_record(d, rec)
    eng.sync()
    for _ in range(a.steps):
        eng.solve_select(d, rec)
    eng.sync()
    eng.close()


if __name__ == "__main__":
    main()
