#!/usr/bin/env python3
"""Randomised parity sweep on the GPU box: tests/test_gpu_fuzz.py's parameter draws for many more
seeds than the committed test runs (config B / C / L; mass, inertia, friction, force bounds, Ts,
weights, odd batch sizes, every gait), each against the oracle at the test's tolerances.
Prints one line per failing draw and a summary.
--dense N adds N draws of the dense config E (test_fuzz_dense_vs_oracle's draws, seeds 6..).
Usage:  python tools/fuzz_sweep.py [--first 24] [--count 200] [--dense 0]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--first", type=int, default=24)
ap.add_argument("--count", type=int, default=200)
ap.add_argument("--dense", type=int, default=0)
args = ap.parse_args()
import oracle  # noqa: E402
from mpcqp.engine import BatchEngine  # noqa: E402
from test_gpu_fuzz import TOL_U, _draw, _draw_dense  # noqa: E402

def draws():
    for seed in range(args.first, args.first + args.count):
        p, batch, gait = _draw(seed)
        yield seed, p, batch, gait, False
    for seed in range(6, 6 + args.dense):
        p, batch = _draw_dense(seed)
        yield seed, p, batch, "dense", True


bad = n = 0
for seed, p, batch, gait, dense in draws():
    n += 1
    eng = BatchEngine(p)
    crash = eng.crash
    d = eng.upload(batch)
    eng.solve(d)
    eng.sync()
    o = {k: d[k].cpu().numpy() for k in ("U", "cost", "status", "iters")}
    eng.close()
    q = dict(p)
    q["crash"] = tuple(crash)
    ref = (oracle.dense_batch(q, batch["x0"], batch["xref"], batch["lin"]) if dense else
           oracle.srbm_batch(q, batch["x0"], batch["xref"], batch["lin"], batch["contact"], nthreads=8))
    ok = ref["status"] == 0
    msgs = []
    if not np.array_equal(o["status"], ref["status"]):
        msgs.append(f"status differs on {int((o['status'] != ref['status']).sum())}")
    scale = np.maximum(1.0, np.abs(ref["U"]).max(axis=1))
    du = np.abs(o["U"] - ref["U"]).max(axis=1) / scale
    if np.any(du[ok] > TOL_U):
        msgs.append(f"U off on {int((du[ok] > TOL_U).sum())} (max {du[ok].max():.2e})")
    if ok.any() and not np.allclose(o["cost"][ok], ref["cost"][ok], rtol=1e-9, atol=1e-9):
        msgs.append("cost off")
    im = float(np.mean(o["iters"][ok] == ref["iters"][ok])) if ok.any() else 1.0
    if im < 0.95:
        msgs.append(f"iterations equal on {im:.3f}")
    if msgs:
        bad += 1
        print(f"seed {seed} {p['config']} {gait} B={batch['x0'].shape[0]} mu={p['mu']:.3f} "
              f"fz_min={p['fz_min']:.2f}: " + "; ".join(msgs), flush=True)
print(f"{n - bad} / {n} draws match the oracle")
