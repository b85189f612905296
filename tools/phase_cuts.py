#!/usr/bin/env python3
"""Per-phase cost of the fused k_mpc kernel at full occupancy, by early exit.

The diagnostic build lib/libmpcqp_cuts.so (-DMPCQP_CUTS) returns from the kernel after phase
k when MPCQP_CUT=k is set at launch.  The kernel time at cut k minus the time at cut k-1 is
what phase k adds with the whole chip busy (stamps measure one wave's elapsed time, which
includes the other waves' issue).  Never benchmark this build.
Usage:  python tools/phase_cuts.py [--configs B,C,L] [--batch 65536] [--reps 10]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("MPCQP_LIB", os.path.join(ROOT, "mpc-limx-control_amd", "lib",
                                                "libmpcqp_cuts.so"))
sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))

import numpy as np  # noqa: E402

CUTS = [(1, "inputs + model + setup"), (2, "S blocks + u/v"), (3, "H_FF build + row load"),
        (4, "Cholesky"), (5, "J = L^-T (+ t)"), (6, "unconstrained min"),
        (7, "dual loop"), (0, "write (full kernel)")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="B,C,L")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--cuts", default="", help="comma list of extra cut ids to time (e.g. 11,12,13)")
    args = ap.parse_args()
    import mpcqp
    from mpcqp.engine import BatchEngine
    for cfg in args.configs.split(","):
        p = mpcqp.model_params(cfg)
        eng = BatchEngine(p)
        d = eng.upload(mpcqp.make_batch(p, args.batch))
        eng.enable_timing(True)
        prev = 0.0
        print(f"config {cfg}: batch {args.batch}, fast path {eng.fast_path}")
        cuts = CUTS if not args.cuts else [(int(c), f"cut {c}") for c in args.cuts.split(",")]
        for cut, name in cuts:
            os.environ["MPCQP_CUT"] = str(cut)
            ts = []
            for r in range(args.reps + 2):
                eng.solve(d)
                eng.sync()
                if r >= 2:
                    ts.append(eng.last_kernel_ms(1))
            ms = float(np.median(ts))
            print(f"  cut {cut}  {name:24s} {ms:8.4f} ms   +{ms - prev:8.4f} ms")
            prev = ms
        if cfg == args.configs.split(",")[-1]:
            print(f"  mean iters {d['iters'].float().mean().item():.2f}")
        eng.close()
    os.environ.pop("MPCQP_CUT", None)


if __name__ == "__main__":
    main()
