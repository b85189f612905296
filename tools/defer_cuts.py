#!/usr/bin/env python3
"""Where the paired kernel's deferral path spends its time (B standing: every instance goes to
the workgroup kernel).  Cuts build (lib/libmpcqp_cuts.so): k_mpc_pair alone (library events,
slot 2) with the kernel returning after the inputs (cut 11), after the free map (cut 1) and in
full (cut 0: + the wavefront's overflow-list append).  Never benchmark that build.
  python tools/defer_cuts.py [--batch 65536] [--reps 10] [--gait standing]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("MPCQP_LIB", os.path.join(ROOT, "mpc-limx-control_amd", "lib",
                                                "libmpcqp_cuts.so"))
sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--gait", default="standing")
    a = ap.parse_args()
    import mpcqp
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params("B")
    eng = BatchEngine(p)
    d = eng.upload(mpcqp.make_batch(p, a.batch, gait=a.gait))
    eng.enable_timing(True)
    for cut, name in ((11, "inputs"), (1, "inputs + free map"), (0, "full (+ append)")):
        os.environ["MPCQP_CUT"] = str(cut)
        ts = []
        for r in range(a.reps + 2):
            eng.solve(d)
            eng.sync()
            if r >= 2:
                ts.append(eng.last_kernel_ms(2))
        print(f"  cut {cut:2d} {name:20s} k_mpc_pair {np.median(ts) * 1e3:7.1f} us", flush=True)
    os.environ.pop("MPCQP_CUT", None)
    eng.close()


if __name__ == "__main__":
    main()
