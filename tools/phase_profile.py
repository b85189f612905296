#!/usr/bin/env python3
"""Per-phase cycle shares of the fused kernels, from the diagnostic build
(lib/libmpcqp_stamps.so, -DMPCQP_STAMPS).  Never benchmark that build: the stamps serialize
the phases.  Usage:  python tools/phase_profile.py [--config B] [--batch 65536]"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("MPCQP_LIB", os.path.join(ROOT, "mpc-limx-control_amd", "lib",
                                                "libmpcqp_stamps.so"))
sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))

import numpy as np  # noqa: E402

NAMES = ["setup", "Phi/xf chains", "Qe (dense TOEP: H tiles)", "H_FF", "gradient", "Cholesky", "J=L^-T",
         "unconstrained min", "dual loop", "write", "model build (dense TOEP: H row pickup)", "expm",
         "  sub 12 (wg: selection, J-row publication)", "  sub 13 (wg: z = J2 d2, |d|^2)",
         "  sub 14 (wg: r = R^-1 d, t1, barrier)", "  sub 15 (wg: step, add/drop, J update)"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="B")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--gait", default="alternating", help="make_batch gait (GAITS)")
    args = ap.parse_args()
    import mpcqp
    from mpcqp._lib import lib
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params(args.config)
    eng = BatchEngine(p)
    d = eng.upload(mpcqp.make_batch(p, args.batch, gait=args.gait))
    buf = (C.c_uint64 * 16)()
    assert lib().mpcqp_debug_phase_cycles(eng.ctx, buf, 16) == 0, "not the stamps build"
    eng.solve(d)
    eng.sync()
    lib().mpcqp_debug_phase_cycles(eng.ctx, buf, 16)  # reset after warm-up
    eng.solve(d)
    eng.sync()
    assert lib().mpcqp_debug_phase_cycles(eng.ctx, buf, 16) == 0
    cyc = np.array(buf[:16], dtype=np.float64) / args.batch
    tot_cs = cyc[:10].sum()
    print(f"config {args.config}, gait {args.gait}, batch {args.batch}, mean iters "
          f"{d['iters'].float().mean().item():.2f}; cycles per QP (wave-serial)")
    for i, n in enumerate(NAMES):
        den = tot_cs if (i < 10 or i >= 12) else cyc[10:12].sum()
        share = cyc[i] / den if den > 0 else 0.0
        print(f"  {i:2d} {n:38s} {cyc[i]:10.0f}  {100 * share:5.1f}%")
    print(f"  condense_solve total {tot_cs:10.0f} ; discretize total {cyc[10:12].sum():10.0f}")
    eng.close()


if __name__ == "__main__":
    main()
