#!/usr/bin/env python3
"""Batch-size sweep of the config-B step (the strong-scaling shard sizes and below).

For each batch size: median over --reps of
  * solve     : mpcqp_batch_solve, HIP events on the ctx stream (k_mpc_pair [+ k_mpc_wg])
  * step      : solve + k_select_min record, torch events (what bench.py's step is at N = 1)
  * fused step: mpcqp_batch_solve_select (the record built by the solve kernels, bench --select fused)
and the mean / max solver passes.  With MPCQP_LIB pointing at libmpcqp_stamps.so it also
prints the per-WAVE cycles of each phase (s_memtime, summed over the wave's phases), which at
small batches is the latency of a lone wavefront.

  python tools/shard_sweep.py [--sizes 512,4096,8192] [--max-free 30] [--reps 50]
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))
import numpy as np  # noqa: E402

PH = {0: "setup", 1: "S+uv", 3: "H build", 5: "chol+inv", 7: "unc min", 8: "dual", 9: "write"}
SUB = {2: "passes", 12: "publish+d", 13: "z+R solve+t", 14: "add/drop", 15: "select+J upd"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="128,512,1024,2048,4096,6144,8192,12288,16384,32768,65536")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--config", default="B")
    ap.add_argument("--max-free", type=int, default=None)
    ap.add_argument("--gait", default=None)
    args = ap.parse_args()
    import torch

    import mpcqp
    from mpcqp._lib import lib
    from mpcqp.engine import BatchEngine
    stamps = "stamps" in os.environ.get("MPCQP_LIB", "")
    p = mpcqp.model_params(args.config)
    if args.max_free is not None:
        p["max_free"] = args.max_free
    print(f"lib {os.environ.get('MPCQP_LIB', 'default')} config {args.config} "
          f"max_free {p.get('max_free')}", flush=True)
    for B in [int(x) for x in args.sizes.split(",")]:
        batch = mpcqp.make_batch(p, B, seed=20250404, **({"gait": args.gait} if args.gait else {}))
        eng = BatchEngine(p)
        d = eng.upload(batch)
        rec = torch.zeros(1 + eng.nV, dtype=torch.int64, device="cuda")
        for _ in range(5):
            eng.solve(d)
            eng.select_record(d, rec)
        eng.sync()
        ks, ss, fs = [], [], []
        st = torch.cuda.current_stream()
        for _ in range(args.reps):  # solve and step, torch events (no library events inside)
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record(st)
            eng.solve(d)
            e1.record(st)
            eng.select_record(d, rec)
            e2.record(st)
            e2.synchronize()
            ks.append(e0.elapsed_time(e1))
            ss.append(e0.elapsed_time(e2))
            e3, e4 = (torch.cuda.Event(enable_timing=True) for _ in range(2))
            e3.record(st)
            eng.solve_select(d, rec)  # fused: the record from the solve kernels' last workgroup
            e4.record(st)
            e4.synchronize()
            fs.append(e3.elapsed_time(e4))
        # the one-wave kernel alone (library events around its launch), a separate pass
        eng.enable_timing(True)
        for _ in range(min(args.reps, 60)):
            eng.solve(d)
        eng.sync()
        kms, kn = eng.kernel_ms_sum(2)
        eng.enable_timing(False)
        it = d["iters"].cpu().numpy()
        stt = d["status"].cpu().numpy()
        line = (f"B {B:6d} kernel {kms / max(1, kn) * 1e3:7.1f} us solve {np.median(ks) * 1e3:7.1f} us"
                f"  step {np.median(ss) * 1e3:7.1f} us  fused step {np.median(fs) * 1e3:7.1f} us"
                f"  ({B / np.median(ss) / 1e3:7.2f} M QP/s)  iters mean {it.mean():.2f} max "
                f"{it.max():3d} solved {np.mean(stt == 0):.3f}")
        if stamps:
            buf = (C.c_uint64 * 16)()
            lib().mpcqp_debug_phase_cycles(eng.ctx, buf, 16)  # allocates the stamp slots
            eng.solve(d)  # (the first launch after allocation records)
            eng.sync()
            lib().mpcqp_debug_phase_cycles(eng.ctx, buf, 16)  # read + reset
            eng.solve(d)
            eng.sync()
            lib().mpcqp_debug_phase_cycles(eng.ctx, buf, 16)
            waves = (B + 1) // 2 if eng.fused_kernel == "k_mpc_pair" else B
            cyc = {n: buf[k] / waves for k, n in PH.items()}
            line += "\n    cycles/wave " + " ".join(f"{n} {v:.0f}" for n, v in cyc.items()) + \
                    f" | total {sum(cyc.values()):.0f}"
            npass = buf[2] / waves
            if npass > 0:
                line += f"\n    dual loop: {npass:.2f} passes/wave; cycles per pass " + " ".join(
                    f"{n} {buf[k] / waves / npass:.0f}" for k, n in SUB.items() if k != 2)
        print(line, flush=True)
        eng.close()


if __name__ == "__main__":
    main()
