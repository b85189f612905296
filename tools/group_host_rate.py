#!/usr/bin/env python3
"""Host-to-host rate of the C-ABI group's host path (mpcqp_group_solve_select_host, one member
on device 0): pageable arrays through the members' pinned staging vs page-locked caller arrays
(mpcqp_host_register on page-aligned copies: each shard DMA'd straight from and into them).
Usage: python tools/group_host_rate.py [--states 4096] [--reps 5]"""
import argparse
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))
import numpy as np  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--states", type=int, default=4096)
ap.add_argument("--reps", type=int, default=5)
args = ap.parse_args()
import mpcqp  # noqa: E402
from mpcqp._lib import lib  # noqa: E402
from mpcqp.group import Group  # noqa: E402

p = mpcqp.model_params("B")
S, Cn = args.states, 16
B, nV = S * Cn, p["nu"] * p["N"]
batch = mpcqp.make_batch(p, B, seed=7)
grp = Group(p, devices=[0])


def rate(b, out=None):
    grp.solve_select_host(S, Cn, b, out=out)
    t = time.perf_counter()
    for _ in range(args.reps):
        grp.solve_select_host(S, Cn, b, out=out)
    return B * args.reps / (time.perf_counter() - t)


for _ in range(2):
    pg = rate(batch)
    locked = {k: mpcqp.page_aligned(batch[k]) for k in ("x0", "xref", "lin", "contact")}
    out = dict(U=mpcqp.page_aligned_empty((B, nV), np.float64),
               cost=mpcqp.page_aligned_empty(B, np.float64),
               status=mpcqp.page_aligned_empty(B, np.int32),
               iters=mpcqp.page_aligned_empty(B, np.int32))
    arrs = list(locked.values()) + list(out.values())
    for a in arrs:
        assert lib().mpcqp_host_register(C.c_void_p(a.ctypes.data), C.c_size_t(a.nbytes)) == 0
    lk = rate(locked, out)
    for a in arrs:
        lib().mpcqp_host_unregister(C.c_void_p(a.ctypes.data))
    print(f"group host path B {B}: page-locked {lk / 1e6:7.2f} M QP/s   pageable {pg / 1e6:7.2f} M QP/s",
          flush=True)
grp.close()
