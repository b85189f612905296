#!/usr/bin/env python3
"""Bitwise comparison of two library builds on the same seeded batches (GPU box):
  python tools/cmp_libs.py LIB_A.so LIB_B.so  -- U, cost, status, iters of B@65536, B@4096, L@4096."""
import os, sys, subprocess, numpy as np
# run in two subprocesses with different MPCQP_LIB, dump results, compare bitwise
code = r'''
import os, sys, numpy as np
sys.path.insert(0, "mpc-limx-control_amd")
import mpcqp
from mpcqp.engine import BatchEngine
out = {}
for cfg, B, gait in (("B", 65536, "alternating"), ("B", 4096, "alternating"), ("L", 4096, "alternating")):
    p = mpcqp.model_params(cfg)
    eng = BatchEngine(p); d = eng.upload(mpcqp.make_batch(p, B, seed=123, gait=gait))
    eng.solve(d); eng.sync()
    for k in ("U", "cost", "status", "iters"):
        out[f"{cfg}{B}_{k}"] = d[k].cpu().numpy()
    eng.close()
np.savez(sys.argv[1], **out)
'''
libs = sys.argv[1:]
for i, l in enumerate(libs):
    env = dict(os.environ, MPCQP_LIB=l)
    subprocess.run([sys.executable, "-c", code, f"/tmp/cmp_{i}.npz"], env=env, check=True)
a = np.load("/tmp/cmp_0.npz"); b = np.load("/tmp/cmp_1.npz")
for k in a.files:
    x, y = a[k], b[k]
    same = np.array_equal(x.view(np.uint8), y.view(np.uint8)) if x.dtype.kind == "f" else np.array_equal(x, y)
    print(k, "bit-identical" if same else f"DIFFERS (max {np.abs(x.astype(float) - y.astype(float)).max():.3g})")
