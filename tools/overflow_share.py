#!/usr/bin/env python3
"""Share of instances whose free-variable count overflows the one-wave kernels (nf > 60 at N = 20,
nf > 30 at N = 10) for the product-envelope gaits.  CPU only."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "mpc-limx-control_amd"))
import mpcqp  # noqa: E402

for cfg, g in (("C", "mixed"), ("B", "standing"), ("B", "mixed")):
    p = mpcqp.model_params(cfg)
    b = mpcqp.make_batch(p, 4096, gait=g)
    nf = np.array([bin(int(x)).count("1") for x in b["contact"]]) * 3
    cap = 3 * p["N"]
    print(f"{cfg} {g}: mean nf {nf.mean():.1f}, overflow (nf > {cap}) {np.mean(nf > cap):.3f}")
