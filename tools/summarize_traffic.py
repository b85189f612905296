#!/usr/bin/env python3
"""profiles/pmc_traffic_<config>.json from a FETCH_SIZE / WRITE_SIZE pass pair (tools/ab_traffic.sh
or the evidence.sh layout: DIR/{FETCH_SIZE,WRITE_SIZE}/run_counter_collection.csv), for one
kernel instantiation at one grid size.  reads = 2 x FETCH_SIZE (gfx950 half count), writes =
WRITE_SIZE, KiB.  bench.py's per_config lines report it beside the algorithmic bytes.
Usage: tools/summarize_traffic.py DIR TAG --config C --batch 65536 --kernel 'k_mpc<6, 20, 0, true, 60>' --grid 4194304"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_profile import counter, lib_build_id  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("tag")
    ap.add_argument("--config", required=True)
    ap.add_argument("--batch", type=int, required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--grid", type=int, required=True)
    a = ap.parse_args()
    sub = (lambda n, alt: n if os.path.isdir(os.path.join(a.dir, n)) else alt)
    fetch, nf = counter(os.path.join(a.dir, sub("FETCH_SIZE", "fetch"), "run_counter_collection.csv"),
                        a.kernel, a.grid)
    write, nw = counter(os.path.join(a.dir, sub("WRITE_SIZE", "write"), "run_counter_collection.csv"),
                        a.kernel, a.grid)
    if fetch is None or write is None:
        sys.exit(f"no launches of {a.kernel} at grid {a.grid} in {a.dir}")
    out = dict(config=a.config, batch=a.batch, kernel=a.kernel, grid=a.grid, tag=a.tag,
               lib_build_id=lib_build_id(),
               read_bytes=2.0 * fetch * 1024, write_bytes=write * 1024,
               hbm_bytes_per_launch=2.0 * fetch * 1024 + write * 1024,
               fetch_samples=nf, write_samples=nw,
               correction="reads = 2 x FETCH_SIZE (gfx950 half-count), writes = WRITE_SIZE")
    json.dump(out, open(os.path.join(ROOT, "profiles", f"pmc_traffic_{a.config}.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
