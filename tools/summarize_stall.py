#!/usr/bin/env python3
"""Per-launch SQ stall / issue counters of one kernel instantiation and grid (tools/pmc_stall.sh
output) -> profiles/<tag>_stall.json.  SQ_*_CYCLES-type counters are in quad-cycles summed over
waves; fractions are taken against SQ_WAVE_CYCLES.
Usage: tools/summarize_stall.py DIR TAG [--kernel 'k_mpc_pair<6, 10, 0, false, 4>'] [--grid 2097152]"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics as st
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def tag(name):
    i = name.find("k_")
    j = name.find(">", i)
    return name[i:j + 1] if i >= 0 and j > i else name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("tag")
    ap.add_argument("--kernel", default="k_mpc_pair<6, 10, 0, false, 4>")
    ap.add_argument("--grid", type=int, default=2097152)
    a = ap.parse_args()
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(a.dir, "g*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if tag(r["Kernel_Name"]) == a.kernel and int(r["Grid_Size"]) == a.grid:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    c = {k: st.median(v) for k, v in vals.items()}
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from summarize_profile import lib_build_id
    out = dict(tag=a.tag, lib_build_id=lib_build_id(), kernel=a.kernel, grid=a.grid, counters=c)
    wc = c.get("SQ_WAVE_CYCLES")
    if wc:
        out["frac_of_wave_cycles"] = {k: c[k] / wc for k in (
            "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
            "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_SCA")
            if k in c}
    if c.get("SQ_WAVES"):
        out["per_wave"] = {k: c[k] / c["SQ_WAVES"] for k in (
            "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH",
            "SQ_LDS_BANK_CONFLICT", "SQ_WAVE_CYCLES") if k in c}
    json.dump(out, open(os.path.join(ROOT, "profiles", f"{a.tag}_stall.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
