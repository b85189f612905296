#!/usr/bin/env python3
"""Per-wave SQ counters of the paired kernel from tools/pmc_env_ab.sh output directories
(median over the profiled launches).  Usage: tools/summarize_pmc_ab.py OUTDIR"""
import collections
import csv
import glob
import os
import statistics as st
import sys

base = sys.argv[1]
for d in sorted(glob.glob(os.path.join(base, "*"))):
    if not os.path.isdir(d):
        continue
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_mpc_pair" in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    c = {k: st.median(v) for k, v in vals.items()}
    w = c.get("SQ_WAVES", 0)
    if not w:
        continue
    per = {k: c[k] / w for k in c if k != "SQ_WAVES"}
    print(os.path.basename(d), "waves", int(w), " ".join(f"{k[3:]}={v:.0f}" for k, v in per.items()))
