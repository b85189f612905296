#!/usr/bin/env python3
"""Per-kernel HBM bytes per launch from tools/ab_traffic.sh / profile_run.sh counter passes:
reads = 2 x FETCH_SIZE (gfx950 half count), writes = WRITE_SIZE (KiB).
Usage: tools/traffic_table.py DIR [DIR ...]   (DIR holds FETCH_SIZE/ and WRITE_SIZE/ or fetch/ and write/)"""
import collections
import csv
import glob
import os
import statistics as st
import sys


def tag(name):
    i = name.find("k_")
    j = name.find(">", i)
    return name[i:j + 1] if i >= 0 and j > i else name[:40]


def load(d, sub):
    f = glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True)
    agg = collections.defaultdict(list)
    for path in f:
        for r in csv.DictReader(open(path)):
            if "mpcqp" in r["Kernel_Name"]:
                agg[(tag(r["Kernel_Name"]), int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return {k: st.median(v) for k, v in agg.items()}


for d in sys.argv[1:]:
    fe = load(d, "FETCH_SIZE") or load(d, "fetch")
    wr = load(d, "WRITE_SIZE") or load(d, "write")
    print(f"== {d}")
    for k in sorted(set(fe) | set(wr)):
        r = 2 * fe.get(k, 0) * 1024 / 1e6
        w = wr.get(k, 0) * 1024 / 1e6
        print(f"  {k[0]:45s} grid {k[1]:8d}  read {r:8.1f} MB  write {w:8.1f} MB  total {r + w:8.1f} MB")
