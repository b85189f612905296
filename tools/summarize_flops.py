#!/usr/bin/env python3
"""Summarize a tools/pmc_flops.sh output directory into profiles/pmc_flops.json: executed FP64
work of one kernel per launch (median over its dispatches).
  executed_flops_per_launch  64 lanes x SQ_INSTS_VALU_FLOPS_FP64 + 512 x SQ_INSTS_VALU_MFMA_MOPS_F64.
                             SQ_INSTS_VALU_FLOPS_FP64 counts per WAVE instruction (it equals
                             2 FMA + MUL + ADD + TRANS F64 instructions exactly, profiles/
                             pmc_flops.json r02_v1), so x 64 counts every lane, EXEC-masked
                             lanes included: an upper bound of the lane FLOPs executed
  lane_flops_upper_bound     the same bound from the per-type counters
  mfma_busy_frac             SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
Usage: tools/summarize_flops.py PROFDIR TAG --kernel k_mpc_pair [--config B --batch 65536]"""
import argparse
import collections
import csv
import json
import os
import statistics as st

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_tag(name):
    i = name.find("k_")
    j = name.find(">", i)
    return name[i:j + 1] if i >= 0 and j > i else name


def per_dispatch(path, kernel, grid=None):
    """{counter: median over dispatches of `kernel` (exact instantiation when it names one,
    e.g. 'k_mpc_pair<6, 10, 0, false, 4>', else a substring) at `grid` threads of the
    per-dispatch total}"""
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if ("<" in kernel and kernel_tag(name) != kernel) or kernel not in name:
            continue
        if grid is not None and int(r["Grid_Size"]) != grid:
            continue
        acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {c: st.median(v.values()) for c, v in acc.items()}, \
        {c: len(v) for c, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof")
    ap.add_argument("tag")
    ap.add_argument("--kernel", default="k_mpc_pair")
    ap.add_argument("--config", default="B")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--out", default="pmc_flops.json")
    ap.add_argument("--grid", type=int, default=None, help="threads per launch (default: all)")
    a = ap.parse_args()
    sq, n = per_dispatch(os.path.join(a.prof, "sq", "run_counter_collection.csv"), a.kernel, a.grid)
    try:
        gr, _ = per_dispatch(os.path.join(a.prof, "grbm", "run_counter_collection.csv"), a.kernel,
                             a.grid)
    except OSError:
        gr = {}
    g = lambda k: sq.get(k, 0.0)
    executed = 64.0 * g("SQ_INSTS_VALU_FLOPS_FP64") + 512.0 * g("SQ_INSTS_VALU_MFMA_MOPS_F64")
    upper = 64.0 * (2 * g("SQ_INSTS_VALU_FMA_F64") + g("SQ_INSTS_VALU_MUL_F64") +
                    g("SQ_INSTS_VALU_ADD_F64") + g("SQ_INSTS_VALU_TRANS_F64")) + \
        512.0 * g("SQ_INSTS_VALU_MFMA_MOPS_F64")
    import summarize_profile
    out = dict(tag=a.tag, lib_build_id=summarize_profile.lib_build_id(), kernel=a.kernel,
               grid=a.grid, config=a.config, batch=a.batch, file=a.out,
               counters=sq, dispatches=n, grbm=gr,
               executed_flops_per_launch=executed, lane_flops_upper_bound=upper,
               mfma_flops_per_launch=512.0 * g("SQ_INSTS_VALU_MFMA_MOPS_F64"))
    if gr.get("GRBM_GUI_ACTIVE"):
        cyc = gr["GRBM_GUI_ACTIVE"] / 8.0  # summed over the 8 XCDs (MI355X_MICROARCH.md)
        out["gui_active_cycles"] = cyc
        out["mfma_busy_frac"] = g("SQ_VALU_MFMA_BUSY_CYCLES") / (cyc * 1024.0)
    json.dump(out, open(os.path.join(ROOT, "profiles", a.out), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
