#!/usr/bin/env python3
"""Summarize a tools/profile_run.sh output directory into profiles/:
  <tag>_kernel_stats.csv   rocprofv3 --stats summary (copied verbatim; it averages by kernel NAME
                           over every grid and workload of the run)
  <tag>_summary.json       per (kernel instantiation, grid, workgroup) average duration from the
                           kernel trace, the headline group (--kernel at --grid), PMC HBM traffic
                           per launch, and the source hash of the profiled library
  pmc_traffic.json         the k_mpc traffic figure bench.py reports as roofline.traffic
HBM bytes follow MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are KiB,
collected in separate passes; on gfx950 FETCH_SIZE counts half of the bytes of a coalesced
stream, so reads are doubled.  Usage: tools/summarize_profile.py PROFDIR TAG [--batch B]"""
import argparse
import csv
import json
import os
import shutil
import statistics as st

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_tag(name):
    """'k_mpc_pair<6, 10, 0, false, 4>' out of the demangled signature."""
    i = name.find("k_")
    j = name.find(">", i)
    return name[i:j + 1] if i >= 0 and j > i else name


def counter(path, kernel, grid):
    """Median counter value over the launches of exactly this kernel instantiation at this
    grid size (other configs and the bench's side measurements launch other instantiations
    or grids of the same kernel family)."""
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
         if kernel_tag(r["Kernel_Name"]) == kernel and int(r["Grid_Size"]) == grid]
    return st.median(v) if v else None, len(v)


def lib_build_id():
    """source hash compiled into the library that was profiled (mpcqp_build_id): the one the GPU
    run recorded (MPCQP_PROFILED_BUILD_ID, set by tools/summarize_evidence.sh from the run's bench
    line), else the in-tree library's"""
    if os.environ.get("MPCQP_PROFILED_BUILD_ID"):
        return os.environ["MPCQP_PROFILED_BUILD_ID"]
    try:
        import ctypes
        L = ctypes.CDLL(os.path.join(ROOT, "mpc-limx-control_amd", "lib", "libmpcqp.so"))
        L.mpcqp_build_id.restype = ctypes.c_char_p
        return L.mpcqp_build_id().decode()
    except (OSError, AttributeError):
        return None


def dispatch_groups(trace):
    """per (kernel instantiation, grid, workgroup) average duration over its dispatches in the
    kernel trace -- the rocprofv3 --stats summary averages by NAME, mixing grids and workloads"""
    g = {}
    for r in csv.DictReader(open(trace)):
        key = (kernel_tag(r["Kernel_Name"]), int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))
        g.setdefault(key, []).append((int(r["Start_Timestamp"]),
                                      (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3))
    out = []
    for (k, grid, wg), tv in sorted(g.items(), key=lambda kv: -sum(d for _, d in kv[1])):
        v = [d for _, d in sorted(tv)]  # in dispatch order
        # the last 40 dispatches: bench.py's two measurement passes after its timed steps (HIP
        # events around the solve, then the library's per-kernel events), at steady clocks --
        # the first launches of a fresh process run while the clocks ramp
        tail = v[-40:]
        out.append(dict(kernel=k, grid_threads=grid, workgroup=wg, calls=len(v),
                        avg_us=st.mean(v), median_us=st.median(v), min_us=min(v), max_us=max(v),
                        last40_avg_us=st.mean(tail), last40_median_us=st.median(tail)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof")
    ap.add_argument("tag")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--config", default="B")
    ap.add_argument("--kernel", default="k_mpc_pair<6, 10, 0, false, 4>")
    ap.add_argument("--grid", type=int, default=None,
                    help="threads per launch (default: 32 x batch, the pair kernel's grid)")
    ap.add_argument("--no-traffic-json", action="store_true",
                    help="per-config runs (C, E): do not overwrite profiles/pmc_traffic.json, the "
                         "headline figure bench.py reads")
    a = ap.parse_args()
    out = os.path.join(ROOT, "profiles")
    stats = os.path.join(a.prof, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(out, f"{a.tag}_kernel_stats.csv"))
    kern = {r["Name"]: dict(calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]),
                            pct=float(r["Percentage"])) for r in csv.DictReader(open(stats))}
    grid = a.grid or 32 * a.batch
    groups = dispatch_groups(os.path.join(a.prof, "trace", "run_kernel_trace.csv"))
    head = [g for g in groups if g["kernel"] == a.kernel and g["grid_threads"] == grid]
    fetch = write = None
    nf = nw = 0
    if os.path.exists(os.path.join(a.prof, "fetch")):  # trace-only runs have no counter passes
        fetch, nf = counter(os.path.join(a.prof, "fetch", "run_counter_collection.csv"), a.kernel, grid)
        write, nw = counter(os.path.join(a.prof, "write", "run_counter_collection.csv"), a.kernel, grid)
    traffic = None
    if fetch is not None and write is not None:
        traffic = 2.0 * fetch * 1024 + write * 1024
    summ = dict(tag=a.tag, lib_build_id=lib_build_id(), kernel=a.kernel, grid=grid, config=a.config,
                batch=a.batch, headline=head[0] if head else None, dispatch_groups=groups,
                kernels_by_name_mixed_grids=kern,
                fetch_size_kib_median=fetch, write_size_kib_median=write, fetch_samples=nf,
                write_samples=nw, hbm_bytes_per_launch=traffic,
                correction="reads = 2 x FETCH_SIZE (gfx950 half-count), writes = WRITE_SIZE")
    json.dump(summ, open(os.path.join(out, f"{a.tag}_summary.json"), "w"), indent=1)
    if traffic is not None and not a.no_traffic_json:
        json.dump(dict(config=a.config, batch=a.batch, kernel=a.kernel, grid=grid, tag=a.tag,
                   lib_build_id=summ["lib_build_id"],
                   hbm_bytes_per_launch=traffic, read_bytes=2.0 * fetch * 1024 if fetch else None,
                   write_bytes=write * 1024 if write else None), open(os.path.join(out, "pmc_traffic.json"), "w"),
                  indent=1)
    print(json.dumps(summ, indent=1)[:1500])


if __name__ == "__main__":
    main()
