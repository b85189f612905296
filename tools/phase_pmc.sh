#!/bin/bash
# Per-phase instruction counts of k_mpc: the cuts build (lib/libmpcqp_cuts.so) run at each
# cut under rocprofv3 --pmc; differences between cuts = what each phase issues.
# Usage (GPU box, repo root): tools/phase_pmc.sh OUT CONFIG
set -e
OUT=${1:-gpurun_out/ppmc}
CFG=${2:-B}
mkdir -p "$OUT"
export TMPDIR=/tmp
export MPCQP_LIB="$(pwd)/mpc-limx-control_amd/lib/libmpcqp_cuts.so"
R=$(pwd)
for cut in 1 2 3 4 5 6 7 0; do
  MPCQP_CUT=$cut timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_LDS_BANK_CONFLICT \
      -d "$R/$OUT/$CFG/c$cut" -o run --output-format csv -- python3 tools/run_once.py --config $CFG \
      > "$OUT/$CFG.c$cut.log" 2>&1
done
python3 - "$OUT/$CFG" <<'PY'
import csv, glob, sys, collections
base = sys.argv[1]
names = {1: "inputs+model+setup", 2: "S+u/v", 3: "H build+load", 4: "Cholesky", 5: "J", 6: "unc. min",
         7: "dual loop", 0: "write"}
prev = None
print(f"{'phase':22s} {'VALU/QP':>9s} {'SALU/QP':>9s} {'LDS/QP':>9s} {'conflict cyc/QP':>16s}")
for cut in (1, 2, 3, 4, 5, 6, 7, 0):
    acc = collections.defaultdict(float)
    for f in glob.glob(f"{base}/c{cut}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_mpc<" in r["Kernel_Name"]:
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
    w = acc["SQ_WAVES"] or 1
    cur = {k: acc[k] / w for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT")}
    d = {k: cur[k] - (prev[k] if prev else 0) for k in cur}
    print(f"{names[cut]:22s} {d['SQ_INSTS_VALU']:9.0f} {d['SQ_INSTS_SALU']:9.0f} {d['SQ_INSTS_LDS']:9.0f}"
          f" {d['SQ_LDS_BANK_CONFLICT']:16.0f}"
          f"   (cum VALU {cur['SQ_INSTS_VALU']:.0f})")
    prev = cur
PY
