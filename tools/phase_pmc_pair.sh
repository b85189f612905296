#!/bin/bash
# Per-phase instruction census of k_mpc_pair (config B): the cuts build (lib/libmpcqp_cuts.so)
# returns after phase k when MPCQP_CUT=k; one rocprofv3 --pmc pass per cut (8 SQ counters), and
# the differences between successive cuts are what each phase issues per wavefront.
# Usage (GPU box, repo root): tools/phase_pmc_pair.sh OUT [CONFIG]
set -e
OUT=${1:-gpurun_out/ppair}
CFG=${2:-B}
mkdir -p "$OUT"
export TMPDIR=/tmp
export MPCQP_LIB="$(pwd)/mpc-limx-control_amd/lib/libmpcqp_cuts.so"
R=$(pwd)
CUTS="11 1 13 2 3 4 6 8 7 0"
for cut in $CUTS; do
  MPCQP_CUT=$cut timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
      SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 \
      -d "$R/$OUT/$CFG/c$cut" -o run --output-format csv -- python3 tools/run_once.py --config $CFG \
      --max-free 30 > "$OUT/$CFG.c$cut.log" 2>&1
done
python3 - "$OUT/$CFG" "$CUTS" <<'PY'
import csv, glob, sys, collections
base, cuts = sys.argv[1], [int(c) for c in sys.argv[2].split()]
names = {11: "inputs (+ pairing)", 1: "free map", 13: "model", 2: "S + u/v", 3: "g + H build + rows",
         4: "Cholesky + inverse", 6: "unconstrained min", 8: "crash start",
         7: "dual loop", 0: "outputs"}
K = ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "F64")
prev = None
print(f"{'phase':22s} {'VALU/wave':>10s} {'F64/wave':>9s} {'SALU/wave':>10s} {'LDS/wave':>9s}")
for cut in cuts:
    acc = collections.defaultdict(float)
    for f in glob.glob(f"{base}/c{cut}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_mpc_pair" in r["Kernel_Name"]:
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
    w = acc["SQ_WAVES"] or 1
    acc["F64"] = sum(acc[k] for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64",
                                      "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64"))
    cur = {k: acc[k] / w for k in K}
    d = {k: cur[k] - (prev[k] if prev else 0) for k in K}
    print(f"{names[cut]:22s} {d[K[0]]:10.0f} {d['F64']:9.0f} {d[K[1]]:10.0f} {d[K[2]]:9.0f}"
          f"   (cum VALU {cur[K[0]]:.0f})")
    prev = cur
PY
