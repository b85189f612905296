#!/bin/bash
# Per-phase census of config E's k_dense_wg (16,384): the cuts build returns after phase k
# (MPCQP_CUT: 91 expm, 92 panels + gradient, 93 H rows, 104 factorisation, 105 J, 106 unconstrained
# minimum, 108 crash, 107 dual loop, 0 all); one rocprofv3 --pmc pass per cut, differences per wave.
# Usage (GPU box, repo root): tools/phase_pmc_e.sh OUT
set -e
OUT=${1:-gpurun_out/pe}
mkdir -p "$OUT"
export TMPDIR=/tmp
export MPCQP_LIB="$(pwd)/mpc-limx-control_amd/lib/libmpcqp_cuts.so"
R=$(pwd)
CUTS="91 92 93 104 105 106 108 107 0"
for cut in $CUTS; do
  MPCQP_CUT=$cut timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
      SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES \
      -d "$R/$OUT/c$cut" -o run --output-format csv -- python3 tools/run_once.py --config E \
      --batch 16384 > "$OUT/c$cut.log" 2>&1
done
python3 - "$OUT" "$CUTS" <<'PY'
import csv, glob, sys, collections
base, cuts = sys.argv[1], [int(c) for c in sys.argv[2].split()]
names = {91: "inputs+expm+free map", 92: "panels+gradient", 93: "H rows", 104: "factorisation",
         105: "J", 106: "unconstrained min", 108: "crash", 107: "dual loop", 0: "outputs"}
K = ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_WAVES",
     "SQ_WAVE_CYCLES")
prev = None
print(f"{'phase':22s} {'VALU/wv':>8s} {'SALU/wv':>8s} {'LDS/wv':>8s} {'confl/wv':>9s} {'cyc/wv':>9s}")
for cut in cuts:
    acc = collections.defaultdict(float)
    for f in glob.glob(f"{base}/c{cut}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_dense_wg" in r["Kernel_Name"]:
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
    w = acc["SQ_WAVES"] or 1
    cur = {k: acc[k] / w for k in K}
    d = {k: cur[k] - (prev[k] if prev else 0) for k in K}
    print(f"{names[cut]:22s} {d[K[0]]:8.0f} {d[K[1]]:8.0f} {d[K[2]]:8.0f} {d[K[3]]:9.0f} {4 * d[K[5]]:9.0f}")
    prev = cur
PY
