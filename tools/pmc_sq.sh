#!/bin/bash
# Instruction-mix counters for the k_mpc kernel (one --pmc pass per group; never combined with
# trace domains).  Usage (GPU box, repo root): tools/pmc_sq.sh OUT [bench args]
set -e
OUT=${1:-gpurun_out/sq}
shift || true
ARGS=${*:-"--steps 3 --warmup 1 --no-cpu-baseline"}
mkdir -p "$OUT"
export TMPDIR=/tmp
R=$(pwd)
rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $grp -d "$R/$OUT/g$i" -o run --output-format csv \
        -- python3 bench.py $ARGS > "$OUT/g$i.log" 2>&1 || echo "group $i failed: $grp" >> "$OUT/fail.txt"
done
