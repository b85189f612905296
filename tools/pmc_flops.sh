#!/bin/bash
# Executed-work counters of the bench's fused kernel (run on the GPU box from the repo root):
# one rocprofv3 --pmc pass (8 SQ counters, the per-pass limit) + one GRBM pass for the clock.
# Never combined with trace domains (pool rule).  Usage: tools/pmc_flops.sh OUT [bench args]
#   or tools/pmc_flops.sh OUT --driver "tools/time_kernel.py --configs C --reps 5"
set -e
OUT=${1:-gpurun_out/pmcf}
shift || true
if [ "$1" = "--driver" ]; then DRV=$2; ARGS=""; else DRV=bench.py; ARGS=${*:-"--steps 5 --warmup 1 --no-cpu-baseline --no-per-config"}; fi
mkdir -p "$OUT"
export TMPDIR=/tmp
R=$(pwd)
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 \
    SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 \
    SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU \
    -d "$R/$OUT/sq" -o run --output-format csv -- python3 $DRV $ARGS > "$OUT/sq.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT \
    -d "$R/$OUT/grbm" -o run --output-format csv -- python3 $DRV $ARGS > "$OUT/grbm.log" 2>&1
