#!/bin/bash
# Stall / issue counters of one kernel (two --pmc passes of <= 8 SQ counters each; never
# combined with trace domains).  Usage (GPU box, repo root):
#   tools/pmc_stall.sh OUT                     the bench's headline kernel ($ARGS: bench flags)
#   tools/pmc_stall.sh OUT --driver "tools/time_kernel.py --configs C --reps 5"
set -o pipefail
OUT=${1:-gpurun_out/stall}
shift || true
if [ "$1" = "--driver" ]; then DRV=$2; ARGS=""; else
  DRV=bench.py; ARGS=${ARGS:-"--steps 20 --warmup 20 --no-cpu-baseline --no-per-config --no-host-path"}; fi
mkdir -p "$OUT"
export TMPDIR=/tmp
R=$(pwd)
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp -d "$R/$OUT/g$i" -o run --output-format csv \
        -- python3 $DRV $ARGS > "$OUT/g$i.log" 2>&1 || { echo "group $i failed: $grp"; tail -3 "$OUT/g$i.log"; exit 1; }
done
echo stall done
