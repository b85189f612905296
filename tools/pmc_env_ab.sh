#!/bin/bash
# One PMC pass (8 SQ counters) of tools/run_once.py per (environment setting, batch) on the GPU
# box: per-wave instruction mix of a library variant selected by an environment variable
# (e.g. MPCQP_CRASH_P).  Usage: tools/pmc_env_ab.sh OUT "MPCQP_CRASH_P=0" "MPCQP_CRASH_P=8" ...
# [BATCHES="4096 65536"] [CONFIG=B] [CTRS="8 SQ counters"]
OUT=${1:-gpurun_out/pmcab}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
R=$(pwd)
CTRS=${CTRS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_BRANCH"}
for spec in "$@"; do
  for B in ${BATCHES:-4096 65536}; do
    d="$OUT/${spec//[=]/_}_$B"
    env "$spec" timeout -s KILL 90 rocprofv3 --pmc $CTRS -d "$R/$d" -o run --output-format csv \
        -- python3 tools/run_once.py --config ${CONFIG:-B} --batch $B --reps 5 > "$d.log" 2>&1 || { echo "failed: $spec $B"; tail -3 "$d.log"; exit 1; }
  done
done
echo pmc done
