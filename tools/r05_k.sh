#!/bin/bash
# r05: A/B of variant libraries against the default, alternating processes, B at 65,536 / 4,096
set -o pipefail
T=${1:-r05k}; shift
mkdir -p gpurun_out
for r in 1 2 3; do
  AB_CONFIGS=B AB_REPS=60 bash tools/ab_libs.sh default "$@"
  AB_CONFIGS=B AB_BATCH=4096 AB_REPS=60 bash tools/ab_libs.sh default "$@"
done > gpurun_out/${T}_ab.log 2>&1 || exit 1
cat gpurun_out/${T}_ab.log
