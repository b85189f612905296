#!/bin/bash
# r05: the evidence set at the current library (tools/evidence.sh), then a paired-kernel A/B
# (libmpcqp_foldasel.so: the folded rows loaded from a selected address) at 65,536 / 4,096
set -o pipefail
T=${1:-r05b}
mkdir -p gpurun_out
bash tools/evidence.sh $T || exit 1
for r in 1 2 3; do
  AB_CONFIGS=B AB_REPS=60 bash tools/ab_libs.sh default foldasel
  AB_CONFIGS=B AB_BATCH=4096 AB_REPS=60 bash tools/ab_libs.sh default foldasel
done > gpurun_out/${T}_ab.log 2>&1 || exit 1
cat gpurun_out/${T}_ab.log
