#!/bin/bash
# r05: A/B only (see r05_o.sh): C with / without the implied fz bound, E Pade swap guard
set -o pipefail
T=${1:-r05p}
mkdir -p gpurun_out
for r in 1 2 3; do
  AB_CONFIGS=C AB_REPS=20 bash tools/ab_libs.sh default noelide_c
  AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384 bash tools/ab_libs.sh default padeskip0_e
done > gpurun_out/${T}_ab.log 2>&1 || exit 1
cat gpurun_out/${T}_ab.log
