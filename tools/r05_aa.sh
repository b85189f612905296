#!/bin/bash
# r05: config E A/B -- the default scheduler instead of max-ilp for fast_dense (noilp_e), the Pade
# column read row by row after the swap (padelate_e)
set -o pipefail
T=${1:-r05aa}
mkdir -p gpurun_out
for r in 1 2 3; do
  AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384 bash tools/ab_libs.sh default noilp_e padelate_e
done > gpurun_out/${T}_ab.log 2>&1 || exit 1
cat gpurun_out/${T}_ab.log
