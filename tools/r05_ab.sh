#!/bin/bash
# r05: default scheduler (no max-ilp) A/B: E with the late Pade column read (noilplate_e) against
# the no-ilp build alone, C (noilp_c) and the paired kernel (noilp_b)
set -o pipefail
T=${1:-r05ab}
mkdir -p gpurun_out
for r in 1 2 3; do
  AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384 bash tools/ab_libs.sh noilp_e noilplate_e
  AB_CONFIGS=C AB_REPS=20 bash tools/ab_libs.sh default noilp_c
  AB_CONFIGS=B AB_REPS=60 bash tools/ab_libs.sh default noilp_b
done > gpurun_out/${T}_ab.log 2>&1 || exit 1
cat gpurun_out/${T}_ab.log
