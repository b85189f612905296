#!/bin/bash
# r05: GPU suite + crash A/B (DPP vs LDS crash; both with the folded sweep)
set -o pipefail
T=${1:-r05f}
mkdir -p gpurun_out
TAG=$T bash tools/gpu_tests.sh || exit 1
for r in 1 2 3; do
  AB_CONFIGS=B AB_REPS=60 bash tools/ab_libs.sh default oldcrash
  AB_CONFIGS=B AB_BATCH=4096 AB_REPS=60 bash tools/ab_libs.sh default oldcrash
done > gpurun_out/${T}_ab.log 2>&1 || exit 1
cat gpurun_out/${T}_ab.log
