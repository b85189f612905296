#!/bin/bash
# r05: GPU suite + fold A/B (alternating processes) at 65,536 and 4,096 (GPU box, repo root)
set -o pipefail
T=${1:-r05c}
mkdir -p gpurun_out
TAG=$T bash tools/gpu_tests.sh || exit 1
for r in 1 2 3; do
  AB_CONFIGS=B,L AB_REPS=60 bash tools/ab_libs.sh default nofold
  AB_CONFIGS=B AB_BATCH=4096 AB_REPS=60 bash tools/ab_libs.sh default nofold
done > gpurun_out/${T}_ab.log 2>&1 || exit 1
cat gpurun_out/${T}_ab.log
