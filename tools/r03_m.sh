#!/bin/bash
# parallel drop rotations in the workgroup solver: GPU tests, A/B vs the sequential drop
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03m}
TAG=$T tools/gpu_tests.sh || exit 1
AB_CONFIGS=C AB_GAIT=mixed AB_REPS=8 timeout -k 10 400 tools/ab_libs.sh default wgd0 default wgd0 > gpurun_out/${T}_Cmix.log 2>&1 || { cat gpurun_out/${T}_Cmix.log; exit 1; }
cat gpurun_out/${T}_Cmix.log
AB_CONFIGS=B AB_GAIT=standing AB_REPS=20 timeout -k 10 300 tools/ab_libs.sh default wgd0 default wgd0 > gpurun_out/${T}_Bst.log 2>&1 || { cat gpurun_out/${T}_Bst.log; exit 1; }
cat gpurun_out/${T}_Bst.log
AB_CONFIGS=E AB_REPS=10 timeout -k 10 300 tools/ab_libs.sh default dnd0 default dnd0 > gpurun_out/${T}_E.log 2>&1 || { cat gpurun_out/${T}_E.log; exit 1; }
cat gpurun_out/${T}_E.log
