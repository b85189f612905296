#!/bin/bash
# wave-split R^-1 product + structural-zero skipping in the workgroup solver: GPU tests, A/B
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03l}
TAG=$T tools/gpu_tests.sh || exit 1
AB_CONFIGS=C AB_GAIT=mixed AB_REPS=8 timeout -k 10 500 tools/ab_libs.sh default wgb wgs0 wgp0 default wgb wgs0 wgp0 > gpurun_out/${T}_Cmix.log 2>&1 || { cat gpurun_out/${T}_Cmix.log; exit 1; }
cat gpurun_out/${T}_Cmix.log
AB_CONFIGS=B AB_GAIT=standing AB_REPS=20 timeout -k 10 300 tools/ab_libs.sh default wgb default wgb > gpurun_out/${T}_Bst.log 2>&1 || { cat gpurun_out/${T}_Bst.log; exit 1; }
cat gpurun_out/${T}_Bst.log
AB_CONFIGS=E AB_REPS=10 timeout -k 10 300 tools/ab_libs.sh default dnb default dnb > gpurun_out/${T}_E.log 2>&1 || { cat gpurun_out/${T}_E.log; exit 1; }
cat gpurun_out/${T}_E.log
