#!/bin/bash
# R^-1 in the workgroup solver: GPU tests, then alternating A/B (default = R^-1, wgr0/dnr0 = R)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03j}
TAG=$T tools/gpu_tests.sh || exit 1
AB_CONFIGS=B AB_GAIT=standing AB_REPS=20 timeout -k 10 300 tools/ab_libs.sh default wgr0 default wgr0 > gpurun_out/${T}_Bst.log 2>&1 || { cat gpurun_out/${T}_Bst.log; exit 1; }
cat gpurun_out/${T}_Bst.log
AB_CONFIGS=C AB_GAIT=mixed AB_REPS=8 timeout -k 10 400 tools/ab_libs.sh default wgr0 default wgr0 > gpurun_out/${T}_Cmix.log 2>&1 || { cat gpurun_out/${T}_Cmix.log; exit 1; }
cat gpurun_out/${T}_Cmix.log
AB_CONFIGS=E AB_REPS=10 timeout -k 10 300 tools/ab_libs.sh default dnr0 default dnr0 > gpurun_out/${T}_E.log 2>&1 || { cat gpurun_out/${T}_E.log; exit 1; }
cat gpurun_out/${T}_E.log
