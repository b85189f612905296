#!/bin/bash
# wg selection bound states in registers (NF > 64) and the fused diagonal-block inverse:
# GPU tests + A/B on E, C mixed, B standing
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03x}
TAG=$T tools/gpu_tests.sh || exit 1
AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384 timeout -k 10 300 tools/ab_libs.sh default ds0 df0 default ds0 df0 > gpurun_out/${T}_E.log 2>&1 || { cat gpurun_out/${T}_E.log; exit 1; }
cat gpurun_out/${T}_E.log
AB_CONFIGS=C AB_GAIT=mixed AB_REPS=5 timeout -k 10 400 tools/ab_libs.sh default ws0 wf0 default ws0 wf0 > gpurun_out/${T}_Cmix.log 2>&1 || { cat gpurun_out/${T}_Cmix.log; exit 1; }
cat gpurun_out/${T}_Cmix.log
AB_CONFIGS=B AB_GAIT=standing AB_REPS=10 timeout -k 10 300 tools/ab_libs.sh default wf0 default wf0 > gpurun_out/${T}_Bst.log 2>&1 || { cat gpurun_out/${T}_Bst.log; exit 1; }
cat gpurun_out/${T}_Bst.log
AB_CONFIGS=C AB_REPS=20 timeout -k 10 300 tools/ab_libs.sh default cf0 default cf0 > gpurun_out/${T}_C.log 2>&1 || { cat gpurun_out/${T}_C.log; exit 1; }
cat gpurun_out/${T}_C.log
