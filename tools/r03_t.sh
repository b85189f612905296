#!/bin/bash
# R^-1 + parallel drop in the one-QP solver (configs C, L): GPU tests, A/B
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03t}
TAG=$T tools/gpu_tests.sh || exit 1
AB_CONFIGS=C AB_REPS=20 timeout -k 10 300 tools/ab_libs.sh default rr0c default rr0c > gpurun_out/${T}_C.log 2>&1 || { cat gpurun_out/${T}_C.log; exit 1; }
cat gpurun_out/${T}_C.log
AB_CONFIGS=L AB_REPS=20 timeout -k 10 300 tools/ab_libs.sh default rr0l default rr0l > gpurun_out/${T}_L.log 2>&1 || { cat gpurun_out/${T}_L.log; exit 1; }
cat gpurun_out/${T}_L.log
AB_CONFIGS=C AB_GAIT=mixed AB_REPS=6 timeout -k 10 300 tools/ab_libs.sh default rr0c > gpurun_out/${T}_Cmix.log 2>&1 || { cat gpurun_out/${T}_Cmix.log; exit 1; }
cat gpurun_out/${T}_Cmix.log
