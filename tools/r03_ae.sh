#!/bin/bash
# diagonal-block factorisation with the next pivot read out first (MPCQP_DIAG_LA): GPU tests, A/B
# on E (dla0e = MPCQP_DIAG_LA=0 in fast_dense) and C (dla0c, fast_srbm20)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03ae}
TAG=$T tools/gpu_tests.sh || exit 1
AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384 timeout -k 10 300 tools/ab_libs.sh default dla0e default dla0e > gpurun_out/${T}_E.log 2>&1 || { cat gpurun_out/${T}_E.log; exit 1; }
cat gpurun_out/${T}_E.log
AB_CONFIGS=C AB_REPS=10 timeout -k 10 300 tools/ab_libs.sh default dla0c default dla0c > gpurun_out/${T}_C.log 2>&1 || { cat gpurun_out/${T}_C.log; exit 1; }
cat gpurun_out/${T}_C.log
