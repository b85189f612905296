#!/bin/bash
# diagonal-block Cholesky with DPP row broadcasts instead of v_readlane: GPU tests, A/B on E
# (edpp0 = MPCQP_DIAG_DPP=0 in fast_dense), C (cdpp0, fast_srbm20), L (ldpp0, fast_literal)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03y}
TAG=$T tools/gpu_tests.sh || exit 1
AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384 timeout -k 10 300 tools/ab_libs.sh default edpp0 default edpp0 > gpurun_out/${T}_E.log 2>&1 || { cat gpurun_out/${T}_E.log; exit 1; }
cat gpurun_out/${T}_E.log
AB_CONFIGS=C AB_REPS=10 timeout -k 10 300 tools/ab_libs.sh default cdpp0 default cdpp0 > gpurun_out/${T}_C.log 2>&1 || { cat gpurun_out/${T}_C.log; exit 1; }
cat gpurun_out/${T}_C.log
AB_CONFIGS=L AB_REPS=10 timeout -k 10 300 tools/ab_libs.sh default ldpp0 default ldpp0 > gpurun_out/${T}_L.log 2>&1 || { cat gpurun_out/${T}_L.log; exit 1; }
cat gpurun_out/${T}_L.log
