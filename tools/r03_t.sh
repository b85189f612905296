#!/bin/bash
# look-ahead diagonal factorisation (chol_mfma.hpp) + E's free-map setup during the Pade solve:
# GPU tests, then alternating A/B: E at 16,384 (dla0 = look-ahead off in fast_dense), B standing
# and C mixed (wla0 = look-ahead off in fast_wg)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03t}
TAG=$T tools/gpu_tests.sh || exit 1
AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384 timeout -k 10 300 tools/ab_libs.sh default dla0 default dla0 > gpurun_out/${T}_E.log 2>&1 || { cat gpurun_out/${T}_E.log; exit 1; }
cat gpurun_out/${T}_E.log
AB_CONFIGS=B AB_GAIT=standing AB_REPS=10 timeout -k 10 300 tools/ab_libs.sh default wla0 default wla0 > gpurun_out/${T}_Bst.log 2>&1 || { cat gpurun_out/${T}_Bst.log; exit 1; }
cat gpurun_out/${T}_Bst.log
AB_CONFIGS=C AB_GAIT=mixed AB_REPS=5 timeout -k 10 300 tools/ab_libs.sh default wla0 default wla0 > gpurun_out/${T}_Cmix.log 2>&1 || { cat gpurun_out/${T}_Cmix.log; exit 1; }
cat gpurun_out/${T}_Cmix.log
