#!/bin/bash
# diagonal-block Cholesky without the per-update mask: GPU tests, A/B on E (dns0) and
# B standing / C mixed (wdns0)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03w}
TAG=$T tools/gpu_tests.sh || exit 1
AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384 timeout -k 10 300 tools/ab_libs.sh default dns0 default dns0 > gpurun_out/${T}_E.log 2>&1 || { cat gpurun_out/${T}_E.log; exit 1; }
cat gpurun_out/${T}_E.log
AB_CONFIGS=B AB_GAIT=standing AB_REPS=10 timeout -k 10 300 tools/ab_libs.sh default wdns0 default wdns0 > gpurun_out/${T}_Bst.log 2>&1 || { cat gpurun_out/${T}_Bst.log; exit 1; }
cat gpurun_out/${T}_Bst.log
AB_CONFIGS=C AB_GAIT=mixed AB_REPS=5 timeout -k 10 300 tools/ab_libs.sh default wdns0 default wdns0 > gpurun_out/${T}_Cmix.log 2>&1 || { cat gpurun_out/${T}_Cmix.log; exit 1; }
cat gpurun_out/${T}_Cmix.log
