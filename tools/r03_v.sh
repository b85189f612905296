#!/bin/bash
# Pade Gauss-Jordan without the per-update selects: GPU tests, then E A/B at 16,384
# (pns0 = MPCQP_PADE_NOSEL=0 in fast_dense)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03v}
TAG=$T tools/gpu_tests.sh || exit 1
AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384 timeout -k 10 300 tools/ab_libs.sh default pns0 default pns0 default pns0 > gpurun_out/${T}_E.log 2>&1 || { cat gpurun_out/${T}_E.log; exit 1; }
cat gpurun_out/${T}_E.log
