#!/bin/bash
# Pade Gauss-Jordan with implicit row swaps: GPU tests, E A/B (pim0 = explicit swaps, pim3 = implicit, positions in a VGPR, column read twice)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03ac}
[ -n "$NOTEST" ] || TAG=$T tools/gpu_tests.sh || exit 1
AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384 timeout -k 10 300 tools/ab_libs.sh pim0 pim3 pim0 pim3 > gpurun_out/${T}_E.log 2>&1 || { cat gpurun_out/${T}_E.log; exit 1; }
cat gpurun_out/${T}_E.log
