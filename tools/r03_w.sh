#!/bin/bash
# one-wave register Gauss-Jordan for E's Pade quotient: dense tests, A/B, stamps
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03w}
true
AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384 timeout -k 10 300 tools/ab_libs.sh default pe0 pl0 ef0 default pe0 pl0 ef0 > gpurun_out/${T}_E16k.log 2>&1 || { cat gpurun_out/${T}_E16k.log; exit 1; }
cat gpurun_out/${T}_E16k.log
true
true
