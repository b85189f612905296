#!/bin/bash
# r05: machine-scheduler strategy A/B per kernel family (B: fast_pair, C: fast_srbm20, E:
# fast_dense) -- max-memory-clause, iterative-ilp, iterative-minreg against the defaults
set -o pipefail
T=${1:-r05ad}
mkdir -p gpurun_out
for r in 1 2; do
  AB_CONFIGS=B AB_REPS=60 bash tools/ab_libs.sh default sb_max-memory-clause sb_iterative-ilp sb_iterative-minreg
  AB_CONFIGS=C AB_REPS=20 bash tools/ab_libs.sh default sc_max-memory-clause sc_iterative-ilp sc_iterative-minreg
  AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384 bash tools/ab_libs.sh default se_max-memory-clause se_iterative-ilp se_iterative-minreg
done > gpurun_out/${T}_ab.log 2>&1 || exit 1
cat gpurun_out/${T}_ab.log
