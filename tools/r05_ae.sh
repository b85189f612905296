#!/bin/bash
# r05: the crash's Gram matrix by entry pairs over every lane (libmpcqp_cpairs.so) -- A/B at
# 65,536 / 4,096 and the crash / parity tests with that build
set -o pipefail
T=${1:-r05ae}
mkdir -p gpurun_out
for r in 1 2 3; do
  AB_CONFIGS=B AB_REPS=60 bash tools/ab_libs.sh default cpairs
  AB_CONFIGS=B AB_BATCH=4096 AB_REPS=60 bash tools/ab_libs.sh default cpairs
done > gpurun_out/${T}_ab.log 2>&1 || exit 1
cat gpurun_out/${T}_ab.log
MPCQP_LIB=$PWD/mpc-limx-control_amd/lib/libmpcqp_cpairs.so TAG=$T bash tools/gpu_tests.sh -k "pair or batch_vs_oracle or gait or crash or flops" || exit 1
