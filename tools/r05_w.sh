#!/bin/bash
# r05: paired-kernel A/B (libmpcqp_hbbases.so: H-build sub-block bases, FMA-masked g terms) at
# 65,536 / 4,096, then the GPU suite with that build as the library under test
set -o pipefail
T=${1:-r05x}
mkdir -p gpurun_out
for r in 1 2 3; do
  AB_CONFIGS=B AB_REPS=60 bash tools/ab_libs.sh default hbbases
  AB_CONFIGS=B AB_BATCH=4096 AB_REPS=60 bash tools/ab_libs.sh default hbbases
done > gpurun_out/${T}_ab.log 2>&1 || exit 1
cat gpurun_out/${T}_ab.log
MPCQP_LIB=$PWD/mpc-limx-control_amd/lib/libmpcqp_hbbases.so TAG=$T bash tools/gpu_tests.sh -k "pair or batch_vs_oracle or gait or crash" || exit 1
