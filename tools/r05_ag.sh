#!/bin/bash
# r05: the paired kernel's factorisation on the matrix cores (libmpcqp_pmfma.so, chol_pair.hpp)
# against the folded DPP sweep -- A/B at 65,536 / 4,096, then the paired-kernel tests with it
set -o pipefail
T=${1:-r05ag}
mkdir -p gpurun_out
MPCQP_LIB=$PWD/mpc-limx-control_amd/lib/libmpcqp_pmfma.so TAG=$T bash tools/gpu_tests.sh -k "pair or batch_vs_oracle or gait or crash or flops" || exit 1
for r in 1 2 3; do
  AB_CONFIGS=B AB_REPS=60 bash tools/ab_libs.sh default pmfma
  AB_CONFIGS=B AB_BATCH=4096 AB_REPS=60 bash tools/ab_libs.sh default pmfma
done > gpurun_out/${T}_ab.log 2>&1 || exit 1
cat gpurun_out/${T}_ab.log
