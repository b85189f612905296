#!/bin/bash
# r05: GPU suite, then A/B: config C with / without the implied fz bound (MPCQP_ELIDE_FZ) and
# config E with the Pade pivot swap behind a p != k branch (MPCQP_PADE_SKIP) / without
set -o pipefail
T=${1:-r05o}
mkdir -p gpurun_out
TAG=$T bash tools/gpu_tests.sh || exit 1
for r in 1 2 3; do
  AB_CONFIGS=C AB_REPS=20 bash tools/ab_libs.sh default noelide_c
  AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384 bash tools/ab_libs.sh default padeskip0_e
done > gpurun_out/${T}_ab.log 2>&1 || exit 1
cat gpurun_out/${T}_ab.log
