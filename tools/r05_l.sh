#!/bin/bash
# r05: GPU suite, then A/B of the DPP diagonal-block factorisation (chol_mfma.hpp
# MPCQP_DIAG_DPP) against the v_readlane form: C (one-wave MFMA start), E (dense workgroup),
# B standing (NF = 64 overflow workgroup kernel); alternating processes, three rounds
set -o pipefail
T=${1:-r05l}
mkdir -p gpurun_out
TAG=$T bash tools/gpu_tests.sh || exit 1
for r in 1 2 3; do
  AB_CONFIGS=C AB_REPS=20 bash tools/ab_libs.sh default diagrl_c
  AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384 bash tools/ab_libs.sh default diagrl_e
  AB_CONFIGS=B AB_GAIT=standing AB_REPS=10 bash tools/ab_libs.sh default diagrl_w
done > gpurun_out/${T}_ab.log 2>&1 || exit 1
cat gpurun_out/${T}_ab.log
