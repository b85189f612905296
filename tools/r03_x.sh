#!/bin/bash
# unmasked diagonal-block Cholesky in the one-QP NF = 60 kernels (chol_reg.hpp): A/B on C
# (cdns0 = MPCQP_DIAG_NOSEL=0 in fast_srbm20) and L (ldns0, fast_literal) at 65,536
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03x}
AB_CONFIGS=C AB_REPS=10 timeout -k 10 300 tools/ab_libs.sh default cdns0 default cdns0 > gpurun_out/${T}_C.log 2>&1 || { cat gpurun_out/${T}_C.log; exit 1; }
cat gpurun_out/${T}_C.log
AB_CONFIGS=L AB_REPS=10 timeout -k 10 300 tools/ab_libs.sh default ldns0 default ldns0 > gpurun_out/${T}_L.log 2>&1 || { cat gpurun_out/${T}_L.log; exit 1; }
cat gpurun_out/${T}_L.log
