#!/bin/bash
# r05: (1) GPU suite; (2) the Pade Gauss-Jordan micro-benchmark (tools/micro/pade_bench);
# (3) config B standing / double support / alternating: the paired kernel's overflow on the
# one-QP-per-wave k_mpc_list (default) against the workgroup kernel (libmpcqp_ovfwg.so)
set -o pipefail
T=${1:-r05s}
mkdir -p gpurun_out
TAG=$T bash tools/gpu_tests.sh || exit 1
{ (cd tools/micro && timeout -k 10 60 ./pade_bench 256 4 && timeout -k 10 60 ./pade_bench 16384 2) &&
  for g in standing double alternating; do
    for r in 1 2; do
      AB_CONFIGS=B AB_GAIT=$g AB_REPS=10 bash tools/ab_libs.sh default ovfwg
    done
  done; } > gpurun_out/${T}.txt 2>&1 || { tail -30 gpurun_out/${T}.txt; exit 1; }
cat gpurun_out/${T}.txt
