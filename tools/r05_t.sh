#!/bin/bash
# r05: the Pade Gauss-Jordan's pivot swap: micro-benchmark (tools/micro, unrolled builds: the
# library's loop with the if-chain swap / with the switch, and the local template variants),
# E A/B (default if-chain vs libmpcqp_padesw_e.so), then the dense parity tests
set -o pipefail
T=${1:-r05t}
mkdir -p gpurun_out
{ (cd tools/micro && timeout -k 10 60 ./pade_bench 256 4 && timeout -k 10 60 ./pade_bench_sw 256 4 &&
   timeout -k 10 60 ./pade_bench 16384 2 && timeout -k 10 60 ./pade_bench_sw 16384 2) &&
  for r in 1 2 3; do AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384 bash tools/ab_libs.sh default padesw_e; done &&
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k "dense or E" 2>&1 | tail -3; } \
  > gpurun_out/${T}.txt 2>&1 || { tail -30 gpurun_out/${T}.txt; exit 1; }
cat gpurun_out/${T}.txt
