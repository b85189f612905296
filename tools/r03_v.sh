#!/bin/bash
# pair-kernel spills (8 -> 2 VGPRs), one-QP kernel defers before the model: tests + timings
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03v}
TAG=$T tools/gpu_tests.sh || exit 1
timeout -k 10 300 python tools/r03_sweep.py --sizes 512,4096,8192,65536 --reps 40 > gpurun_out/${T}_sweep.log 2>&1 || { cat gpurun_out/${T}_sweep.log; exit 1; }
cat gpurun_out/${T}_sweep.log
timeout -k 10 200 python tools/defer_cuts.py > gpurun_out/${T}_defer.log 2>&1 || { cat gpurun_out/${T}_defer.log; exit 1; }
cat gpurun_out/${T}_defer.log
AB_CONFIGS=B,C,L AB_REPS=20 timeout -k 10 200 tools/ab_libs.sh default > gpurun_out/${T}_BCL.log 2>&1 || { cat gpurun_out/${T}_BCL.log; exit 1; }
cat gpurun_out/${T}_BCL.log
AB_CONFIGS=C AB_GAIT=mixed AB_REPS=6 timeout -k 10 200 tools/ab_libs.sh default > gpurun_out/${T}_Cmix.log 2>&1 || { cat gpurun_out/${T}_Cmix.log; exit 1; }
cat gpurun_out/${T}_Cmix.log
