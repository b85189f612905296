#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03h}
TAG=$T tools/gpu_tests.sh || exit 1
timeout -k 10 200 python -u tools/r03_sweep.py --reps 30 --sizes 512,4096,8192,65536 > gpurun_out/${T}_sweep.log 2>&1 || { echo sweep failed; exit 1; }
cat gpurun_out/${T}_sweep.log
AB_CONFIGS=E AB_REPS=10 timeout -k 10 300 tools/ab_libs.sh default dw1 default dw1 > gpurun_out/${T}_dense_ab.log 2>&1 || { echo ab failed; cat gpurun_out/${T}_dense_ab.log; exit 1; }
cat gpurun_out/${T}_dense_ab.log
timeout -k 10 900 tools/phase_pmc_pair.sh gpurun_out/${T}_ppair B > gpurun_out/${T}_ppair.log 2>&1 || { echo ppair failed; tail gpurun_out/${T}_ppair.log; exit 1; }
cat gpurun_out/${T}_ppair.log
