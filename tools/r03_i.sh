#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03i}
AB_CONFIGS=E AB_REPS=10 timeout -k 10 300 tools/ab_libs.sh default dw1 default dw1 > gpurun_out/${T}_dense_ab.log 2>&1 || { echo ab failed; cat gpurun_out/${T}_dense_ab.log; exit 1; }
cat gpurun_out/${T}_dense_ab.log
timeout -k 10 200 python tools/phase_profile.py --config E --batch 16384 > gpurun_out/${T}_E_stamps.log 2>&1 || { echo stamps failed; tail gpurun_out/${T}_E_stamps.log; exit 1; }
cat gpurun_out/${T}_E_stamps.log
timeout -k 10 900 tools/phase_pmc_pair.sh gpurun_out/${T}_ppair B > gpurun_out/${T}_ppair.log 2>&1 || { echo ppair failed; tail gpurun_out/${T}_ppair.log; exit 1; }
cat gpurun_out/${T}_ppair.log
