#!/bin/bash
# Toeplitz condensing for the dense model: GPU tests, E A/B at 16384 and 65536, E stamps
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03q}
TAG=$T tools/gpu_tests.sh || exit 1
AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384 timeout -k 10 300 tools/ab_libs.sh default dnt0 default dnt0 > gpurun_out/${T}_E16k.log 2>&1 || { cat gpurun_out/${T}_E16k.log; exit 1; }
cat gpurun_out/${T}_E16k.log
AB_CONFIGS=E AB_REPS=10 timeout -k 10 300 tools/ab_libs.sh default dnt0 > gpurun_out/${T}_E64k.log 2>&1 || { cat gpurun_out/${T}_E64k.log; exit 1; }
cat gpurun_out/${T}_E64k.log
timeout -k 10 200 python tools/phase_profile.py --config E --batch 16384 > gpurun_out/${T}_E_stamps.log 2>&1 || { tail gpurun_out/${T}_E_stamps.log; exit 1; }
cat gpurun_out/${T}_E_stamps.log
