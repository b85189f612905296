#!/bin/bash
# one-wave register Gauss-Jordan for E's Pade quotient: dense tests, A/B, stamps
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03w}
TAG=$T tools/gpu_tests.sh -k "dense or E or expm or discret" || exit 1
AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384 timeout -k 10 300 tools/ab_libs.sh default pw0 default pw0 > gpurun_out/${T}_E16k.log 2>&1 || { cat gpurun_out/${T}_E16k.log; exit 1; }
cat gpurun_out/${T}_E16k.log
MPCQP_LIB=$PWD/mpc-limx-control_amd/lib/libmpcqp_stamps_dsub.so timeout -k 10 200 python tools/phase_profile.py --config E --batch 16384 > gpurun_out/${T}_E_stamps.log 2>&1 || { tail gpurun_out/${T}_E_stamps.log; exit 1; }
cat gpurun_out/${T}_E_stamps.log
