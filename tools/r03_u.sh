#!/bin/bash
# overflow routing by per-instance flags (no returned atomic): GPU tests, deferral cuts,
# B standing / C mixed / B alternating timings, small-batch sweep
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03u}
TAG=$T tools/gpu_tests.sh || exit 1
timeout -k 10 200 python tools/defer_cuts.py > gpurun_out/${T}_defer.log 2>&1 || { cat gpurun_out/${T}_defer.log; exit 1; }
cat gpurun_out/${T}_defer.log
AB_CONFIGS=B AB_GAIT=standing AB_REPS=10 timeout -k 10 200 tools/ab_libs.sh default > gpurun_out/${T}_Bst.log 2>&1 || { cat gpurun_out/${T}_Bst.log; exit 1; }
cat gpurun_out/${T}_Bst.log
AB_CONFIGS=C AB_GAIT=mixed AB_REPS=6 timeout -k 10 200 tools/ab_libs.sh default > gpurun_out/${T}_Cmix.log 2>&1 || { cat gpurun_out/${T}_Cmix.log; exit 1; }
cat gpurun_out/${T}_Cmix.log
timeout -k 10 300 python tools/r03_sweep.py --sizes 512,4096,8192,65536 --reps 40 > gpurun_out/${T}_sweep.log 2>&1 || { cat gpurun_out/${T}_sweep.log; exit 1; }
cat gpurun_out/${T}_sweep.log
