#!/bin/bash
# fused-selection tickets only for workgroups with instances: GPU tests + sweep
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03p}
TAG=$T tools/gpu_tests.sh || exit 1
timeout -k 10 300 python tools/r03_sweep.py --sizes 512,4096,8192,65536 --reps 40 > gpurun_out/${T}_sweep.log 2>&1 || { cat gpurun_out/${T}_sweep.log; exit 1; }
cat gpurun_out/${T}_sweep.log
