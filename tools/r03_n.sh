#!/bin/bash
# small-batch sweep at HEAD (kernel / solve / step) and lone-wave stamps
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03n}
TAG=$T tools/gpu_tests.sh || exit 1
timeout -k 10 300 python tools/r03_sweep.py --sizes 512,2048,4096,6144,8192,16384,65536 --reps 40 > gpurun_out/${T}_sweep.log 2>&1 || { cat gpurun_out/${T}_sweep.log; exit 1; }
cat gpurun_out/${T}_sweep.log
MPCQP_LIB=$PWD/mpc-limx-control_amd/lib/libmpcqp_stamps.so timeout -k 10 300 python tools/r03_sweep.py --sizes 512,4096,8192 --reps 5 > gpurun_out/${T}_stamps.log 2>&1 || { cat gpurun_out/${T}_stamps.log; exit 1; }
cat gpurun_out/${T}_stamps.log
