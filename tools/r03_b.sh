#!/bin/bash
# overflow sub-lists + early exit: the suite, B standing / C mixed timing, lone-wave dual-pass stamps
set -o pipefail
mkdir -p gpurun_out
TAG=r03b tools/gpu_tests.sh || exit 1
timeout -k 10 200 python -u tools/time_kernel.py --configs B,C --gait standing --reps 10 > gpurun_out/r03b_standing.log 2>&1 || { echo standing failed; tail -5 gpurun_out/r03b_standing.log; exit 1; }
cat gpurun_out/r03b_standing.log
timeout -k 10 200 python -u tools/time_kernel.py --configs C --gait mixed --reps 5 > gpurun_out/r03b_mixed.log 2>&1 || { echo mixed failed; exit 1; }
cat gpurun_out/r03b_mixed.log
MPCQP_LIB=$PWD/mpc-limx-control_amd/lib/libmpcqp_stamps.so timeout -k 10 200 python -u tools/r03_sweep.py --max-free 30 --reps 5 --sizes 128,256,512 > gpurun_out/r03b_stamps.log 2>&1 || { echo stamps failed; exit 1; }
cat gpurun_out/r03b_stamps.log
timeout -k 10 200 python -u tools/r03_sweep.py --reps 30 --sizes 4096,8192,65536 > gpurun_out/r03b_sweep.log 2>&1 || { echo sweep failed; exit 1; }
cat gpurun_out/r03b_sweep.log
