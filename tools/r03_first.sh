#!/bin/bash
# round 3, first GPU call: the suite, the batch-size sweep (release / no overflow launch / stamps),
# a kernel trace of the sweep, the default bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r03a tools/gpu_tests.sh || exit 1
timeout -k 10 240 python -u tools/r03_sweep.py > gpurun_out/r03_sweep_rel.log 2>&1 || { echo sweep failed; tail -5 gpurun_out/r03_sweep_rel.log; exit 1; }
cat gpurun_out/r03_sweep_rel.log
timeout -k 10 240 python -u tools/r03_sweep.py --max-free 30 --sizes 512,2048,4096,8192,16384,65536 > gpurun_out/r03_sweep_mf30.log 2>&1 || { echo sweep2 failed; exit 1; }
cat gpurun_out/r03_sweep_mf30.log
MPCQP_LIB=$PWD/mpc-limx-control_amd/lib/libmpcqp_stamps.so timeout -k 10 240 python -u tools/r03_sweep.py --max-free 30 --reps 5 --sizes 256,512,2048,4096,8192,65536 > gpurun_out/r03_sweep_stamps.log 2>&1 || { echo sweep3 failed; exit 1; }
cat gpurun_out/r03_sweep_stamps.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/r03_sweep_trace -o run --output-format csv -- python3 tools/r03_sweep.py --reps 20 --sizes 512,4096,8192,65536 > gpurun_out/r03_sweep_trace.log 2>&1 || { echo trace failed; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/r03_bench0.log 2>&1 || { echo bench failed; tail -5 gpurun_out/r03_bench0.log; exit 1; }
tail -c 600 gpurun_out/r03_bench0.log
