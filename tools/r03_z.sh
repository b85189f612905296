#!/bin/bash
# lone-wavefront latency of the paired kernel at small shards: per-phase cycles per wave and the
# dual loop's per-pass split (stamps build), 512 .. 8,192 instances
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03z}
MPCQP_LIB=$PWD/mpc-limx-control_amd/lib/libmpcqp_stamps.so timeout -k 10 300 python -u tools/r03_sweep.py --sizes 512,2048,4096,8192,65536 --reps 5 > gpurun_out/${T}_stamps.log 2>&1 || { tail gpurun_out/${T}_stamps.log; exit 1; }
cat gpurun_out/${T}_stamps.log
