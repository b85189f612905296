#!/bin/bash
# r05: where config C's and E's time goes at the DPP-diagonal library: per-phase stamps
# (lib/libmpcqp_stamps.so) and early-exit cuts (lib/libmpcqp_cuts.so)
set -o pipefail
T=${1:-r05m}
mkdir -p gpurun_out
{ timeout -k 10 120 python tools/phase_profile.py --config C &&
  timeout -k 10 120 python tools/phase_profile.py --config E --batch 16384 &&
  timeout -k 10 300 python tools/phase_cuts.py --configs C --reps 10 --cuts 11,13,1,2,3,4,6,7,0; } \
  > gpurun_out/${T}_phases.txt 2>&1 || { tail -30 gpurun_out/${T}_phases.txt; exit 1; }
cat gpurun_out/${T}_phases.txt
