#!/bin/bash
# r05: config E -- the one-wave Pade solve against the last wave's side work (probe stamps:
# slot 15 = wave 0's Gauss-Jordan, slot 0 = the free map), and an A/B of the LDS column broadcast
set -o pipefail
T=${1:-r05n}
mkdir -p gpurun_out
{ MPCQP_LIB=$PWD/mpc-limx-control_amd/lib/libmpcqp_probe.so timeout -k 10 120 python tools/phase_profile.py --config E --batch 16384 &&
  for r in 1 2 3; do AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384 bash tools/ab_libs.sh default padelds_e; done; } \
  > gpurun_out/${T}.txt 2>&1 || { tail -30 gpurun_out/${T}.txt; exit 1; }
cat gpurun_out/${T}.txt
