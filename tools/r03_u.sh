#!/bin/bash
# E per-phase stamps (expm split into products / Pade solve / squarings by the sub-stamps)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03u}
MPCQP_LIB=$PWD/mpc-limx-control_amd/lib/libmpcqp_stampsE.so timeout -k 10 200 python tools/phase_profile.py --config E --batch 16384 > gpurun_out/${T}_E_stamps.log 2>&1 || { tail gpurun_out/${T}_E_stamps.log; exit 1; }
cat gpurun_out/${T}_E_stamps.log
