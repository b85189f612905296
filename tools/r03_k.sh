#!/bin/bash
# per-phase stamps of the workgroup kernels after R^-1 (C mixed, B standing)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03k}
timeout -k 10 200 python tools/phase_profile.py --config C --gait mixed --batch 16384 > gpurun_out/${T}_Cmix_stamps.log 2>&1 || { tail gpurun_out/${T}_Cmix_stamps.log; exit 1; }
cat gpurun_out/${T}_Cmix_stamps.log
timeout -k 10 200 python tools/phase_profile.py --config C --gait standing --batch 16384 > gpurun_out/${T}_Cst_stamps.log 2>&1 || { tail gpurun_out/${T}_Cst_stamps.log; exit 1; }
cat gpurun_out/${T}_Cst_stamps.log
timeout -k 10 200 python tools/phase_profile.py --config B --gait standing --batch 16384 > gpurun_out/${T}_Bst_stamps.log 2>&1 || { tail gpurun_out/${T}_Bst_stamps.log; exit 1; }
cat gpurun_out/${T}_Bst_stamps.log
