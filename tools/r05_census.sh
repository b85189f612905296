#!/bin/bash
# r05: per-phase census (PMC per early-exit cut) and per-phase time (cuts) of k_mpc_pair, config B
set -o pipefail
T=${1:-r05e}
mkdir -p gpurun_out
bash tools/phase_pmc_pair.sh gpurun_out/pp_$T B > gpurun_out/${T}_census.txt 2>&1 || { tail gpurun_out/${T}_census.txt; exit 1; }
timeout -k 10 300 python tools/phase_cuts.py --configs B --reps 20 --cuts 11,1,13,2,3,4,6,8,7,0 > gpurun_out/${T}_cuts.txt 2>&1 || exit 1
cat gpurun_out/${T}_census.txt gpurun_out/${T}_cuts.txt
