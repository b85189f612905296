#!/bin/bash
# Round-5 stall profiles at the current library: headline B, config C, config E (GPU box).
set -o pipefail
T=${1:-r05a}
bash tools/pmc_stall.sh gpurun_out/st_$T/B && \
bash tools/pmc_stall.sh gpurun_out/st_$T/C --driver "tools/time_kernel.py --configs C --batch 65536 --reps 5" && \
bash tools/pmc_stall.sh gpurun_out/st_$T/E --driver "tools/time_kernel.py --configs E --batch 16384 --reps 5"
