#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/${1:-r02p2}
: > $O.phase.log
timeout -k 10 120 python tools/phase_profile.py --config E --batch 4096 >> $O.phase.log 2>&1 || { cat $O.phase.log; exit 1; }
timeout -k 10 120 python tools/phase_profile.py --config B --gait standing --batch 16384 >> $O.phase.log 2>&1 || { cat $O.phase.log; exit 1; }
timeout -k 10 120 python tools/phase_profile.py --config C --gait mixed --batch 4096 >> $O.phase.log 2>&1 || { cat $O.phase.log; exit 1; }
grep -v amdgpu.ids $O.phase.log | grep -v RuntimeWarning | grep -v "share = "
