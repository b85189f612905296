#!/bin/bash
# round-2 GPU check: -m gpu suite, overflow-launch overhead at config B, workgroup-kernel timing
# and phase cycles (stamps build).  Each GPU step has its own time limit; stops at a failure.
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/${1:-r02}
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu \
    > $O.tests.log 2>&1; echo "tests rc=$?"; tail -n 3 $O.tests.log
timeout -k 10 120 python tools/time_kernel.py --configs B > $O.time.log 2>&1 || exit 1
timeout -k 10 120 python tools/time_kernel.py --configs B --max-free 30 >> $O.time.log 2>&1 || exit 1
timeout -k 10 200 python tools/time_kernel.py --configs B --gait standing --reps 5 >> $O.time.log 2>&1 || exit 1
timeout -k 10 200 python tools/time_kernel.py --configs C --gait mixed --reps 3 --batch 16384 >> $O.time.log 2>&1 || exit 1
cat $O.time.log
timeout -k 10 200 python tools/phase_profile.py --config B --gait standing --batch 16384 > $O.phase.log 2>&1 || exit 1
timeout -k 10 200 python tools/phase_profile.py --config C --gait standing --batch 8192 >> $O.phase.log 2>&1 || exit 1
cat $O.phase.log
