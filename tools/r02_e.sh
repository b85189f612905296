#!/bin/bash
# config E on the GPU box: dense-model parity tests, kernel time at batch 16,384, phase cycles
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/${1:-r02e}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k dense \
    > $O.tests.log 2>&1; rc=$?; echo "dense tests rc=$rc"; tail -n 25 $O.tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python tools/time_kernel.py --configs E --batch 16384 --reps 5 > $O.time.log 2>&1 || exit 1
cat $O.time.log
timeout -k 10 200 python tools/phase_profile.py --config E --batch 4096 > $O.phase.log 2>&1 || exit 1
cat $O.phase.log
