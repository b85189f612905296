#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/${1:-r02e2}
timeout -k 10 600 python -u -m pytest -v --maxfail=5 --timeout 200 --timeout-method thread tests -m gpu \
    > $O.tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $O.tests.log | tail -n 12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 200 python tools/time_kernel.py --configs E --batch 16384 --reps 5 > $O.time.log 2>&1 || { cat $O.time.log; exit 1; }
cat $O.time.log
timeout -k 10 120 python tools/phase_profile.py --config E --batch 4096 > $O.phase.log 2>&1 || { cat $O.phase.log; exit 1; }
grep -v amdgpu.ids $O.phase.log | grep -v RuntimeWarning | grep -v "share = "
