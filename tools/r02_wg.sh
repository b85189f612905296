#!/bin/bash
# -m gpu suite, then kernel time of the workgroup-kernel configs (E, B standing, C mixed)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/${1:-r02w}
timeout -k 10 600 python -u -m pytest -v --maxfail=5 --timeout 200 --timeout-method thread tests -m gpu \
    > $O.tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $O.tests.log | tail -n 12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 200 python tools/time_kernel.py --configs E --batch 16384 --reps 5 > $O.time.log 2>&1 || { cat $O.time.log; exit 1; }
timeout -k 10 200 python tools/time_kernel.py --configs B --gait standing --reps 5 >> $O.time.log 2>&1 || { cat $O.time.log; exit 1; }
timeout -k 10 200 python tools/time_kernel.py --configs C --gait mixed --reps 3 >> $O.time.log 2>&1 || { cat $O.time.log; exit 1; }
cat $O.time.log
