#!/bin/bash
# round-2 re-entry check on the GPU box: full -m gpu suite, config E timing, default bench line.
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r02a
timeout -k 10 500 python -u -m pytest -v --maxfail=5 --timeout 200 --timeout-method thread tests -m gpu \
    > $O.tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $O.tests.log | tail -n 15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 200 python tools/time_kernel.py --configs E --batch 16384 --reps 5 > $O.timeE.log 2>&1 || { cat $O.timeE.log; exit 1; }
cat $O.timeE.log
timeout -k 10 400 python bench.py > $O.bench.log 2>&1 || { tail -n 20 $O.bench.log; exit 1; }
grep '^{' $O.bench.log > $O.bench.json
echo done
