#!/bin/bash
# -m gpu suite on the GPU box (verbose, one process, per-test time limit); extra args go to pytest
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/${TAG:-t}
timeout -k 10 600 python -u -m pytest -v --maxfail=5 --timeout 200 --timeout-method thread tests -m gpu "$@" \
    > $O.tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $O.tests.log | tail -n 15
exit $rc
